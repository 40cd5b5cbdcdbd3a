export TMPDIR=/tmp; mkdir -p gpurun_out/r06g
timeout -k 5 120 rocprofv3 --kernel-trace -d gpurun_out/r06g/probe -o run --output-format csv -- tools/bin/bulk_probe 129 113 1024 20 1 > gpurun_out/r06g/probe.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r06g/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --skip-cpu --no-extra --no-profile > gpurun_out/r06g/trace.log 2>&1 || exit 2
python tools/launch_list.py gpurun_out/r06g/trace > gpurun_out/r06g/launches.txt
grep -E "mode|sustained" gpurun_out/r06g/probe.txt
python - <<PY
import csv
tr=list(csv.DictReader(open("gpurun_out/r06g/probe/run_kernel_trace.csv")))
d=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in tr if "tile_syrk" in r["Kernel_Name"]]
print("probe launches (us):", [round(x) for x in d])
tr=list(csv.DictReader(open("gpurun_out/r06g/trace/run_kernel_trace.csv")))
tr.sort(key=lambda r:int(r["Start_Timestamp"]))
d=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in tr if "tile_syrk" in r["Kernel_Name"]]
print("eval first launches (us):", [round(x) for x in d[0::8]])
PY
timeout -k 10 600 python tools/ab.py r06g --reps 2 --ns 16384,8192 cur gw8:lib=tools/bin/lib_gw8_60.so
