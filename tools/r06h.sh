export TMPDIR=/tmp; mkdir -p gpurun_out/r06h
for arm in cur skip2; do
  if [ $arm = skip2 ]; then export GAPLAC_LIB_PATH=tools/bin/lib_skip2.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r06h/trace_$arm -o run --output-format csv -- python tools/ab_n.py GAPLAC_NONE - 16384 > gpurun_out/r06h/trace_$arm.log 2>&1 || exit 2
done
unset GAPLAC_LIB_PATH
timeout -k 5 120 rocprofv3 --kernel-trace -d gpurun_out/r06h/probe -o run --output-format csv -- tools/bin/bulk_probe 129 113 1024 20 1 > gpurun_out/r06h/probe.txt 2>&1 || exit 1
python - <<PY
import csv, statistics
def launches(d, name):
    tr=list(csv.DictReader(open(f"gpurun_out/r06h/{d}/run_kernel_trace.csv")))
    tr.sort(key=lambda r:int(r["Start_Timestamp"]))
    return [(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in tr if name in r["Kernel_Name"]]
p = launches("probe", "tile_syrk")[10:]
print("probe m=113 K=1024: median %.0f us" % statistics.median(p))
for arm in ("cur", "skip2"):
    d = launches("trace_" + arm, "tile_syrk")
    print(arm, "syrk launch medians by index:", [round(statistics.median(d[i::8][2:])) for i in range(8)])
    b = launches("trace_" + arm, "tile_band")
    nb = 17 if arm else 17
    print(arm, "band launch medians by index:", [round(statistics.median(b[i::12][2:])) for i in range(12)])
    t = launches("trace_" + arm, "tail_kernel")
    print(arm, "tail median %.0f" % statistics.median(t[2:]))
PY
