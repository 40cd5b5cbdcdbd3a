export TMPDIR=/tmp; mkdir -p gpurun_out/r06o
python - <<PY
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
print("priority range rc", hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), "least", lo.value, "greatest", hi.value)
PY
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r06o/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --skip-cpu --no-extra --no-profile > gpurun_out/r06o/trace.log 2>&1 || exit 2
python tools/launch_list.py gpurun_out/r06o/trace > gpurun_out/r06o/launches.txt
grep -E "tile_|tail_|gram" gpurun_out/r06o/launches.txt | head -60; tail -4 gpurun_out/r06o/launches.txt
