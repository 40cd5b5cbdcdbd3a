export TMPDIR=/tmp; mkdir -p gpurun_out/r06t
timeout -k 10 900 python tools/ab.py r06t --reps 3 --ns 16384,8192,4096 cur cx150:lib=tools/bin/lib_cx150.so cx200:lib=tools/bin/lib_cx200.so cx70:lib=tools/bin/lib_cx70.so
