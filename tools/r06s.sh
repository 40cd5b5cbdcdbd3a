export TMPDIR=/tmp; mkdir -p gpurun_out/r06s
timeout -k 10 900 python tools/ab.py r06s --reps 3 --ns 16384,8192,4096 cur simconst:lib=tools/bin/lib_simconst.so
