export TMPDIR=/tmp; mkdir -p gpurun_out/r06q
timeout -k 10 900 python tools/ab.py r06q --reps 2 --ns 65536,16384 cur split4:lib=tools/bin/lib_split4.so
