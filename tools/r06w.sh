export TMPDIR=/tmp; mkdir -p gpurun_out/r06w
timeout -k 10 1000 python tools/ab.py r06w --reps 2 --ns "" --grad cur r05:lib=tools/bin/lib_r05.so
