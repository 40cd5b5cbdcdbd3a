export TMPDIR=/tmp; mkdir -p gpurun_out/r06v
timeout -k 10 1000 python tools/ab.py r06v --reps 2 --ns "" --grad r05:lib=tools/bin/lib_r05.so c1:lib=tools/bin/lib_c1.so c2:lib=tools/bin/lib_c2.so low:lib=tools/bin/lib_split_low.so
