export TMPDIR=/tmp; R=r04i; mkdir -p gpurun_out/$R
timeout -k 10 600 python -u tools/ab.py $R --reps 3 --ns 4096,16384 cur r03:lib=tools/bin/lib_r03.so || exit 3
