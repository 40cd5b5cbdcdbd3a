export TMPDIR=/tmp; R=r04k; mkdir -p gpurun_out/$R
timeout -k 10 800 python -u tools/ab.py $R --reps 2 --ns 4096 cur nofault:lib=tools/bin/lib_nofault.so rowf03:lib=tools/bin/lib_rowf03.so r03:lib=tools/bin/lib_r03.so || exit 3
