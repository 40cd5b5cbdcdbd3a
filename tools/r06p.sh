export TMPDIR=/tmp; mkdir -p gpurun_out/r06p
timeout -k 10 900 python tools/ab.py r06p --reps 3 --ns 16384,12000,4096 --select cur low:lib=tools/bin/lib_split_low.so nosplit:lib=tools/bin/lib_nosplit.so
