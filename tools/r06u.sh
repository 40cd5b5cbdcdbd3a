export TMPDIR=/tmp; mkdir -p gpurun_out/r06u
timeout -k 10 1000 python tools/ab.py r06u --reps 2 --ns "" --grad --posterior cur low:lib=tools/bin/lib_split_low.so r05:lib=tools/bin/lib_r05.so
