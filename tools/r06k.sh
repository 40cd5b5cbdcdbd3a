export TMPDIR=/tmp; mkdir -p gpurun_out/r06k
timeout -k 10 500 python tools/ab.py r06k --reps 2 --ns 16384 cur t104:GAPLAC_TAIL_S=104 t128:GAPLAC_TAIL_S=128 || exit 1
GAPLAC_TAIL_S=128 bash tools/gpu_trace.sh r06k 16384 > gpurun_out/r06k/tail_stats_t128.txt 2>&1
head -14 gpurun_out/r06k/tail_stats_t128.txt
