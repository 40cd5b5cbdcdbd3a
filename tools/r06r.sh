export TMPDIR=/tmp; mkdir -p gpurun_out/r06r
bash tools/gpu_trace.sh r06r 4096 > gpurun_out/r06r/tail_stats_4096.txt 2>&1 || exit 1
GAPLAC_TAIL_SIM=1 bash tools/gpu_trace.sh r06r 8192 > gpurun_out/r06r/tail_stats_8192.txt 2>&1 || exit 2
head -20 gpurun_out/r06r/tail_stats_4096.txt
