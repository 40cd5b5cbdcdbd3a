export TMPDIR=/tmp; mkdir -p gpurun_out/r06m
bash tools/gpu_trace.sh r06m 16384 > gpurun_out/r06m/tail_stats_16384.txt 2>&1
bash tools/gpu_trace.sh r06m 4096 > gpurun_out/r06m/tail_stats_4096.txt 2>&1
head -16 gpurun_out/r06m/tail_stats_16384.txt; head -40 gpurun_out/r06m/tail_stats_4096.txt
