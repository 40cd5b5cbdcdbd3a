#!/bin/bash
# Development GPU round: parity probe, overlapped trace + timeline, bench.
# usage: bash tools/gpu_round.sh TAG [extra-env]
TAG=${1:-dev}
export TMPDIR=/tmp
timeout -k 10 200 python tools/quick_gpu_check.py > gpurun_out/quick_$TAG.log 2>&1 || { cat gpurun_out/quick_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu --no-extra --no-profile > gpurun_out/prof_$TAG.log 2>&1 || { tail gpurun_out/prof_$TAG.log; exit 2; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --skip-cpu --no-extra > gpurun_out/bench_$TAG.json 2>&1 || { tail gpurun_out/bench_$TAG.json; exit 3; }
tail -3 gpurun_out/quick_$TAG.log; grep -h metric gpurun_out/bench_$TAG.json | cut -c 150-260
python tools/kstats.py gpurun_out/prof_$TAG
python tools/timeline.py gpurun_out/prof_$TAG 10 20
