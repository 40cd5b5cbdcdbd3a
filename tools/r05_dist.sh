#!/bin/bash
# Round 5: distributed-path tests, then the one-GPU replay of configs[3].
# usage: bash tools/r05_dist.sh TAG [replay args...]
R=${1:-r05a}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dist_replay.py tests/test_gpu_nccl.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_dist.log 2>&1 || { tail -40 gpurun_out/$R/pytest_dist.log; exit 1; }
tail -3 gpurun_out/$R/pytest_dist.log
timeout -k 10 500 python -u tools/dist_replay.py --out gpurun_out/$R/replay.jsonl "$@" > gpurun_out/$R/replay.log 2>&1 || { tail -30 gpurun_out/$R/replay.log; exit 2; }
cut -c1-600 gpurun_out/$R/replay.log
