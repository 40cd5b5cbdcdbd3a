#!/bin/bash
# Round 7 (round-6 continuation): the Gram inside the tail (TAIL_G tasks) for whole-in-tail
# single evaluations. Parity first (the whole-in-tail sizes and the bitwise batch-vs-single
# checks), then an A/B against the previous library at N = 4096 / 8192 / 16384 and select.
R=${1:-r07g}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_first.log 2>&1 || { tail -30 gpurun_out/$R/pytest_first.log; exit 1; }
tail -2 gpurun_out/$R/pytest_first.log
bash tools/n4096_timeline.sh $R || exit 2
timeout -k 10 560 python tools/ab.py $R --reps 2 --ns 4096,8192,16384 --select cur prev:lib=tools/bin/lib_head.so || exit 3
cat gpurun_out/$R/ab.txt
