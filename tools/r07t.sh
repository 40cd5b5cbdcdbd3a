#!/bin/bash
# Round 6 (continued): the term descriptor stored by the first launch instead of a copy. Every
# GPU test and smoke, the N = 4096 timeline, then the A/B against the library before the
# Gram inside the tail (tools/bin/lib_prev.so = 474f613) at N = 4096 / 8192 / 16384 and select.
R=${1:-r07t}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 2; }
tail -3 gpurun_out/$R/smoke.log
bash tools/n4096_timeline.sh $R || exit 3
timeout -k 10 560 python tools/ab.py $R --reps 2 --ns 4096,8192,16384 --select cur prev:lib=tools/bin/lib_prev.so || exit 4
cat gpurun_out/$R/ab.txt
