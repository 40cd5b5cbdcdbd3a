#!/bin/bash
# diag probe, the tail quick check, then the GPU suite
R=${1:-r03f}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 60 ./tools/bin/diag_probe > gpurun_out/$R/diag_probe.txt 2>&1; rc=$?
head -30 gpurun_out/$R/diag_probe.txt
[ $rc -eq 0 ] || exit 11
timeout -k 10 120 python -u tools/quick_tail.py > gpurun_out/$R/quick_tail.txt 2>&1; rc=$?
cat gpurun_out/$R/quick_tail.txt
[ $rc -eq 0 ] || exit 12
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/$R/pytest_gpu.log
exit $rc
