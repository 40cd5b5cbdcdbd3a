#!/bin/bash
# TRSM / Q probe, the tail trace at configs[1], the tail quick check, then the GPU suite
R=${1:-r03l}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 60 ./tools/bin/trsm_probe > gpurun_out/$R/trsm_probe.txt 2>&1; rc=$?
cat gpurun_out/$R/trsm_probe.txt
[ $rc -eq 0 ] || exit 11
bash tools/gpu_trace.sh $R > gpurun_out/$R/trace.txt 2>&1; rc=$?
cat gpurun_out/$R/trace.txt
[ $rc -eq 0 ] || exit 12
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/$R/pytest_gpu.log
exit $rc
