#!/bin/bash
# tail trace at configs[1], tail-length sweep, a 16k kernel trace (span), GPU suite
R=${1:-r03q}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
bash tools/gpu_trace.sh $R > gpurun_out/$R/trace.txt 2>&1; rc=$?
cat gpurun_out/$R/trace.txt
[ $rc -eq 0 ] || exit 12
timeout -k 10 240 python -u tools/tail_sweep.py > gpurun_out/$R/tail_sweep.txt 2>&1; rc=$?
cat gpurun_out/$R/tail_sweep.txt
[ $rc -eq 0 ] || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace16k -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu > gpurun_out/$R/trace16k.log 2>&1 || exit 14
python tools/span.py gpurun_out/$R/trace16k | head -12
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/$R/pytest_gpu.log
exit $rc
