#!/bin/bash
# Final state check: full -m gpu suite, smoke, the default bench (CPU leg included).
# usage: bash tools/final_check.sh rNN
R=${1:-r02f}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 2; }
timeout -k 10 400 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { tail gpurun_out/$R/bench.err; exit 3; }
cut -c1-400 gpurun_out/$R/bench.json
