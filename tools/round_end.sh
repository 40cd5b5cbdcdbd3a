#!/bin/bash
# Round-end GPU pass: full -m gpu suite, smoke, then the round profile (tools/profile_round.sh).
# usage: bash tools/round_end.sh rNN
R=${1:-r02c}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || { tail -20 gpurun_out/$R/smoke.log; exit 2; }
cat gpurun_out/$R/smoke.log
bash tools/profile_round.sh $R
