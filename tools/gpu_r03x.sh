#!/bin/bash
# deep tail tasks + batched tail: GPU suite, tail-length sweeps, select variants
R=${1:-r03x}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 300 python -u tools/ab_sweep.py GAPLAC_TAIL_S 48,64,80,96 > gpurun_out/$R/tail_sweep.txt 2>&1 || { cat gpurun_out/$R/tail_sweep.txt; exit 11; }
cat gpurun_out/$R/tail_sweep.txt
timeout -k 10 300 python -u tools/ab_n.py GAPLAC_TAIL_WHOLE 0,80 8192,10000 > gpurun_out/$R/whole_sweep.txt 2>&1 || { cat gpurun_out/$R/whole_sweep.txt; exit 12; }
cat gpurun_out/$R/whole_sweep.txt
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel batch8 || exit 13
sel batch4 GAPLAC_BATCH_W=4 || exit 14
sel batch16 GAPLAC_BATCH_W=16 || exit 15
sel lanes GAPLAC_TAIL_WHOLE=0 || exit 16
