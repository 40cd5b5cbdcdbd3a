#!/bin/bash
# batched tail as a software pipeline (GAPLAC_BATCH_W models per launch, model m GAPLAC_BATCH_LAG*m
# tile columns behind model 0): bitwise batch-vs-single test under the pipelined setting, then the
# select sweep
R=${1:-r03z}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k config4 --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_cfg4.log 2>&1 || { tail -30 gpurun_out/$R/pytest_cfg4.log; exit 1; }
tail -2 gpurun_out/$R/pytest_cfg4.log
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel w4lag0 GAPLAC_BATCH_W=4 GAPLAC_BATCH_LAG=0 || exit 11
sel w32lag16 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=16 || exit 12
sel w32lag8 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=8 || exit 13
sel w32lag24 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=24 || exit 14
sel w32lag12 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=12 || exit 15
sel w16lag16 GAPLAC_BATCH_W=16 GAPLAC_BATCH_LAG=16 || exit 16
sel w8lag8 GAPLAC_BATCH_W=8 GAPLAC_BATCH_LAG=8 || exit 17
sel w4lag0b GAPLAC_BATCH_W=4 GAPLAC_BATCH_LAG=0 || exit 18
