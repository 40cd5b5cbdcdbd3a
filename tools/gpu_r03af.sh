#!/bin/bash
# batched lists without quadrant tasks (tools/bin/lib_noquads.so) vs the current build: bitwise batch tests, select
R=${1:-r03af}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
NQ=$PWD/tools/bin/lib_noquads.so
GAPLAC_LIB_PATH=$NQ timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q -k "config4 or batch" --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_batch.log 2>&1 || { tail -30 gpurun_out/$R/pytest_batch.log; exit 1; }
tail -2 gpurun_out/$R/pytest_batch.log
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel cur || exit 11
sel noquads GAPLAC_LIB_PATH=$NQ || exit 12
sel cur_b || exit 13
sel noquads_b GAPLAC_LIB_PATH=$NQ || exit 14
sel noquads_lag32 GAPLAC_LIB_PATH=$NQ GAPLAC_BATCH_LAG=32 || exit 15
sel noquads_lag16 GAPLAC_LIB_PATH=$NQ GAPLAC_BATCH_LAG=16 || exit 16
