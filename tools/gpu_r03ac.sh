#!/bin/bash
# batched tail task-list shape (GAPLAC_BATCH_TASKS=gw,near) and lag: bitwise batch tests, select sweep
R=${1:-r03ac}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q -k "config4 or batch" --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_batch.log 2>&1 || { tail -30 gpurun_out/$R/pytest_batch.log; exit 1; }
tail -2 gpurun_out/$R/pytest_batch.log
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel default || exit 11
sel gw4n2 GAPLAC_BATCH_TASKS=4,2 || exit 12
sel gw8n3 GAPLAC_BATCH_TASKS=8,3 || exit 13
sel gw8n4 GAPLAC_BATCH_TASKS=8,4 || exit 14
sel gw8n2lag16 GAPLAC_BATCH_LAG=16 || exit 15
sel gw8n2lag32 GAPLAC_BATCH_LAG=32 || exit 16
sel gw8n2lag20 GAPLAC_BATCH_LAG=20 || exit 17
sel default_b || exit 18
