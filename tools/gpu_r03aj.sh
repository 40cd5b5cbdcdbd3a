#!/bin/bash
# select: models per launch x lag with the current batched lists
R=${1:-r03aj}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel default || exit 11
for w in 32 16; do for lag in 16 20 28 32; do sel w${w}lag$lag GAPLAC_BATCH_W=$w GAPLAC_BATCH_LAG=$lag || exit 12; done; done
sel w16lag24 GAPLAC_BATCH_W=16 GAPLAC_BATCH_LAG=24 || exit 13
sel default_b || exit 14
