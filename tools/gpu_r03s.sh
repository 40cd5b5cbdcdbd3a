#!/bin/bash
# A/B: diagonal kernel in the super-panel chain (GAPLAC_DIAG1), select lane variants, a trace
R=${1:-r03s}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
for v in 0 1; do
  GAPLAC_DIAG1=$v timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_SPW 4 > gpurun_out/$R/ab_diag1_$v.txt 2>&1 || { cat gpurun_out/$R/ab_diag1_$v.txt; exit 11; }
  cat gpurun_out/$R/ab_diag1_$v.txt
done
GAPLAC_DIAG1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace_d1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/trace_d1.log 2>&1 || exit 12
python tools/timeline2.py gpurun_out/$R/trace_d1
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel lanes2 GAPLAC_BATCH_LANES=2 || exit 13
sel lanes2_d1 GAPLAC_BATCH_LANES=2 GAPLAC_DIAG1=1 || exit 14
sel lanes4_serial GAPLAC_BATCH_LANES=4 GAPLAC_SERIAL=1 || exit 15
sel lanes4_q8_d1 GAPLAC_BATCH_LANES=4 GPU_MAX_HW_QUEUES=8 GAPLAC_DIAG1=1 || exit 16
