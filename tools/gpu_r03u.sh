#!/bin/bash
# tail-length sweep after the chain diag fix, a gradient-mode kernel trace, select variants
R=${1:-r03u}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u tools/tail_sweep.py > gpurun_out/$R/tail_sweep.txt 2>&1 || { cat gpurun_out/$R/tail_sweep.txt; exit 11; }
cat gpurun_out/$R/tail_sweep.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace_grad -o run --output-format csv -- python bench.py --mode grad --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/trace_grad.log 2>&1 || exit 12
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel t32 GAPLAC_TAIL_S=32 || exit 13
sel t24 GAPLAC_TAIL_S=24 || exit 14
sel l3q8 GAPLAC_BATCH_LANES=3 GPU_MAX_HW_QUEUES=8 || exit 15
sel l4q8 GAPLAC_BATCH_LANES=4 GPU_MAX_HW_QUEUES=8 || exit 16
sel l4q8t32 GAPLAC_BATCH_LANES=4 GPU_MAX_HW_QUEUES=8 GAPLAC_TAIL_S=32 || exit 17
