#!/bin/bash
# tail trace + quick check at configs[1], select variants (lanes, HW queues), GPU suite
R=${1:-r03p}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
bash tools/gpu_trace.sh $R > gpurun_out/$R/trace.txt 2>&1; rc=$?
cat gpurun_out/$R/trace.txt
[ $rc -eq 0 ] || exit 12
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel lanes2 GAPLAC_BATCH_LANES=2 || exit 13
sel lanes3_q8 GAPLAC_BATCH_LANES=3 GPU_MAX_HW_QUEUES=8 || exit 14
sel lanes4_q8 GAPLAC_BATCH_LANES=4 GPU_MAX_HW_QUEUES=8 || exit 15
sel lanes4_q8_noshare GAPLAC_BATCH_LANES=4 GPU_MAX_HW_QUEUES=8 GAPLAC_TAIL_SHARE=0 || exit 16
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/$R/pytest_gpu.log
exit $rc
