#!/bin/bash
# tail trace + quick check at configs[1], select with / without the tail CU share, GPU suite
R=${1:-r03o}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
bash tools/gpu_trace.sh $R > gpurun_out/$R/trace.txt 2>&1; rc=$?
cat gpurun_out/$R/trace.txt
[ $rc -eq 0 ] || exit 12
timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu > gpurun_out/$R/select.json 2> gpurun_out/$R/select.err || { tail -5 gpurun_out/$R/select.err; exit 13; }
GAPLAC_TAIL_SHARE=0 timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu > gpurun_out/$R/select_noshare.json 2>> gpurun_out/$R/select.err || exit 14
python -c "
import json
for f in ['select', 'select_noshare']:
    d = json.loads(open('gpurun_out/$R/' + f + '.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'])
"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/$R/pytest_gpu.log
exit $rc
