#!/bin/bash
# batched lists with paired (K = 256) near-tile updates vs without (tools/bin/lib_nopairs.so):
# bitwise batch tests, select alternating, one batched-launch trace
R=${1:-r03am}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q -k "config4 or batch" --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_batch.log 2>&1 || { tail -30 gpurun_out/$R/pytest_batch.log; exit 1; }
tail -2 gpurun_out/$R/pytest_batch.log
NP=$PWD/tools/bin/lib_nopairs.so
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel pairs || exit 11
sel nopairs GAPLAC_LIB_PATH=$NP || exit 12
sel pairs_b || exit 13
sel nopairs_b GAPLAC_LIB_PATH=$NP || exit 14
timeout -k 10 200 python -u tools/batch_trace.py gpurun_out/$R/btrace.txt > gpurun_out/$R/btrace.log 2>&1 || { tail gpurun_out/$R/btrace.log; exit 2; }
python tools/tail_trace.py gpurun_out/$R/btrace.txt | grep -vE "^ *[0-9]+ " > gpurun_out/$R/btrace_summary.txt
cat gpurun_out/$R/btrace_summary.txt
rm -f gpurun_out/$R/btrace.txt
