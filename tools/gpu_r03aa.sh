#!/bin/bash
# LDS-staged tail updates (tail_update_lds): GPU suite, A/B against tools/bin/libbase.so at
# N = 4096 / 8192 / 16384 (bitwise logpdf), tail task traces, select with the pipelined batch
R=${1:-r03aa}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
fi
BASE=$PWD/tools/bin/libbase.so
for arm in new base new base; do
  if [ $arm = base ]; then L=$BASE; else L=$PWD/gaplac_amd/_lib/libgaplac_hip.so; fi
  GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_$arm.txt 2>&1 || { cat gpurun_out/$R/ab_$arm.txt; exit 2; }
  GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_$arm.txt 2>&1 || { cat gpurun_out/$R/ab_$arm.txt; exit 2; }
  sed "s/^/$arm /" gpurun_out/$R/ab_$arm.txt | grep N=
done
for arm in new base; do
  if [ $arm = base ]; then L=$BASE; else L=$PWD/gaplac_amd/_lib/libgaplac_hip.so; fi
  for N in 16384 8192; do
    GAPLAC_LIB_PATH=$L GAPLAC_TAIL_TRACE=$PWD/gpurun_out/$R/ttrace_${arm}_$N.txt timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - $N > /dev/null 2>&1 || exit 3
    echo "== $arm N=$N"; python tools/tail_trace.py gpurun_out/$R/ttrace_${arm}_$N.txt | grep -vE "^ *[0-9]+ " 
  done
done
sel() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel w4lag0 GAPLAC_BATCH_W=4 GAPLAC_BATCH_LAG=0 || exit 11
sel w32lag24 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=24 || exit 12
sel w32lag32 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=32 || exit 13
sel w32lag48 GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=48 || exit 14
