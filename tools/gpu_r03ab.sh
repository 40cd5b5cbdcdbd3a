#!/bin/bash
# pipelined batch as the default (GPU suite), then tail deep-task variants (GAPLAC_TAIL_GW /
# GAPLAC_TAIL_NEAR builds in tools/bin) against the current build: single evaluations at
# N = 16384 / 4096 / 8192 and select (64 x N = 8192, 32 models per launch, lag 24)
R=${1:-r03ab}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
fi
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
for rep in 1 2; do
  for arm in cur gw8n4 gw4n2 gw4n8 gw8n2; do
    if [ $arm = cur ]; then L=$CUR; else L=$PWD/tools/bin/lib_$arm.so; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
  done
done
sel() {  # name, lib, env...
  local name=$1; shift; local L=$1; shift
  env GAPLAC_LIB_PATH=$L GAPLAC_BATCH_W=32 GAPLAC_BATCH_LAG=24 "$@" timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$name.json 2>> gpurun_out/$R/select.err || return 1
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$name.json').read().strip().splitlines()[-1]); print('select $name', round(d['value'], 1), round(d['ms_per_step'], 1))"
}
sel cur $CUR || exit 11
for arm in gw8n4 gw4n2 gw4n8 gw8n2; do sel $arm $PWD/tools/bin/lib_$arm.so || exit 12; done
timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_default.json 2>> gpurun_out/$R/select.err || exit 13
python -c "import json; d = json.loads(open('gpurun_out/$R/sel_default.json').read().strip().splitlines()[-1]); print('select default', round(d['value'], 1), round(d['ms_per_step'], 1))"
