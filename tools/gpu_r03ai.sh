#!/bin/bash
# whole-tile TRSM tasks before the latency-shaped last columns: GPU suite, then single
# evaluations and select against tools/bin/lib_ql24.so (the previous default lists)
R=${1:-r03ai}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
PREV=$PWD/tools/bin/lib_ql24.so
for rep in 1 2; do
  for arm in cur prev; do
    if [ $arm = cur ]; then L=$CUR; else L=$PREV; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_${arm}_$rep.json 2>> gpurun_out/$R/select.err || exit 11
    python -c "import json; d = json.loads(open('gpurun_out/$R/sel_${arm}_$rep.json').read().strip().splitlines()[-1]); print('$arm select', round(d['value'], 1), round(d['ms_per_step'], 1))"
  done
done
