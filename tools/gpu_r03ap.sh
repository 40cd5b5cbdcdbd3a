#!/bin/bash
# near-tile column groups of 4 (K = 512; tools/bin/lib_g4.so, single and batched lists) vs 2 (current)
R=${1:-r03ap}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
G4=$PWD/tools/bin/lib_g4.so
GAPLAC_LIB_PATH=$G4 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_schedules.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_g4.log 2>&1 || { tail -30 gpurun_out/$R/pytest_g4.log; exit 1; }
tail -2 gpurun_out/$R/pytest_g4.log
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
for rep in 1 2; do
  for arm in g2 g4; do
    if [ $arm = g2 ]; then L=$CUR; else L=$G4; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_${arm}_$rep.json 2>> gpurun_out/$R/select.err || exit 11
    python -c "import json; d = json.loads(open('gpurun_out/$R/sel_${arm}_$rep.json').read().strip().splitlines()[-1]); print('$arm select', round(d['value'], 1), round(d['ms_per_step'], 1))"
  done
done
