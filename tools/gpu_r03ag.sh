#!/bin/bash
# single evaluations with whole-tile next-column updates (tools/bin/lib_single_noquads.so) vs the
# current build; select with the new batch default
R=${1:-r03ag}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
for rep in 1 2; do
  for arm in cur single_noquads; do
    if [ $arm = cur ]; then L=$CUR; else L=$PWD/tools/bin/lib_$arm.so; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
  done
done
for i in 1 2; do
timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$i.json 2>> gpurun_out/$R/select.err || exit 11
python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$i.json').read().strip().splitlines()[-1]); print('select', round(d['value'], 1), round(d['ms_per_step'], 1))"
done
