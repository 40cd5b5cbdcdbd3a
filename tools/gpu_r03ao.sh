#!/bin/bash
# with paired updates: latency-shaped end length (GAPLAC_QUAD_LAST 16 / 24 / 32 builds) and tail length
R=${1:-r03ao}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
for rep in 1 2; do
  for arm in ql24 ql16 ql32; do
    if [ $arm = ql24 ]; then L=$CUR; else L=$PWD/tools/bin/lib_$arm.so; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
  done
done
timeout -k 10 300 python -u tools/ab_n.py GAPLAC_TAIL_S 80,88,96,72,80 16384 > gpurun_out/$R/tail.txt 2>&1 || { cat gpurun_out/$R/tail.txt; exit 3; }
grep N= gpurun_out/$R/tail.txt
