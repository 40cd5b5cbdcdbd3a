#!/bin/bash
# GPU suite (batched lists with pairs), then single evaluations with pairs before the last 24
# columns (tools/bin/lib_spairs.so) vs without (current), alternating
R=${1:-r03an}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
CUR=$PWD/gaplac_amd/_lib/libgaplac_hip.so
for rep in 1 2; do
  for arm in cur spairs; do
    if [ $arm = cur ]; then L=$CUR; else L=$PWD/tools/bin/lib_$arm.so; fi
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_NONE - > gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    GAPLAC_LIB_PATH=$L timeout -k 10 200 python -u tools/ab_n.py GAPLAC_NONE - 8192 >> gpurun_out/$R/ab_${arm}_$rep.txt 2>&1 || { cat gpurun_out/$R/ab_${arm}_$rep.txt; exit 2; }
    sed "s/^/$arm /" gpurun_out/$R/ab_${arm}_$rep.txt | grep N=
  done
done
