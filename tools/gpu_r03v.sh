#!/bin/bash
# Gram-in-bulk: GPU suite, A/B against the previous build (GAPLAC_LIB_PATH), trace, select
R=${1:-r03v}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
for i in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export GAPLAC_LIB_PATH=$PWD/gaplac_amd/_lib/libgaplac_hip_base.so; else unset GAPLAC_LIB_PATH; fi
    timeout -k 10 200 python -u tools/ab_sweep.py GAPLAC_SPW 4 > gpurun_out/$R/ab_${lib}_$i.txt 2>&1 || { cat gpurun_out/$R/ab_${lib}_$i.txt; exit 11; }
    echo "$lib: $(grep ms/eval gpurun_out/$R/ab_${lib}_$i.txt | tr '\n' ' ')"
  done
done
unset GAPLAC_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/trace.log 2>&1 || exit 12
python tools/timeline2.py gpurun_out/$R/trace
for lib in base new; do
  if [ $lib = base ]; then export GAPLAC_LIB_PATH=$PWD/gaplac_amd/_lib/libgaplac_hip_base.so; else unset GAPLAC_LIB_PATH; fi
  timeout -k 10 200 python bench.py --mode select --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$lib.json 2>> gpurun_out/$R/select.err || exit 13
  python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$lib.json').read().strip().splitlines()[-1]); print('select $lib', round(d['value'], 1), round(d['ms_per_step'], 1))"
done
