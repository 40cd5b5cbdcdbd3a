#!/bin/bash
# Kernel trace of a short bench run under one environment setting, plus the span summary.
# usage: bash tools/trace_env.sh TAG "ENV=..." ["ENV2=..."...]
TAG=$1; shift
export TMPDIR=/tmp
for e in "$@"; do
  d=gpurun_out/tr_${TAG}_$(echo "$e" | tr ' =' '__')
  env $e timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu --no-extra --no-profile > $d.log 2>&1 || { tail $d.log; exit 1; }
  echo "== $e: $(grep -h -o '"ms_per_step": [0-9.]*' $d.log)"
  python tools/span.py $d | head -1
done
