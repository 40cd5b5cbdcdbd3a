#!/bin/bash
# the other entry points on the current build: gradient, posterior, rand (N = 16384)
R=${1:-r03al}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
for m in grad posterior rand; do
  timeout -k 10 300 python bench.py --mode $m --steps 4 --warmup 1 --skip-cpu > gpurun_out/$R/$m.json 2> gpurun_out/$R/$m.err || { tail gpurun_out/$R/$m.err; exit 1; }
  python -c "import json; d = json.loads(open('gpurun_out/$R/$m.json').read().strip().splitlines()[-1]); print('$m', round(d['value'], 2), d['unit'], round(d['ms_per_step'], 2), 'ms')"
done
