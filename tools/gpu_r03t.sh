#!/bin/bash
# after the chain diag-kernel switch: GPU suite, modes (grad, posterior, select), bench
R=${1:-r03t}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
for m in grad posterior select; do
  timeout -k 10 300 python bench.py --mode $m --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/$m.json 2> gpurun_out/$R/$m.err || { tail gpurun_out/$R/$m.err; exit 2; }
  python -c "import json; d = json.loads(open('gpurun_out/$R/$m.json').read().strip().splitlines()[-1]); print('$m', round(d['value'], 2), round(d['ms_per_step'], 2))"
done
timeout -k 10 400 python bench.py --skip-cpu > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { tail gpurun_out/$R/bench.err; exit 3; }
cut -c1-300 gpurun_out/$R/bench.json
