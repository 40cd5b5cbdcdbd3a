#!/bin/bash
# N = 65536 (BASELINE configs[3]) on one GPU: the single-GPU path, the distributed schedule
# at 1 rank and as 2 / 8 in-process loopback ranks (schedule overhead; broadcasts are D2D
# copies). usage: bash tools/dist_bench.sh TAG   -> gpurun_out/TAG/dist65k_1gpu.jsonl
R=${1:-dev}
export TMPDIR=/tmp; mkdir -p gpurun_out/$R; O=gpurun_out/$R/dist65k_1gpu.jsonl; : > $O
for args in "--mode single" "--mode dist" "--mode dist --loopback 2" "--mode dist --loopback 8"; do
  timeout -k 10 200 python bench.py $args --steps 3 --warmup 1 > gpurun_out/$R/d.json 2> gpurun_out/$R/d.err || { tail gpurun_out/$R/d.err; exit 1; }
  tail -1 gpurun_out/$R/d.json >> $O
  python -c "import json,sys; d=json.loads(open('gpurun_out/$R/d.json').read().strip().splitlines()[-1]); print('$args', round(d['ms_per_step'],1), 'ms', d['extra'].get('last_logpdf'))"
done
