#!/bin/bash
# env_sweep.sh for another bench mode: bash tools/env_sweep_mode.sh TAG MODE "ENV1" "ENV2" ...
TAG=$1; MODE=$2; shift 2
export TMPDIR=/tmp
out=gpurun_out/sweep_$TAG.txt
: > $out
for e in "$@"; do
  env $e timeout -k 10 200 python bench.py --mode $MODE --steps 6 --warmup 2 --skip-cpu --no-profile > gpurun_out/sweep_tmp.json 2>&1 || { echo "FAIL $e"; tail -5 gpurun_out/sweep_tmp.json; exit 1; }
  python - "$e" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/sweep_tmp.json") if l.startswith("{")][-1])
print(f"{sys.argv[1]:40s} ms/step {d['ms_per_step']:7.2f}  value {d['value']:8.3f}")
PY
done
cat $out
