#!/bin/bash
# Bench under several environment settings (one line each): bash tools/env_sweep.sh TAG "ENV1" "ENV2" ...
TAG=$1; shift
export TMPDIR=/tmp
out=gpurun_out/sweep_$TAG.txt
: > $out
for e in "$@"; do
  env $e timeout -k 10 200 python bench.py --steps 10 --warmup 2 --skip-cpu > gpurun_out/sweep_tmp.json 2>&1 || { echo "FAIL $e"; tail -5 gpurun_out/sweep_tmp.json; exit 1; }
  python - "$e" >> $out <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/sweep_tmp.json") if l.startswith("{")][-1])
x = d["extra"]
print(f"{sys.argv[1]:40s} ms/step {d['ms_per_step']:7.2f}  syrk {x.get('syrk_ms_per_eval',0):6.2f} diag {x.get('diag_ms_per_eval',0):6.2f} trsm {x.get('trsm_ms_per_eval',0):6.2f} col {x.get('colupd_ms_per_eval',0):6.2f} span {x.get('profiled_span_ms_per_eval',0):6.2f}")
PY
done
cat $out
