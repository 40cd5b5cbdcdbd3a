#!/bin/bash
# GPU check after a change: a chosen test file first, then the whole -m gpu suite, then a
# short bench line (headline, configs[1], select).  usage: bash tools/gpu_check.sh TAG [first-test-file]
R=${1:-dev}; FIRST=${2:-tests/test_gpu_parity.py}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 200 python -u -m pytest $FIRST -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$R/first.log 2>&1 || { tail -30 gpurun_out/$R/first.log; exit 1; }
tail -3 gpurun_out/$R/first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/$R/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { tail gpurun_out/$R/bench.err; exit 3; }
python - "$R" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}/bench.json").read().strip().splitlines()[-1])
e = d["extra"]
print("headline %.3f evals/s %.3f ms  bulk frac %.4f  n4096 %.4f ms  n65536 %.1f ms  select %.1f/s" % (
    d["value"], d["ms_per_step"], d["roofline"]["frac"], e["n4096"]["ms_per_eval"], e["n65536"]["ms_per_eval"],
    e["select"]["evals_per_s"]))
PY
