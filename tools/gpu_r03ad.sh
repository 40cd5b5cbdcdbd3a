#!/bin/bash
# double-buffered batched tail (Grams on s_panel beside the previous tail): GPU suite, select, default bench
R=${1:-r03ad}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$R/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$R/pytest_gpu.log
for i in 1 2; do
timeout -k 10 200 python bench.py --mode select --steps 3 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/sel_$i.json 2>> gpurun_out/$R/select.err || exit 11
python -c "import json; d = json.loads(open('gpurun_out/$R/sel_$i.json').read().strip().splitlines()[-1]); print('select', round(d['value'], 1), round(d['ms_per_step'], 1))"
done
timeout -k 10 500 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { tail gpurun_out/$R/bench.err; exit 12; }
python - <<PY
import json
d = json.loads(open("gpurun_out/$R/bench.json").read().strip().splitlines()[-1])
e = d["extra"]
print("bench", round(d["value"], 2), "evals/s", round(d["ms_per_step"], 3), "ms; frac", d["roofline"]["frac"], "cpu", d["cpu_baseline"]["value"])
print("n4096", e["n4096"] and round(e["n4096"]["evals_per_s"], 1), "n65536", e["n65536"] and round(e["n65536"]["ms_per_eval"], 1), "select", e["select"] and round(e["select"]["evals_per_s"], 1))
PY
