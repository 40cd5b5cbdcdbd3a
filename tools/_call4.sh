export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --skip-cpu > gpurun_out/c4_bench.json 2> gpurun_out/c4_bench.err || { tail gpurun_out/c4_bench.err; exit 1; }
timeout -k 10 400 python bench.py --mode grad --steps 5 --warmup 1 > gpurun_out/c4_grad.json 2> gpurun_out/c4_grad.err || { tail gpurun_out/c4_grad.err; exit 2; }
python - <<'PY'
import json
for f in ("gpurun_out/c4_bench.json", "gpurun_out/c4_grad.json"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, d["value"], d["ms_per_step"], json.dumps(d.get("roofline"))[:300])
    print(json.dumps(d.get("extra"))[:900]); print(json.dumps(d.get("cpu_baseline")))
PY
