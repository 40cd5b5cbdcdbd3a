export TMPDIR=/tmp; R=r04c; mkdir -p gpurun_out/$R
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_grad.py tests/test_gpu_schedules.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest.log 2>&1 || { tail -30 gpurun_out/$R/pytest.log; exit 1; }
tail -1 gpurun_out/$R/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { tail gpurun_out/$R/bench.err; exit 3; }
python - $R <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}/bench.json").read().strip().splitlines()[-1]); e = d["extra"]
print("headline %.3f evals/s %.3f ms bulk %.4f n4096 %.4f ms n65536 %.1f ms select %.1f/s" % (d["value"], d["ms_per_step"], d["roofline"]["frac"], e["n4096"]["ms_per_eval"], e["n65536"]["ms_per_eval"], e["select"]["evals_per_s"]))
PY
timeout -k 10 300 python bench.py --mode grad --steps 6 --warmup 2 --skip-cpu > gpurun_out/$R/grad.json 2>&1 || { tail gpurun_out/$R/grad.json; exit 4; }
python -c "import json; d=json.loads(open('gpurun_out/$R/grad.json').read().strip().splitlines()[-1]); print('grad', d['value'], d['ms_per_step'])"
bash tools/gpu_trace.sh $R 4096 > gpurun_out/$R/t4096.txt 2>&1 || exit 5
bash tools/gpu_trace.sh $R 16384 > gpurun_out/$R/t16384.txt 2>&1 || exit 6
cat gpurun_out/$R/t4096.txt gpurun_out/$R/t16384.txt
