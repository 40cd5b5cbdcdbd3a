export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_grad.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c8_grad.log 2>&1 || { tail -20 gpurun_out/c8_grad.log; exit 1; }
tail -1 gpurun_out/c8_grad.log
timeout -k 10 300 python bench.py --mode grad --steps 5 --warmup 1 --skip-cpu > gpurun_out/c8_grad.json 2>&1 || exit 2
grep -h '^{' gpurun_out/c8_grad.json | cut -c 1-200
python -c "import json;d=json.loads([l for l in open('gpurun_out/c8_grad.json') if l.startswith('{')][-1]);print(d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c8_pf -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-profile > gpurun_out/c8_pf.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c8_pw -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-profile > gpurun_out/c8_pw.log 2>&1 || exit 4
python tools/pmc_traffic.py gpurun_out/c8_pf gpurun_out/c8_pw gpurun_out/c8_traffic_cinv.json cinv_tile_kernel
