#!/bin/bash
# cinv_tile_kernel k-walk A/B: new build (downward) vs tools/bin/libbase.so (upward):
# gradient tests, grad bench, FETCH/WRITE PMC of cinv per build
R=${1:-r03y}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u -m pytest tests/test_gpu_grad.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$R/pytest_grad.log 2>&1 || { tail -30 gpurun_out/$R/pytest_grad.log; exit 1; }
tail -2 gpurun_out/$R/pytest_grad.log
for arm in new base new base; do
  if [ $arm = base ]; then export GAPLAC_LIB_PATH=$PWD/tools/bin/libbase.so; else unset GAPLAC_LIB_PATH; fi
  timeout -k 10 120 python bench.py --mode grad --steps 4 --warmup 1 --skip-cpu > gpurun_out/$R/grad_$arm.json 2> gpurun_out/$R/grad_$arm.err || { tail gpurun_out/$R/grad_$arm.err; exit 2; }
  python -c "import json; d=json.loads(open('gpurun_out/$R/grad_$arm.json').read().strip().splitlines()[-1]); print('$arm', round(d['ms_per_step'],2), 'ms cinv', (d.get('roofline') or {}).get('avg_launch_ms'), d['extra'].get('last_logpdf'))"
done
for arm in new base; do
  if [ $arm = base ]; then export GAPLAC_LIB_PATH=$PWD/tools/bin/libbase.so; else unset GAPLAC_LIB_PATH; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$R/pf_$arm -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/pf_$arm.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$R/pw_$arm -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/pw_$arm.log 2>&1 || exit 4
  python tools/pmc_traffic.py gpurun_out/$R/pf_$arm gpurun_out/$R/pw_$arm gpurun_out/$R/traffic_cinv_$arm.json cinv_tile_kernel || exit 5
done
