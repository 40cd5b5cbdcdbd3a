#!/bin/bash
# Round profile capture: kernel-trace stats of the benchmark command (default mode and the
# gradient mode), two PMC passes per dominant kernel (FETCH_SIZE, WRITE_SIZE; counters never
# combined with tracing domains), then the full default bench.
# usage: bash tools/profile_round.sh rNN
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --skip-cpu --no-extra > gpurun_out/$R/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace_grad -o run --output-format csv -- python bench.py --mode grad --steps 3 --warmup 1 --skip-cpu --no-extra > gpurun_out/$R/trace_grad.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$R/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --skip-cpu --no-extra --no-profile > gpurun_out/$R/pmc_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$R/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --skip-cpu --no-extra --no-profile > gpurun_out/$R/pmc_write.log 2>&1 || exit 4
python tools/pmc_traffic.py gpurun_out/$R/pmc_fetch gpurun_out/$R/pmc_write gpurun_out/$R/traffic_syrk.json || exit 5
python tools/pmc_traffic.py gpurun_out/$R/pmc_fetch gpurun_out/$R/pmc_write gpurun_out/$R/traffic_gram.json gram_queue_kernel || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$R/pmc_fetch_g -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-extra --no-profile > gpurun_out/$R/pmc_fetch_g.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$R/pmc_write_g -o run --output-format csv -- python bench.py --mode grad --steps 1 --warmup 1 --skip-cpu --no-extra --no-profile > gpurun_out/$R/pmc_write_g.log 2>&1 || exit 7
python tools/pmc_traffic.py gpurun_out/$R/pmc_fetch_g gpurun_out/$R/pmc_write_g gpurun_out/$R/traffic_cinv.json cinv_contract_kernel || exit 8
timeout -k 10 400 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || exit 9
cat gpurun_out/$R/bench.json
