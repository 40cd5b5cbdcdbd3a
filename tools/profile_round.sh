#!/bin/bash
# Round profile capture: kernel-trace stats of the benchmark command, two PMC passes
# (FETCH_SIZE, WRITE_SIZE; counters never combined with tracing domains), full bench.
# usage: bash tools/profile_round.sh rNN
R=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --skip-cpu > gpurun_out/$R/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$R/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/pmc_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$R/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --skip-cpu --no-profile > gpurun_out/$R/pmc_write.log 2>&1 || exit 3
python tools/pmc_traffic.py gpurun_out/$R/pmc_fetch gpurun_out/$R/pmc_write gpurun_out/$R/traffic_syrk.json || exit 4
timeout -k 10 400 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || exit 5
cat gpurun_out/$R/bench.json
