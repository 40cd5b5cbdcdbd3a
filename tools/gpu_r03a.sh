#!/bin/bash
# Round-3 first GPU check: latency probes, diag probe, GPU suite, smoke, bench.
R=${1:-r03a}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 60 ./tools/bin/lat_chain_probe > gpurun_out/$R/lat_chain.txt 2>&1 || exit 11
cat gpurun_out/$R/lat_chain.txt
timeout -k 10 60 ./tools/bin/diag_probe > gpurun_out/$R/diag_probe.txt 2>&1 || exit 12
head -20 gpurun_out/$R/diag_probe.txt
bash tools/final_check.sh $R
