#!/bin/bash
R=${1:-r03j}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u tools/tail_sweep.py 2>&1 | tee gpurun_out/$R/tail_sweep.txt
