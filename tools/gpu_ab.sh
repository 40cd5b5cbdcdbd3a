#!/bin/bash
# A/B sweep of one switch (args: R VAR values), then a 16k kernel trace with VAR=last value
R=$1; VAR=$2; VALS=$3
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 300 python -u tools/ab_sweep.py $VAR $VALS > gpurun_out/$R/ab.txt 2>&1; rc=$?
cat gpurun_out/$R/ab.txt
[ $rc -eq 0 ] || exit 13
LAST=${VALS##*,}
env $VAR=$LAST timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/trace16k -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --skip-cpu > gpurun_out/$R/trace16k.log 2>&1 || exit 14
python tools/span.py gpurun_out/$R/trace16k | head -3
