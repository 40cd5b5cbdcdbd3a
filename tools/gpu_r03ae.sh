#!/bin/bash
# batched-tail task timeline (32 x N = 8192)
R=${1:-r03ae}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 200 python -u tools/batch_trace.py gpurun_out/$R/btrace.txt > gpurun_out/$R/btrace.log 2>&1 || { tail gpurun_out/$R/btrace.log; exit 1; }
python tools/tail_trace.py gpurun_out/$R/btrace.txt | grep -vE "^ *[0-9]+ " > gpurun_out/$R/btrace_summary.txt
cat gpurun_out/$R/btrace_summary.txt
rm -f gpurun_out/$R/btrace.txt
