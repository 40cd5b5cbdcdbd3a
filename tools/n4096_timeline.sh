#!/bin/bash
# configs[1] wall time per evaluation, then the same evaluations under a kernel trace and
# their split into kernels and gaps (tools/n4096_timeline.py).  usage: bash tools/n4096_timeline.sh TAG
R=${1:-dev}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
timeout -k 10 120 python -u tools/n4096_timeline.py run 40 > gpurun_out/$R/n4096_wall.txt 2>&1 || { cat gpurun_out/$R/n4096_wall.txt; exit 1; }
cat gpurun_out/$R/n4096_wall.txt
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$R/n4096_trace -o run -- python3 tools/n4096_timeline.py run 20 > gpurun_out/$R/n4096_prof.log 2>&1 || { tail -20 gpurun_out/$R/n4096_prof.log; exit 2; }
D=$(dirname $(find gpurun_out/$R/n4096_trace -name run_kernel_trace.csv | head -1))
python tools/n4096_timeline.py analyse $D > gpurun_out/$R/n4096_timeline.txt && cat gpurun_out/$R/n4096_timeline.txt
