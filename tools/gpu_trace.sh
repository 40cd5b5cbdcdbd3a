#!/bin/bash
# Task trace of the persistent tail (GAPLAC_TAIL_TRACE) at order N (configs[1]/[2]-style
# terms, 3 evaluations; the last one is analysed by tools/tail_stats.py).
# usage: bash tools/gpu_trace.sh TAG [N]
R=${1:-dev}; N=${2:-4096}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
rm -f gpurun_out/$R/tail_trace_$N.txt
GAPLAC_TAIL_TRACE=gpurun_out/$R/tail_trace_$N.txt timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0, '.')
import numpy as np
from gaplac_amd.backend import Context
from gaplac_amd import configs as CF
c = Context(0)
N = $N
if N == 4096:
    x, v = CF.config1_inputs(); X = x.reshape(N, 1); terms = CF.config1_terms(1.5)
else:
    X, v = CF.config2_inputs(N); terms = CF.config2_terms(1.5)
for i in range(3): c.logpdf(X, terms, CF.NOISE_VAR, v)
" > gpurun_out/$R/trace_run_$N.txt 2>&1 || { cat gpurun_out/$R/trace_run_$N.txt; exit 11; }
python tools/tail_stats.py gpurun_out/$R/tail_trace_$N.txt
