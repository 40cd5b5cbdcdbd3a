#!/bin/bash
R=${1:-r03g}
export TMPDIR=/tmp
mkdir -p gpurun_out/$R
rm -f gpurun_out/$R/tail_trace.txt
GAPLAC_TAIL_TRACE=gpurun_out/$R/tail_trace.txt timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0, '.')
from tools.quick_tail import *
from gaplac_amd import configs as CF
import numpy as np
c = Context(0)
x, v = CF.config1_inputs(); N = x.shape[0]
for i in range(3): c.logpdf(x.reshape(N, 1), CF.config1_terms(1.5), CF.NOISE_VAR, v)
" > gpurun_out/$R/trace_run.txt 2>&1 || { cat gpurun_out/$R/trace_run.txt; exit 11; }
python tools/tail_trace.py gpurun_out/$R/tail_trace.txt && timeout -k 10 120 python -u tools/quick_tail.py
