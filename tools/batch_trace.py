"""Task timeline of one batched tail launch: 32 configs[4] models at
N = 8192 through gaplac_logpdf_batch with GAPLAC_TAIL_TRACE set, then tools/tail_trace.py
on the last launch.  usage: python tools/batch_trace.py OUT_FILE"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = sys.argv[1]
if os.path.exists(out):
    os.remove(out)
os.environ["GAPLAC_TAIL_TRACE"] = out
from gaplac_amd import configs as CF  # noqa: E402
from gaplac_amd.backend import Context  # noqa: E402

X, y = CF.config4_inputs(CF.N4)
models = CF.select_models()[:32]
with Context(0) as c:
    c.logpdf_batch(X, models, CF.NOISE_VAR, y)
    c.logpdf_batch(X, models, CF.NOISE_VAR, y)
