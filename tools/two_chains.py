"""Two chains per GPU (bench.py's extra.two_chains_evals_per_s): 16 configs[2] evaluations
at N=16384 through gaplac_logpdf_batch (two lanes), after single evaluations on the same
context (as the bench runs them). usage: python tools/two_chains.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gaplac_amd import configs as CF  # noqa: E402
from gaplac_amd.backend import Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N = CF.N2
X, v = CF.config2_inputs(N)
ctx = Context(0)
dX = torch.from_numpy(np.ascontiguousarray(X.T)).to("cuda")
dv = torch.from_numpy(v).to("cuda")
for i in range(3):  # single evaluations first (the split's second stream, if any, exists now)
    ctx.logpdf_device(N, 2, dX.data_ptr(), N, CF.config2_terms(CF.LENGTHSCALES_2[i % 4]), CF.NOISE_VAR, dv.data_ptr())
models = [CF.config2_terms(CF.LENGTHSCALES_2[i % 4]) for i in range(8)]
ctx.logpdf_batch(X, models[:2], CF.NOISE_VAR, v)
for r in range(reps):
    t0 = time.perf_counter()
    for _ in range(2):
        ctx.logpdf_batch(X, models, CF.NOISE_VAR, v)
    print(f"two chains: {16 / (time.perf_counter() - t0):.2f} evals/s", flush=True)
