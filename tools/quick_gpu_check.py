"""Quick GPU parity probe used during development (not a test)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gaplac_amd.backend import Context
from oracle import restatement as R

ctx = Context(0)
rng = np.random.default_rng(1)
for N in [5, 100, 127, 128, 129, 300, 1000, 2047]:
    X = np.column_stack([rng.uniform(-5, 5, N), rng.integers(0, max(1, N // 3), N).astype(float)])
    v = rng.standard_normal(N)
    terms = [(1, 0, 1.5, 0), (2, 0, 3.0, 1), (4, 1, 0.0, 2)]
    t0 = time.time(); lp, ld, q = ctx.logpdf(X, terms, 0.1, v, full=True); t1 = time.time()
    rl, rd, rq = R.logpdf(X, terms, 0.1, v)
    G = ctx.gram(X, terms, 0.1); Gr = R.gram(X, terms, 0.1)
    print(N, lp, rl, abs(lp - rl) / abs(rl), "ld", abs(ld-rd)/abs(rd), "q", abs(q-rq)/abs(rq), "gram maxdiff", np.abs(G-Gr).max(), f"{(t1-t0)*1e3:.2f}ms", flush=True)
