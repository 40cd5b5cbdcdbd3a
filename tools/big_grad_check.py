"""One-off check of the gradient / posterior entries at BASELINE configs[3]'s N=65536
(workspace offsets beyond 2^31 elements): dlogp/dl against a central difference of the
GPU logpdf, and the posterior-mean identity mean(X) = y - noise * alpha."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gaplac_amd.backend import Context  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rng = np.random.default_rng(3)
x = rng.uniform(-5, 5, N)
v = rng.standard_normal(N)
X = x[:, None]
terms = [(1, 0, 1.5, 0)]
ctx = Context(0)
t = time.perf_counter()
lp, dv, dp, dn = ctx.logpdf_grad(X, terms, 0.1, v)
print(f"N={N} grad eval {time.perf_counter() - t:.2f} s  logpdf {lp!r}  dl {dp[0]!r}  dnoise {dn!r}", flush=True)
h = 1e-4 * 1.5
fd = (ctx.logpdf(X, [(1, 0, 1.5 + h, 0)], 0.1, v) - ctx.logpdf(X, [(1, 0, 1.5 - h, 0)], 0.1, v)) / (2 * h)
print(f"central difference {fd!r}  rel {abs(fd - dp[0]) / abs(fd):.2e}", flush=True)
assert abs(fd - dp[0]) <= 1e-5 * abs(fd) + 1e-8 * abs(lp) / h
idx = rng.choice(N, 256, replace=False)
m, var = ctx.posterior_mean_var(X, terms, 0.1, v, X[idx])
err = np.max(np.abs(m - (v[idx] + 0.1 * dv[idx])))
print(f"posterior mean identity max err {err:.2e}; var range [{var.min():.3e}, {var.max():.3e}]", flush=True)
assert err <= 1e-7 * max(1.0, np.max(np.abs(v)))
print("ok")
