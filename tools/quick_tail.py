"""Quick check of the persistent tail (tail_kernel) against the per-column tail and the
oracle, and evals/s at BASELINE configs[1] (N = 4096) and a few other sizes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaplac_amd.backend import Context  # noqa: E402
from gaplac_amd import configs as CF  # noqa: E402
from oracle import restatement as R  # noqa: E402
from gaplac_amd._native import CAT, NOISE, OU, SQEXP  # noqa: E402

TERMS = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]


def ctx_env(v):
    os.environ["GAPLAC_TAILK"] = v
    c = Context(0)
    os.environ.pop("GAPLAC_TAILK")
    return c


def main():
    on, off = ctx_env("1"), ctx_env("0")
    for N in [129, 700, 2049, 3000, 4096, 9000]:
        rng = np.random.default_rng(N)
        X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, max(1, N // 3), N).astype(float)])
        v = rng.standard_normal(N)
        a = on.logpdf(X, TERMS, 0.1, v, full=True)
        b = off.logpdf(X, TERMS, 0.1, v, full=True)
        r = R.logpdf(X, TERMS, 0.1, v)[0] if N <= 4096 else b[0]
        print(f"N={N}: tailk {a[0]!r} launches {b[0]!r} oracle {r!r} rel {abs(a[0] - r) / abs(r):.2e}", flush=True)
    x, v = CF.config1_inputs()
    N = x.shape[0]
    X = x.reshape(N, 1)
    for name, c in (("tailk", on), ("launches", off)):
        for i in range(3):
            c.logpdf(X, CF.config1_terms(CF.LENGTHSCALES_1[i % 4]), CF.NOISE_VAR, v)
        t0 = time.perf_counter()
        n = 20
        for i in range(n):
            c.logpdf(X, CF.config1_terms(CF.LENGTHSCALES_1[i % 4]), CF.NOISE_VAR, v)
        dt = (time.perf_counter() - t0) / n
        print(f"configs[1] N={N} {name}: {dt * 1e3:.3f} ms/eval ({1 / dt:.1f} evals/s, host inputs)", flush=True)
    on.close()
    off.close()


if __name__ == "__main__":
    main()
