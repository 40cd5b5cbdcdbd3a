"""A/B of the tail length at N = 4096 and 16384 (configs[1], configs[2] workloads,
device-resident inputs): ms per evaluation for GAPLAC_TAIL_S in a list (default 48)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from gaplac_amd.backend import Context, PosDefException  # noqa: E402
from gaplac_amd import configs as CF  # noqa: E402
from gaplac_amd._native import CAT, NOISE, OU, SQEXP  # noqa: E402


def bench(env, N, terms_fn, reps):
    for k, v in env.items():
        os.environ[k] = v
    c = Context(0)
    for k in env:
        os.environ.pop(k)
    if N == 4096:
        x, v = CF.config1_inputs()
        X = x.reshape(N, 1)
    else:
        rng = np.random.default_rng(2)
        X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, N // 3, N).astype(float)])
        v = rng.standard_normal(N)
    dX = torch.from_numpy(np.ascontiguousarray(X.T)).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    D = X.shape[1]
    lp = None

    def one(i):
        # a timing-only build (GAPLAC_CHAIN_SKIP) factors garbage: its non-PD result is
        # reported as lp = None, the evaluation's time still counts
        try:
            return c.logpdf_device(N, D, dX.data_ptr(), N, terms_fn(i), 0.1, dv.data_ptr())
        except PosDefException:
            return None

    for i in range(2):
        lp = one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        lp = one(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    c.close()
    return dt * 1e3, lp


def main():
    t1 = lambda i: CF.config1_terms(CF.LENGTHSCALES_1[i % 4])  # noqa: E731
    t2 = lambda i: [(SQEXP, 0, (0.8, 1.0, 1.2, 1.5)[i % 4], 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]  # noqa: E731
    envs = [("tail64", {"GAPLAC_TAIL_S": "64"}), ("tail48", {}), ("tail40", {"GAPLAC_TAIL_S": "40"}),
            ("tail32", {"GAPLAC_TAIL_S": "32"}), ("tail24", {"GAPLAC_TAIL_S": "24"})]
    for N, fn, reps in ((4096, t1, 20), (16384, t2, 6)):
        for name, env in envs:
            ms, lp = bench(env, N, fn, reps)
            print(f"N={N} {name:10s} {ms:8.3f} ms/eval  logpdf {lp!r}", flush=True)


if __name__ == "__main__":
    main()
