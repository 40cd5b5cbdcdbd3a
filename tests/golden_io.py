"""Load the golden fixtures in tests/golden (written by tests/golden/make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _f(x):
    return None if x is None else float.fromhex(x)


def load_cases():
    with open(os.path.join(GOLDEN, "index.json")) as fh:
        names = json.load(fh)
    out = []
    for n in names:
        with open(os.path.join(GOLDEN, n)) as fh:
            c = json.load(fh)
        N, D = c["N"], c["D"]
        c["X"] = np.array([float.fromhex(h) for h in c["X"]]).reshape((N, D), order="F")
        c["v"] = np.array([float.fromhex(h) for h in c["v"]])
        c["terms"] = [(k, col, float.fromhex(p), g) for (k, col, p, g) in c["terms"]]
        c["noise"] = float.fromhex(c["noise"])
        for key in ("logpdf", "logdet", "quad", "gram_sum", "gram_diag_sum", "logpdf_gemm_distances", "dnoise",
                    "dnoise_scale"):
            c[key] = _f(c.get(key))
        for key in ("dv", "dparam", "dparam_scale"):
            if c.get(key) is not None:
                c[key] = np.array([float.fromhex(h) for h in c[key]])
        out.append(c)
    return out
