"""A/B of one environment switch at chosen sizes (configs[2]-style terms; configs[1] at
N = 4096; device-resident inputs; tail_sweep.bench).  usage: python tools/ab_n.py VAR v1,v2,.. N1,N2,.."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tail_sweep import CAT, CF, NOISE, OU, SQEXP, bench  # noqa: E402


def main():
    var = sys.argv[1]
    vals = sys.argv[2].split(",")
    ns = [int(x) for x in sys.argv[3].split(",")]
    t2 = lambda i: [(SQEXP, 0, (0.8, 1.0, 1.2, 1.5)[i % 4], 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]  # noqa: E731
    for N in ns:
        reps = max(4, min(40, int(4 * (16384 / N) ** 2)))
        for v in vals:
            fn = (lambda i: CF.config1_terms(CF.LENGTHSCALES_1[i % 4])) if N == 4096 else t2  # configs[1] at 4096
            ms, lp = bench({var: v} if v != "-" else {}, N, fn, reps)
            print(f"N={N} {var}={v:4s} {ms:8.3f} ms/eval  logpdf {lp!r}", flush=True)


if __name__ == "__main__":
    main()
