"""A/B of one environment switch at N = 4096 and 16384 (configs[1], configs[2] workloads,
device-resident inputs; tail_sweep.bench).  usage: python tools/ab_sweep.py VAR v1,v2,..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tail_sweep import CF, CAT, NOISE, OU, SQEXP, bench  # noqa: E402


def main():
    var = sys.argv[1]
    vals = sys.argv[2].split(",")
    t1 = lambda i: CF.config1_terms(CF.LENGTHSCALES_1[i % 4])  # noqa: E731
    t2 = lambda i: [(SQEXP, 0, (0.8, 1.0, 1.2, 1.5)[i % 4], 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]  # noqa: E731
    for N, fn, reps in ((16384, t2, 6), (4096, t1, 20)):
        for v in vals:
            ms, lp = bench({var: v} if v != "-" else {}, N, fn, reps)
            print(f"N={N} {var}={v:4s} {ms:8.3f} ms/eval  logpdf {lp!r}", flush=True)


if __name__ == "__main__":
    main()
