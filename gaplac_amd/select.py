"""`select` model comparison on the host: the `--chains` path and
the table output helper, mirroring CLI/src/select.jl:9-20,54 and src/utils.jl:30-40.

    --chains c1.csv c2.csv:
        lp_k  = log2(harmmean([BigFloat(2)^x for x in chain_k[!, :lp]]))   (select.jl:16-19)
        bayes = log2(BigFloat(2)^lp1 / BigFloat(2)^lp2)                   (select.jl:20)
    --formulae f1 f2: lp_k = logpdf(FiniteGP_k, y_k) on the GPU (abstractgps.select_formulae),
        bayes as above (select.jl:54).

The reference works in BigFloat so that 2^x neither overflows nor underflows. Here the
same quantities are computed in log space: harmmean(2^x) = n / sum(2^-x), so
lp = log2(n) - log2(sum_i 2^-x_i) with a max-shifted sum, and log2(2^a / 2^b) = a - b
(the printed "Log2 Bayes" is exactly lp1 - lp2). Relative to the BigFloat value
rounded to Float64 this is within a few ulps, far inside the 3 decimals the CLI prints.
"""
from __future__ import annotations

import csv
import math
import os
from typing import Dict, Iterable, List, Sequence

import numpy as np

from . import formula as F


def log2_harmmean_pow2(xs: Iterable[float]) -> float:
    """log2(harmmean(2 .^ xs)) (StatsBase.harmmean on BigFloat(2)^x, select.jl:17)."""
    x = np.asarray(list(xs), dtype=np.float64)
    if x.size == 0:
        raise F.ArgumentError("harmmean of an empty collection")
    if np.any(np.isnan(x)):
        return math.nan
    neg = -x
    m = float(np.max(neg))
    if math.isinf(m):  # some x = -inf: 2^x = 0, harmmean = 0
        return -math.inf if m > 0 else math.inf
    s = float(np.sum(np.exp2(neg - m)))
    return math.log2(x.size) - (m + math.log2(s))


def read_table(path: str) -> Dict[str, List[str]]:
    """CSV.read(path, DataFrame) for the delimited files the CLI writes (',' or tab)."""
    with open(path, newline="") as fh:
        head = fh.readline()
        delim = "\t" if head.count("\t") > head.count(",") else ","
        fh.seek(0)
        rows = list(csv.reader(fh, delimiter=delim))
    if not rows:
        raise F.ArgumentError(f"{path}: empty table")
    names = [c.strip() for c in rows[0]]
    cols: Dict[str, List[str]] = {n: [] for n in names}
    for r in rows[1:]:
        if not r:
            continue
        for n, v in zip(names, r):
            cols[n].append(v.strip())
    return cols


def select_chains(chain1: str, chain2: str):
    """`gaplac select --chains chain1 chain2`: (bayes, lp1, lp2) from the chains' :lp columns."""
    lps = []
    for path in (chain1, chain2):
        t = read_table(path)
        if "lp" not in t:
            raise F.ArgumentError(f"{path}: no :lp column")
        lps.append(log2_harmmean_pow2(float(v) for v in t["lp"]))
    lp1, lp2 = lps
    return lp1 - lp2, lp1, lp2


def df_output(table: Dict[str, Sequence], output: str | None):
    """src/utils.jl:30-40 (_df_output): write the table as .csv / .tsv, or return its text
    rendering when no output path is given (the reference @shows the DataFrame)."""
    names = list(table.keys())
    n = len(next(iter(table.values()))) if names else 0
    if output is None:
        lines = ["\t".join(names)] + ["\t".join(_fmt(table[c][i]) for c in names) for i in range(n)]
        return "\n".join(lines)
    if output.endswith("csv"):
        delim = ","
    elif output.endswith("tsv"):
        delim = "\t"
    else:
        raise RuntimeError("--output arg must be '.tsv' or '.csv'")
    with open(os.path.expanduser(output), "w", newline="") as fh:
        w = csv.writer(fh, delimiter=delim, lineterminator="\n")
        w.writerow(names)
        for i in range(n):
            w.writerow([_fmt(table[c][i]) for c in names])
    return output


def julia_float(f: float) -> str:
    """Float64 as Julia prints it (CSV.jl / show): the shortest round-trip digits (the same
    digits Python's repr picks), decimal notation for 1e-4 <= |x| < 1e6, otherwise
    d.ddde[-]x; always at least one fractional digit; NaN / Inf / -Inf."""
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "Inf" if f > 0 else "-Inf"
    if f == 0.0:
        return "-0.0" if math.copysign(1.0, f) < 0 else "0.0"
    from decimal import Decimal
    sign, digits, exp = Decimal(repr(f)).as_tuple()
    digits = list(digits)
    while len(digits) > 1 and digits[-1] == 0:
        digits.pop()
        exp += 1
    e10 = len(digits) - 1 + exp
    sgn = "-" if sign else ""
    ds = "".join(str(d) for d in digits)
    if -4 <= e10 < 6:
        if e10 >= 0:
            ip = ds[: e10 + 1].ljust(e10 + 1, "0")
            fp = ds[e10 + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e10 - 1) + ds
        return f"{sgn}{ip}.{fp}"
    return f"{sgn}{ds[0]}.{ds[1:] or '0'}e{e10}"


def _fmt(v) -> str:
    if isinstance(v, (float, np.floating)):
        return julia_float(float(v))
    return str(v)
