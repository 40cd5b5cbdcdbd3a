"""`select --chains` (host arithmetic, CLI/src/select.jl:16-20) and the table writer
(src/utils.jl:30-40). The BigFloat harmonic mean is re-derived with Python's decimal
module at 80 digits; no GPU needed."""
import math
from decimal import Decimal, getcontext

import numpy as np
import pytest

from gaplac_amd import select as S


def _ref_log2_harmmean(xs):
    getcontext().prec = 80
    two = Decimal(2)
    n = len(xs)
    inv = sum((two ** Decimal(-float(x))) for x in xs)
    hm = Decimal(n) / inv
    return float(hm.ln() / two.ln())


@pytest.mark.parametrize("scale", [1.0, 50.0, 2000.0])
def test_log2_harmmean_matches_bigfloat(scale):
    rng = np.random.default_rng(int(scale))
    xs = -scale * rng.uniform(0.5, 1.5, 400)  # 2^x under/overflows Float64 for scale 2000
    got = S.log2_harmmean_pow2(xs)
    ref = _ref_log2_harmmean(xs)
    assert abs(got - ref) <= 1e-12 * abs(ref)


def test_select_chains_files(tmp_path):
    rng = np.random.default_rng(1)
    a = -81.0 + rng.normal(size=300)
    b = -89.5 + rng.normal(size=300)
    p1, p2 = tmp_path / "c1.csv", tmp_path / "c2.tsv"
    S.df_output({"iteration": list(range(1, 301)), "lp": list(a)}, str(p1))
    S.df_output({"iteration": list(range(1, 301)), "lp": list(b)}, str(p2))
    bayes, lp1, lp2 = S.select_chains(str(p1), str(p2))
    assert abs(lp1 - _ref_log2_harmmean(a)) <= 1e-12 * abs(lp1)
    assert abs(lp2 - _ref_log2_harmmean(b)) <= 1e-12 * abs(lp2)
    # the printed "Log2 Bayes" is lp1 - lp2 (README.md:84-89: -81.29118 vs
    # -89.69639 -> 8.405)
    assert bayes == lp1 - lp2
    assert round(-81.29118 - -89.69639, 3) == 8.405


def test_df_output_formats(tmp_path):
    t = {"x": [1.0, 1e-5, 1234567.0, -0.5], "g": ["a", "b", "c", "d"]}
    out = tmp_path / "o.tsv"
    S.df_output(t, str(out))
    lines = out.read_text().splitlines()
    assert lines[0] == "x\tg"
    assert lines[1:] == ["1.0\ta", "1.0e-5\tb", "1.234567e6\tc", "-0.5\td"]
    with pytest.raises(RuntimeError):
        S.df_output(t, str(tmp_path / "o.txt"))
    assert S.julia_float(float("nan")) == "NaN" and S.julia_float(-math.inf) == "-Inf"
    assert S.julia_float(0.1) == "0.1" and S.julia_float(123456.0) == "123456.0"
