"""The gradient restatement (oracle.restatement.logpdf_grad) and the mcmc model's host logic.

The gradient is pinned independently of its closed form: central finite differences of the
(sklearn-pinned, tests/test_oracle.py) logpdf restatement, per term parameter, for the
observation variance and for v. The golden fixtures' gradient fields are re-derived here so
a change to the restatement cannot silently move them. No GPU needed.
"""
import math

import numpy as np
import pytest

from gaplac_amd import formula as F
from gaplac_amd import mcmc as M
from gaplac_amd._native import CAT, LINEAR, NOISE, OU, SQEXP
from oracle import restatement as R
from tests.golden_io import load_cases

CASES = [c for c in load_cases() if not c["info"]]


def _fd_param(X, terms, noise, v, t, rel_h=1e-5):
    h = rel_h * terms[t][2]
    tp = [list(x) for x in terms]
    tm = [list(x) for x in terms]
    tp[t][2] += h
    tm[t][2] -= h
    f = lambda tt: R.logpdf(X, [tuple(x) for x in tt], noise, v)[0]
    return (f(tp) - f(tm)) / (2 * h)


@pytest.mark.parametrize("case", [c for c in CASES if c["N"] <= 300], ids=lambda c: c["name"][:60])
def test_gradient_matches_finite_differences(case):
    X, terms, noise, v = case["X"], case["terms"], case["noise"], case["v"]
    lp, dv, dp, dn = R.logpdf_grad(X, terms, noise, v)
    sc, scn = R.logpdf_grad_scale(X, terms, noise, v)
    assert lp == case["logpdf"]
    for t, (kind, col, param, g) in enumerate(terms):
        if kind == CAT:
            assert dp[t] == 0.0
            continue
        if kind == LINEAR and param == 0.0:
            continue  # c = 0 sits on the boundary c >= 0: no central difference
        fd = _fd_param(X, terms, noise, v, t)
        floor = 10 * 2.2e-16 * max(1.0, abs(lp)) / (1e-5 * param)  # rounding of the difference
        assert abs(dp[t] - fd) <= 1e-6 * (abs(fd) + sc[t]) + floor, (t, dp[t], fd)
    h = 1e-6
    fdn = (R.logpdf(X, terms, noise + h, v)[0] - R.logpdf(X, terms, noise - h, v)[0]) / (2 * h)
    assert abs(dn - fdn) <= 1e-6 * (abs(fdn) + scn)
    i = len(v) // 2
    e = np.zeros(len(v))
    e[i] = 1e-6
    fdv = (R.logpdf(X, terms, noise, v + e)[0] - R.logpdf(X, terms, noise, v - e)[0]) / 2e-6
    assert abs(dv[i] - fdv) <= 1e-6 * max(1.0, abs(fdv))


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"][:60])
def test_golden_gradient_fields_reproduce(case):
    _, dv, dp, dn = R.logpdf_grad(case["X"], case["terms"], case["noise"], case["v"])
    assert np.array_equal(dp, case["dparam"])
    assert dn == case["dnoise"]
    assert np.array_equal(dv, case["dv"])


def test_product_group_gradient_matches_finite_differences():
    rng = np.random.default_rng(7)
    N = 90
    X = np.column_stack([rng.uniform(0, 5, N), rng.normal(size=N), rng.integers(0, 9, N).astype(float)])
    v = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.3, 0), (LINEAR, 1, 0.4, 0), (CAT, 2, 0.0, 0), (OU, 0, 2.5, 1), (NOISE, -1, 0.2, 2)]
    lp, dv, dp, dn = R.logpdf_grad(X, terms, 0.1, v)
    sc, _ = R.logpdf_grad_scale(X, terms, 0.1, v)
    for t in (0, 1, 3, 4):
        fd = _fd_param(X, terms, 0.1, v, t)
        assert abs(dp[t] - fd) <= 1e-6 * (abs(fd) + sc[t])


class _RecordingCtx:
    """Stands in for backend.Context in host-logic tests (no GPU): returns fixed gradients."""

    def __init__(self):
        self.calls = []

    def logpdf_grad(self, X, terms, noise, v):
        self.calls.append((X.copy(), list(terms), noise, np.array(v)))
        T = len(terms)
        return -10.0, -np.asarray(v) * 0.5, np.arange(1.0, T + 1.0), 0.0


def _table(N=20, seed=3):
    rng = np.random.default_rng(seed)
    return {"y": rng.normal(size=N), "x": rng.uniform(-5, 5, N), "t": rng.uniform(0, 10, N),
            "g": rng.integers(0, 4, N).astype(float)}


def test_mcmc_model_ties_lengthscale_to_inferred_variables():
    ctx = _RecordingCtx()
    tab = _table()
    m = M.MCMCModel("y ~| SqExp(:x) + OU(:t; l=3) + Linear(:x)", tab, ["x"], ctx=ctx)
    fx = np.zeros(m.N)
    lp, dell, dfx = m.logdensity_and_gradient(2.5, fx)
    _, terms, noise, _ = ctx.calls[-1]
    assert noise == 0.1
    assert [(k, c, p) for (k, c, p, g) in terms] == [(SQEXP, 0, 2.5), (OU, 1, 3.0), (LINEAR, 2, 2.5)]
    assert dell == 1.0 + 3.0  # terms 0 and 2 carry ℓ (fake dparam = 1, 2, 3)
    r = tab["y"] - fx
    assert lp == pytest.approx(-math.log(20) - 10.0 + float(np.sum(-(R.LOG2PI + r * r) / 2)), rel=1e-15)
    assert np.allclose(dfx, -fx * 0.5 + r)


def test_mcmc_model_lengthscale_one_drops_sqexp_dependence():
    # makekernel(::SqExp, l) = l == 1 ? SqExponentialKernel() : with_lengthscale(...): at ℓ == 1
    # the reference's ForwardDiff sees no ℓ in the SqExp / OU terms; Linear keeps c = ℓ.
    ctx = _RecordingCtx()
    m = M.MCMCModel("y ~| SqExp(:x) + Linear(:t)", _table(), ["x", "t"], ctx=ctx)
    _, dell, _ = m.logdensity_and_gradient(1.0, np.zeros(m.N))
    assert dell == 2.0
    _, dell, _ = m.logdensity_and_gradient(1.5, np.zeros(m.N))
    assert dell == 3.0


def test_mcmc_model_support_and_cat_inference():
    ctx = _RecordingCtx()
    m = M.MCMCModel("y ~| SqExp(:x)", _table(), ["x"], ctx=ctx)
    lp, dell, dfx = m.logdensity_and_gradient(25.0, np.zeros(m.N))
    assert lp == -math.inf and math.isnan(dell) and np.all(np.isnan(dfx))
    assert not ctx.calls
    mc = M.MCMCModel("y ~| Cat(:g)", _table(), ["g"], ctx=ctx)
    with pytest.raises(F.MethodError):
        mc.logdensity_and_gradient(2.0, np.zeros(mc.N))
