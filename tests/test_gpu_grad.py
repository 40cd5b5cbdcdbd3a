"""Parity of gaplac_logpdf_grad (HIP, through the C-ABI) against the gradient restatement.

Tolerance (north_star: <= 1e-9 relative fp64): logpdf <= 1e-9 relative; every gradient
entry within 1e-9 of the magnitude it is summed from, |g - g_ref| <= 1e-9 * (|g_ref| +
scale), scale = 1/2 sum_ij |alpha_i alpha_j - Cinv_ij| |dC_ij| (oracle.logpdf_grad_scale;
an entry that cancels to ~0 is judged against the size of its addends); dv within 1e-9 of
max |dv|. At N = 4096 / 16384 (beyond the oracle's budget) the gradient is checked against
central differences of the GPU's own logpdf (a size-independent property).
"""
import math

import numpy as np
import pytest

from gaplac_amd import mcmc as M
from gaplac_amd._native import CAT, LINEAR, NOISE, OU, SQEXP
from gaplac_amd.backend import Context, PosDefException
from oracle import restatement as R
from tests.conftest import gpu_available
from tests.golden_io import load_cases

pytestmark = pytest.mark.gpu
TOL = 1e-9

CASES = load_cases()


@pytest.fixture(scope="module")
def ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    c = Context(0)
    yield c
    c.close()


def check_grad(got, ref, scale, scalen):
    lp, dv, dp, dn = got
    rlp, rdv, rdp, rdn = ref
    assert abs(lp - rlp) <= TOL * abs(rlp)
    assert np.max(np.abs(dv - rdv)) <= TOL * max(1.0, np.max(np.abs(rdv)))
    for t in range(len(rdp)):
        assert abs(dp[t] - rdp[t]) <= TOL * (abs(rdp[t]) + scale[t]), (t, dp[t], rdp[t], scale[t])
    assert abs(dn - rdn) <= TOL * (abs(rdn) + scalen), (dn, rdn)


@pytest.mark.parametrize("case", CASES, ids=[c["name"][:60] for c in CASES])
def test_golden_gradients(ctx, case):
    if case["info"]:
        with pytest.raises(PosDefException) as ei:
            ctx.logpdf_grad(case["X"], case["terms"], case["noise"], case["v"])
        assert ei.value.info == case["info"]
        return
    got = ctx.logpdf_grad(case["X"], case["terms"], case["noise"], case["v"])
    ref = (case["logpdf"], case["dv"], case["dparam"], case["dnoise"])
    check_grad(got, ref, case["dparam_scale"], case["dnoise_scale"])


@pytest.mark.parametrize("N", [1, 3, 127, 128, 129, 255, 256, 257, 511, 513, 640, 1000])
def test_sizes_composite(ctx, N):
    rng = np.random.default_rng(N)
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, max(1, N // 3), N).astype(float),
                         rng.normal(size=N)])
    v = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (LINEAR, 2, 0.5, 3), (NOISE, -1, 0.05, 4)]
    got = ctx.logpdf_grad(X, terms, 0.1, v)
    ref = R.logpdf_grad(X, terms, 0.1, v)
    sc, scn = R.logpdf_grad_scale(X, terms, 0.1, v)
    check_grad(got, ref, sc, scn)


def test_product_groups(ctx):
    rng = np.random.default_rng(11)
    N = 333
    X = np.column_stack([rng.uniform(0, 5, N), rng.normal(size=N), rng.integers(0, 20, N).astype(float)])
    v = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.3, 0), (LINEAR, 1, 0.4, 0), (CAT, 2, 0.0, 0), (OU, 0, 2.5, 1), (NOISE, -1, 0.2, 2)]
    got = ctx.logpdf_grad(X, terms, 0.1, v)
    check_grad(got, R.logpdf_grad(X, terms, 0.1, v), *R.logpdf_grad_scale(X, terms, 0.1, v))


def test_grad_and_plain_evaluations_interleave(ctx):
    # the workspace switches between the plain (lda = Np) and gradient (lda = 2 Np) layouts
    rng = np.random.default_rng(5)
    N = 700
    X = rng.uniform(-5, 5, (N, 1))
    v = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.1, 0)]
    a = ctx.logpdf(X, terms, 0.1, v)
    g1 = ctx.logpdf_grad(X, terms, 0.1, v)
    b = ctx.logpdf(X, terms, 0.1, v)
    g2 = ctx.logpdf_grad(X, terms, 0.1, v)
    assert a == b == g1[0] == g2[0]
    assert np.array_equal(g1[1], g2[1]) and np.array_equal(g1[2], g2[2]) and g1[3] == g2[3]


def test_nonpd_raises(ctx):
    N = 64
    X = np.repeat(np.arange(16.0), 4)[:, None]
    with pytest.raises(PosDefException) as ei:
        ctx.logpdf_grad(X, [(CAT, 0, 0.0, 0)], 0.0, np.ones(N))
    assert ei.value.info > 0


@pytest.mark.parametrize("N", [4096, 16384])
def test_large_n_finite_differences(ctx, N):
    rng = np.random.default_rng(2)
    t = rng.uniform(0, 10, N)
    g = rng.integers(0, N // 3, N).astype(float)
    X = np.column_stack([t, t, g])
    v = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.5, 0), (OU, 1, 3.0, 1), (CAT, 2, 0.0, 2)]
    lp, dv, dp, dn = ctx.logpdf_grad(X, terms, 0.1, v)
    assert lp == ctx.logpdf(X, terms, 0.1, v)
    for k in (0, 1):
        h = 1e-4 * terms[k][2]
        tp = list(terms)
        tm = list(terms)
        tp[k] = (terms[k][0], terms[k][1], terms[k][2] + h, terms[k][3])
        tm[k] = (terms[k][0], terms[k][1], terms[k][2] - h, terms[k][3])
        fd = (ctx.logpdf(X, tp, 0.1, v) - ctx.logpdf(X, tm, 0.1, v)) / (2 * h)
        assert abs(dp[k] - fd) <= 1e-5 * abs(fd) + 1e-8 * abs(lp) / h, (k, dp[k], fd)
    h = 1e-5
    fdn = (ctx.logpdf(X, terms, 0.1 + h, v) - ctx.logpdf(X, terms, 0.1 - h, v)) / (2 * h)
    assert abs(dn - fdn) <= 1e-5 * abs(fdn) + 1e-8 * abs(lp) / h
    # d/dv along a random direction: (lp(v + h u) - lp(v - h u)) / 2h = dv . u
    u = rng.normal(size=N)
    h = 1e-4
    fdv = (ctx.logpdf(X, terms, 0.1, v + h * u) - ctx.logpdf(X, terms, 0.1, v - h * u)) / (2 * h)
    assert abs(float(dv @ u) - fdv) <= 1e-5 * abs(fdv) + 1e-8 * abs(lp) / h


def test_mcmc_model_against_oracle(ctx):
    rng = np.random.default_rng(9)
    N = 200
    tab = {"y": rng.normal(size=N), "x": rng.uniform(-5, 5, N), "t": rng.uniform(0, 10, N)}
    m = M.MCMCModel("y ~| SqExp(:x) + OU(:t; l=3) + Linear(:x)", tab, ["x"], ctx=ctx)
    fx = rng.normal(size=N)
    ell = 2.5
    lp, dell, dfx = m.logdensity_and_gradient(ell, fx)
    terms = m.terms(ell)
    rlp, rdv, rdp, _ = R.logpdf_grad(m.X, terms, 0.1, fx)
    r = tab["y"] - fx
    ref = -math.log(20.0) + rlp + float(np.sum(-(R.LOG2PI + r * r) / 2))
    assert abs(lp - ref) <= TOL * abs(ref)
    assert abs(dell - (rdp[0] + rdp[2])) <= TOL * (abs(rdp[0]) + abs(rdp[2]))
    assert np.max(np.abs(dfx - (rdv + r))) <= TOL * np.max(np.abs(rdv + r))
    assert abs(m.logdensity(ell, fx) - lp) <= 1e-12 * abs(lp)


def test_after_dirty_workspace(ctx):
    # the workspace keeps whatever earlier evaluations (other N, other layout) left in it;
    # the gradient must not read any of it
    rng = np.random.default_rng(21)
    big = 2100
    Xb = rng.uniform(0, 10, (big, 1))
    ctx.logpdf(Xb, [(SQEXP, 0, 0.7, 0)], 0.1, rng.normal(size=big))
    ctx.logpdf_grad(Xb, [(OU, 0, 0.9, 0)], 0.1, rng.normal(size=big))
    for N in (513, 1029, 300, 1700):
        X = np.column_stack([rng.uniform(0, 10, N), rng.normal(size=N)])
        v = rng.normal(size=N)
        terms = [(SQEXP, 0, 1.2, 0), (LINEAR, 1, 0.3, 1)]
        got = ctx.logpdf_grad(X, terms, 0.1, v)
        check_grad(got, R.logpdf_grad(X, terms, 0.1, v), *R.logpdf_grad_scale(X, terms, 0.1, v))
