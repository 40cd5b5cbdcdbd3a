"""The mcmc boundary's memo (gaplac_amd/mcmc.py GradMemo), on the CPU.

NUTS in CLI/src/mcmc.jl:31-41 differentiates the log joint with ForwardDiff, which
evaluates it in ceil((N+1)/chunk) chunked Dual passes at one primal point (ℓ, fx). The
binding must answer all of them from ONE gaplac_logpdf_grad call and rebuild each pass's
partials from the analytic gradient. Here the device is stood in for by the oracle's
analytic gradient (tests only), and the call count is asserted.
"""
import math

import numpy as np

from gaplac_amd import mcmc as M
from oracle import restatement as R


class _OracleGradCtx:
    """Stands in for backend.Context.logpdf_grad; counts calls."""

    def __init__(self):
        self.calls = 0

    def logpdf_grad(self, X, terms, noise, v):
        self.calls += 1
        return R.logpdf_grad(X, terms, noise, v)


def _model(N=150, seed=3):
    rng = np.random.default_rng(seed)
    tab = {"y": rng.normal(size=N), "x": rng.uniform(-5, 5, N), "t": rng.uniform(0, 10, N)}
    ctx = _OracleGradCtx()
    m = M.MCMCModel("y ~| SqExp(:x) + OU(:t; l=3) + Linear(:x)", tab, ["x"], ctx=ctx)
    return m, ctx, rng.normal(size=N), tab


def test_chunked_passes_make_one_library_call():
    m, ctx, fx, tab = _model()
    ell = 2.5
    lp, dell, dfx, passes = m.gradient_chunked(ell, fx, chunk=12)
    assert passes == math.ceil((m.N + 1) / 12) == 13
    assert ctx.calls == 1 and m.memo.calls == 1
    # the same gradient as one direct evaluation, and as the oracle's
    lp2, dell2, dfx2 = m.logdensity_and_gradient(ell, fx)
    assert ctx.calls == 1
    assert lp == lp2 and dell == dell2 and np.array_equal(dfx, dfx2)
    terms = m.terms(ell)
    rlp, rdv, rdp, _ = R.logpdf_grad(m.X, terms, 0.1, fx)
    r = tab["y"] - fx
    assert abs(dell - (rdp[0] + rdp[2])) <= 1e-12 * (abs(rdp[0]) + abs(rdp[2]))
    assert np.max(np.abs(dfx - (rdv + r))) <= 1e-12 * np.max(np.abs(rdv + r))


def test_new_primal_point_makes_a_new_call():
    m, ctx, fx, _ = _model()
    m.gradient_chunked(1.7, fx, chunk=8)
    m.gradient_chunked(1.7, fx, chunk=8)
    assert ctx.calls == 1
    m.gradient_chunked(1.8, fx, chunk=8)       # new ℓ
    assert ctx.calls == 2
    fx2 = fx.copy()
    fx2[5] += 1e-3                               # new fx
    m.gradient_chunked(1.8, fx2, chunk=8)
    assert ctx.calls == 3
    m.gradient_chunked(1.8, fx2.copy(), chunk=8)  # equal values, another array
    assert ctx.calls == 3


def test_dual_pass_partials_are_directional_derivatives():
    m, ctx, fx, _ = _model(N=40)
    ell = 0.9
    lp, dell, dfx = m.logdensity_and_gradient(ell, fx)
    rng = np.random.default_rng(1)
    d_ell, d_fx = rng.normal(size=3), rng.normal(size=(40, 3))
    lp2, part = m.dual_pass(ell, fx, d_ell, d_fx)
    assert lp2 == lp and ctx.calls == 1
    assert np.allclose(part, dell * d_ell + dfx @ d_fx, rtol=1e-14, atol=0)


def test_ell_equal_one_drops_the_tied_terms_like_forwarddiff():
    # makekernel(::SqExp, 1) has no ScaleTransform: ForwardDiff sees no ℓ in that term
    m, ctx, fx, _ = _model(N=60)
    _, dell, _, _ = m.gradient_chunked(1.0, fx, chunk=12)
    terms = m.terms(1.0)
    _, _, rdp, _ = R.logpdf_grad(m.X, terms, 0.1, fx)
    assert dell == rdp[2]  # only the Linear(:x) intercept depends on ℓ at ℓ == 1


def test_memo_keys_on_values_not_buffer_address():
    # keyed on X.ctypes.data, an X modified in place returned a stale gradient
    m, ctx, fx, tab = _model(N=60)
    terms = m.terms(2.0)
    X = m.X.copy()
    a = m.memo(ctx, X, terms, 0.1, fx)
    X[:, 0] *= 1.5  # same buffer, new values (a shift would leave a stationary kernel unchanged)
    b = m.memo(ctx, X, terms, 0.1, fx)
    assert ctx.calls == 2
    assert not np.array_equal(a[1], b[1])
    c = m.memo(ctx, X.copy(), terms, 0.1, fx)  # new buffer, same values: a hit
    assert ctx.calls == 2 and c is b
