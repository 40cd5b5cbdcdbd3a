"""The library's non-default paths that change only the order or grouping of the same
arithmetic, in fresh contexts, against the default path:

* GAPLAC_TAIL_SIM=0 / =1: the tail list in its built order / always simulated-ordered.
  Every tile still takes its column updates in order, so logpdf, logdet and quad are
  bitwise those of the default;
* GAPLAC_TAILK=0: the tail as per-column launches (the same per-column arithmetic as the
  persistent tail's update tasks only up to summation order: 1e-12 relative);
* GAPLAC_GRAD_FUSED=0: the gradient's -C^{-1} tiles stored, then contracted (the
  product-group path forced on a singleton formula): the gradient within 1e-10 relative
  of its scale, logpdf bitwise.
"""
import os

import numpy as np
import pytest

from gaplac_amd._native import CAT, NOISE, OU, SQEXP
from gaplac_amd.backend import Context
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu
TERMS = [(SQEXP, 0, 1.5, 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]


def inputs(N, seed=3):
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, max(1, N // 3), N).astype(float)])
    return X, rng.standard_normal(N)


def ctx_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def base():
    if not gpu_available():
        pytest.skip("no GPU")
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("N", [4096, 8192])
@pytest.mark.parametrize("sim", ["0", "1"])
def test_tail_order_bitwise(base, N, sim):
    X, v = inputs(N)
    ref = base.logpdf(X, TERMS, 0.1, v, full=True)
    with ctx_with({"GAPLAC_TAIL_SIM": sim}) as c:
        got = c.logpdf(X, TERMS, 0.1, v, full=True)
    assert got == ref, (got, ref)


def test_tail_launches(base):
    N = 8192
    X, v = inputs(N, seed=4)
    ref = base.logpdf(X, TERMS, 0.1, v, full=True)
    with ctx_with({"GAPLAC_TAILK": "0"}) as c:
        got = c.logpdf(X, TERMS, 0.1, v, full=True)
    assert abs(got[0] - ref[0]) <= 1e-12 * abs(ref[0]), (got, ref)


@pytest.mark.parametrize("N", [4096, 8192])
def test_grad_unfused(base, N):
    X, v = inputs(N, seed=5)
    lp, dv, dp, dn = base.logpdf_grad(X, TERMS, 0.1, v)
    with ctx_with({"GAPLAC_GRAD_FUSED": "0"}) as c:
        lp2, dv2, dp2, dn2 = c.logpdf_grad(X, TERMS, 0.1, v)
    assert lp2 == lp
    assert np.array_equal(dv2, dv)
    scale = np.abs(dp).max() + 1.0
    assert np.max(np.abs(np.asarray(dp2) - np.asarray(dp))) <= 1e-10 * scale, (dp2, dp)
    assert abs(dn2 - dn) <= 1e-10 * (abs(dn) + 1.0), (dn2, dn)


def test_split_bulk_profiling_stats(base):
    """Profiling mode 2 with the split bulk updates: the triangle launches
    (syrk_*) and every bulk-type launch of the super-panel phase (bulk_*, overlapping since
    the split) are event-timed; the union of their intervals is at most their summed time
    and at least the longest launch, and the evaluation is unchanged by the events."""
    N = 16384
    X, v = inputs(N, seed=6)
    ref = base.logpdf(X, TERMS, 0.1, v, full=True)
    base.reset_stats()
    base.set_profiling(2)
    got = base.logpdf(X, TERMS, 0.1, v, full=True)
    base.set_profiling(0)
    st = base.stats()
    base.reset_stats()
    assert got == ref
    assert st["syrk_launches"] > 0 and st["bulk_launches"] > st["syrk_launches"]
    assert st["bulk_flops"] > st["syrk_flops"] > 0
    assert 0 < st["bulk_union_ms"] < 40.0
    assert st["bulk_union_ms"] >= st["syrk_ms"] / st["syrk_launches"]
