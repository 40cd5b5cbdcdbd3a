"""Failure detection in the persistent tail ("Hand-offs"): every wait of
tail_kernel is bounded, and an expired wait must come back as GAPLAC_E_HIP, never as a
logpdf computed on stale tiles with rc = 0.

GAPLAC_TAIL_FAULT=k (a test-only switch read at context creation) skips the diagonal-block
task of tail column k: it neither factors nor publishes, so the TRSM staging waves behind it
(pipelined single evaluations) and the update / TRSM waits (batched select, whole-tile
TRSMs) expire. After the first expiry every later wait returns at once, so the launch
drains in ~0.2 s. A fresh context without the switch must then evaluate normally on the
same device.
"""
import numpy as np
import pytest

from gaplac_amd import _native
from gaplac_amd.backend import Context, GaplacError
from oracle import restatement as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    # the torch probe first, before this module loads the library (like the other GPU files)
    if not gpu_available():
        pytest.skip("no GPU")


TERMS = [(_native.SQEXP, 0, 1.5, 0)]


def _inputs(N, seed=11):
    rng = np.random.default_rng(seed)
    return rng.uniform(-5, 5, (N, 1)), rng.standard_normal(N)


@pytest.mark.parametrize("N,fault", [(1000, 3), (3000, 0), (3000, 20)])
def test_forced_tail_expiry_is_reported(monkeypatch, N, fault):
    X, v = _inputs(N)
    monkeypatch.setenv("GAPLAC_TAIL_FAULT", str(fault))
    with Context(0) as ctx:
        with pytest.raises(GaplacError) as ei:
            ctx.logpdf(X, TERMS, 0.1, v)
        assert ei.value.code == _native.E_HIP
        assert "wait expired" in str(ei.value)
    monkeypatch.delenv("GAPLAC_TAIL_FAULT")
    with Context(0) as ctx:
        lp = ctx.logpdf(X, TERMS, 0.1, v)
    ref = R.logpdf(X, TERMS, 0.1, v)[0]
    assert abs(lp - ref) <= 1e-12 * abs(ref)


def test_forced_tail_expiry_in_batched_select(monkeypatch):
    N = 1500
    X, v = _inputs(N, seed=12)
    models = [[(_native.SQEXP, 0, l, 0)] for l in (0.5, 1.0, 1.5, 2.0)]
    monkeypatch.setenv("GAPLAC_TAIL_FAULT", "5")
    with Context(0) as ctx:
        with pytest.raises(GaplacError) as ei:
            ctx.logpdf_batch(X, models, 0.1, v)
        assert ei.value.code == _native.E_HIP
    monkeypatch.delenv("GAPLAC_TAIL_FAULT")
    with Context(0) as ctx:
        out, info = ctx.logpdf_batch(X, models, 0.1, v)
    for m, terms in enumerate(models):
        ref = R.logpdf(X, terms, 0.1, v)[0]
        assert info[m] == 0 and abs(out[m] - ref) <= 1e-12 * abs(ref)


def test_release_frees_and_reallocates():
    X, v = _inputs(2000, seed=13)
    models = [[(_native.SQEXP, 0, l, 0)] for l in (0.7, 1.3, 2.1)]
    with Context(0) as ctx:
        a = ctx.logpdf(X, TERMS, 0.1, v)
        b, _ = ctx.logpdf_batch(X, models, 0.1, v)
        ctx.release()
        assert ctx.logpdf(X, TERMS, 0.1, v) == a
        b2, _ = ctx.logpdf_batch(X, models, 0.1, v)
        ctx.release()
    assert np.array_equal(b, b2)
