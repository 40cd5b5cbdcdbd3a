"""The backend switch is read at call time.

The Julia glue defines its overloads unconditionally and consults a flag that __init__
sets from GAPLAC_HIP at every package load (not at precompile time). The Python twin
reads GAPLAC_HIP at every call: flipping it after import must change what the next call
does. CPU only: with the switch on, the call reaches the backend (which on a machine
without a GPU fails with its own error, not BackendDisabled)."""
import numpy as np
import pytest

from gaplac_amd import abstractgps as AG
from gaplac_amd import backend
from gaplac_amd import formula as F


def _fx():
    gp, _ = AG.make_gp(F.gp_spec("y ~| SqExp(:x; l=1.5)"))
    return AG.FiniteGP(gp, np.linspace(0, 1, 8)[:, None], 0.1)


def test_switch_is_read_at_call_time(monkeypatch):
    fx = _fx()
    y = np.zeros(8)
    monkeypatch.setenv("GAPLAC_HIP", "0")  # after import
    with pytest.raises(AG.BackendDisabled):
        AG.logpdf(fx, y)
    with pytest.raises(AG.BackendDisabled):
        AG.logpdf_and_gradient(fx, y)
    with pytest.raises(AG.BackendDisabled):
        AG.rand(fx, z=np.zeros(8))
    with pytest.raises(AG.BackendDisabled):
        AG.posterior(fx, y).mean_and_var(np.zeros((2, 1)))
    monkeypatch.setenv("GAPLAC_HIP", "1")
    assert AG.hip_enabled()
    sentinel = RuntimeError("backend reached")

    def fake_ctx():
        raise sentinel

    monkeypatch.setattr(backend, "default_context", fake_ctx)
    with pytest.raises(RuntimeError) as ei:
        AG.logpdf(fx, y)
    assert ei.value is sentinel
    monkeypatch.delenv("GAPLAC_HIP")
    assert AG.hip_enabled()  # default on in the twin
