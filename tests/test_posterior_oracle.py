"""Posterior mean / variance and rand restatements (oracle.restatement), pinned to
scikit-learn's independent GaussianProcessRegressor.predict (latent mean and std with the
observation variance as `alpha`) and to numpy's Cholesky. No GPU needed."""
import numpy as np
import pytest
from sklearn.gaussian_process import GaussianProcessRegressor
from sklearn.gaussian_process.kernels import RBF, Matern

from gaplac_amd._native import CAT, LINEAR, NOISE, OU, SQEXP
from oracle import restatement as R


@pytest.mark.parametrize("kind,l", [(SQEXP, 1.5), (SQEXP, 0.4), (OU, 2.0)])
def test_posterior_matches_sklearn(kind, l):
    rng = np.random.default_rng(3)
    N, M = 120, 37
    X = rng.uniform(-5, 5, (N, 1))
    Xs = np.vstack([rng.uniform(-6, 6, (M - 2, 1)), X[:2]])  # two test points on training inputs
    y = rng.normal(size=N)
    k = RBF(length_scale=l) if kind == SQEXP else Matern(length_scale=l, nu=0.5)
    gpr = GaussianProcessRegressor(kernel=k, alpha=0.1, optimizer=None, normalize_y=False).fit(X, y)
    m_ref, sd_ref = gpr.predict(Xs, return_std=True)
    m, v = R.posterior_mean_var(X, [(kind, 0, l, 0)], 0.1, y, Xs)
    assert np.max(np.abs(m - m_ref)) <= 1e-10 * max(1.0, np.max(np.abs(m_ref)))
    assert np.max(np.abs(np.sqrt(np.maximum(v, 0)) - sd_ref)) <= 1e-7


def test_posterior_sum_kernel_matches_sklearn():
    rng = np.random.default_rng(4)
    N, M = 90, 25
    x = rng.uniform(0, 10, N)
    X = np.column_stack([x, x])
    xs = rng.uniform(0, 10, M)
    Xs = np.column_stack([xs, xs])
    y = rng.normal(size=N)
    gpr = GaussianProcessRegressor(kernel=RBF(1.3) + Matern(3.0, nu=0.5), alpha=0.1, optimizer=None).fit(x[:, None], y)
    m_ref, sd_ref = gpr.predict(xs[:, None], return_std=True)
    m, v = R.posterior_mean_var(X, [(SQEXP, 0, 1.3, 0), (OU, 1, 3.0, 1)], 0.1, y, Xs)
    assert np.max(np.abs(m - m_ref)) <= 1e-10 * max(1.0, np.max(np.abs(m_ref)))
    assert np.max(np.abs(np.sqrt(np.maximum(v, 0)) - sd_ref)) <= 1e-7


def test_posterior_at_training_inputs_identities():
    # mean(X) = K alpha = y - noise * alpha; kernel_diag covers Linear / Cat / Noise terms
    rng = np.random.default_rng(5)
    N = 80
    X = np.column_stack([rng.uniform(0, 5, N), rng.normal(size=N), rng.integers(0, 7, N).astype(float)])
    y = rng.normal(size=N)
    terms = [(SQEXP, 0, 1.1, 0), (LINEAR, 1, 0.5, 1), (CAT, 2, 0.0, 2)]
    m, v = R.posterior_mean_var(X, terms, 0.1, y, X)
    _, dv, _, _ = R.logpdf_grad(X, terms, 0.1, y)
    assert np.allclose(m, y + 0.1 * dv, rtol=0, atol=1e-10)
    assert np.all(v > 0) and np.all(v <= R.kernel_diag(X, terms) + 1e-12)


def test_rand_is_cholesky_times_z():
    rng = np.random.default_rng(6)
    N = 150
    X = rng.uniform(-3, 3, (N, 1))
    terms = [(SQEXP, 0, 0.8, 0), (NOISE, -1, 0.05, 1)]
    z = rng.normal(size=N)
    s = R.rand_from(X, terms, 0.1, z)
    L = np.linalg.cholesky(R.gram(X, terms, 0.1))
    assert np.max(np.abs(s - L @ z)) <= 1e-12 * np.max(np.abs(s))
