"""CPU restatement (oracle/) checks: independent cross-checks and the golden fixtures.

The reference itself cannot run here (Julia absent), so the oracle is "parity unpinned"
by the reference; these tests pin it against an independent implementation
(scikit-learn's GaussianProcessRegressor) and the Distances.jl distance formulation.
"""
import math

import numpy as np
import pytest

from oracle import restatement as R
from tests.golden_io import load_cases

CASES = load_cases()


def _sk_lml(x, y, kernel):
    from sklearn.gaussian_process import GaussianProcessRegressor
    gpr = GaussianProcessRegressor(kernel=kernel, alpha=0.1, optimizer=None, normalize_y=False)
    gpr.fit(x[:, None], y)
    return gpr.log_marginal_likelihood_value_


@pytest.mark.parametrize("l", [0.5, 1.0, 1.5, 3.0])
@pytest.mark.parametrize("N", [50, 400])
def test_sqexp_matches_sklearn(N, l):
    from sklearn.gaussian_process.kernels import RBF
    rng = np.random.default_rng(N)
    x = rng.uniform(-5, 5, N)
    y = rng.standard_normal(N)
    lp, _, _ = R.logpdf(x, [(R.SQEXP, 0, l, 0)], 0.1, y)
    ref = _sk_lml(x, y, RBF(length_scale=l))
    assert abs(lp - ref) <= 1e-12 * abs(ref)


@pytest.mark.parametrize("l", [0.7, 1.5])
def test_ou_matches_sklearn(l):
    from sklearn.gaussian_process.kernels import Matern
    rng = np.random.default_rng(7)
    x = rng.uniform(-5, 5, 300)
    y = rng.standard_normal(300)
    lp, _, _ = R.logpdf(x, [(R.OU, 0, l, 0)], 0.1, y)
    ref = _sk_lml(x, y, Matern(length_scale=l, nu=0.5))
    assert abs(lp - ref) <= 1e-12 * abs(ref)


def test_linear_and_cat_semantics():
    x = np.array([1.0, 2.0, 2.0, -3.0])
    K = R.term_matrix(x[:, None], R.LINEAR, 0, 0.5)
    assert np.array_equal(K, np.outer(x, x) + 0.5)
    K = R.term_matrix(x[:, None], R.CAT, 0, 0.0)
    assert K[1, 2] == 1.0 and K[0, 1] == 0.0 and np.all(np.diag(K) == 1.0)
    # Cat on the reference's PersonID-sized integers: the gemm distance form stays exact
    ids = np.array([10042055.0, 10042055.0, 72251940.0, 72251631.0])
    Kd = R.term_matrix(ids[:, None], R.CAT, 0, 0.0)
    Kg = R.term_matrix(ids[:, None], R.CAT, 0, 0.0, distances="gemm")
    assert np.array_equal(Kd, Kg)


def test_products_and_noise_extension():
    rng = np.random.default_rng(3)
    X = np.column_stack([rng.uniform(-2, 2, 30), rng.integers(0, 4, 30).astype(float)])
    C = R.gram(X, [(R.SQEXP, 0, 1.0, 0), (R.CAT, 1, 0.0, 0), (R.NOISE, -1, 0.5, 1)], 0.1)
    expect = R.term_matrix(X, R.SQEXP, 0, 1.0) * R.term_matrix(X, R.CAT, 1, 0.0) + 0.5 * np.eye(30) + 0.1 * np.eye(30)
    assert np.allclose(C, expect, rtol=0, atol=1e-15)


def test_posdef_info_known_answer():
    # Cat-only without noise: 0/1 arithmetic is exact, first repeated level -> zero pivot
    g = np.array([3.0, 1.0, 4.0, 1.0, 5.0])
    with pytest.raises(R.PosDefException) as ei:
        R.logpdf(g, [(R.CAT, 0, 0.0, 0)], 0.0, np.ones(5))
    assert ei.value.info == 4


def test_empty_is_zero():
    lp, ld, q = R.logpdf(np.zeros((0, 1)), [(R.SQEXP, 0, 1.0, 0)], 0.1, np.zeros(0))
    assert lp == 0.0 and ld == 0.0 and q == 0.0


def test_select_bayes_is_difference_of_logpdfs():
    # CLI/src/select.jl:54: log2(2^lp1 / 2^lp2) == lp1 - lp2; README.md:111-115 known answer
    lp1, lp2 = -31.53397005887427, -35.97395926954643
    assert round(lp1 - lp2, 2) == 4.44


@pytest.mark.parametrize("case", CASES, ids=[c["name"][:60] for c in CASES])
def test_golden_fixture_reproduces(case):
    """The committed fixtures are what the oracle computes (guards oracle drift)."""
    if case["info"]:
        with pytest.raises(R.PosDefException) as ei:
            R.logpdf(case["X"], case["terms"], case["noise"], case["v"])
        assert ei.value.info == case["info"]
        return
    lp, ld, q = R.logpdf(case["X"], case["terms"], case["noise"], case["v"])
    assert abs(lp - case["logpdf"]) <= 1e-12 * abs(case["logpdf"])
    assert abs(ld - case["logdet"]) <= 1e-12 * max(1.0, abs(case["logdet"]))
    assert abs(q - case["quad"]) <= 1e-12 * max(1.0, abs(case["quad"]))
    C = R.gram(case["X"], case["terms"], case["noise"])
    assert abs(C.sum() - case["gram_sum"]) <= 1e-12 * max(1.0, abs(case["gram_sum"]))


@pytest.mark.parametrize("case", [c for c in CASES if c.get("logpdf_gemm_distances")],
                         ids=lambda c: c["name"][:60])
def test_distance_formulation_within_tolerance(case):
    """Distances.jl's |a|^2+|b|^2-2ab form vs direct differences: far below the 1e-9 bar."""
    rel = abs(case["logpdf_gemm_distances"] - case["logpdf"]) / abs(case["logpdf"])
    assert rel < 1e-11
