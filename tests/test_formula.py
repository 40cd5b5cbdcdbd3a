"""Host-side mirror of the reference's formula/kernel API (no GPU needed).

Mirrors the reference's own inline tests (src/interface.jl:68-87, "Formula Parsing") and
pins the lowering quirks documented in SURVEY.md Q1-Q4, Q12.
"""
import numpy as np
import pytest

from gaplac_amd import formula as F
from gaplac_amd import kernels as K
from gaplac_amd._native import CAT, LINEAR, NOISE, OU, SQEXP
from gaplac_amd.abstractgps import FiniteGP, design_matrix, make_gp


# --- src/interface.jl:69-87 -------------------------------------------------------
def test_formula_parsing_reference_testset():
    spec1 = F.gp_spec("y ~| SqExp(:t)")
    assert isinstance(F.likelihood(spec1), F.Gaussian)
    assert F.response(spec1) == "y"
    assert isinstance(F.formula(spec1), F.GPCompnent)
    assert isinstance(F.formula(spec1), F.SqExp)

    spec2 = F.gp_spec("bug ~| SqExp(:t) + Linear(:x)")
    assert isinstance(F.likelihood(spec2), F.Gaussian)
    assert F.response(spec2) == "bug"
    assert isinstance(F.formula(spec2), F.GPOperation)

    spec3 = F.gp_spec("bug ~| SqExp(:t) * Cat(:g) + Linear(:x)")
    assert isinstance(F.likelihood(spec3), F.Gaussian)
    assert F.response(spec3) == "bug"
    assert isinstance(F.formula(spec3), F.GPOperation)


def test_explicit_empty_likelihood_and_kwarg_forms():
    s = F.gp_spec("y :~| SqExp(:x; l=1)")
    assert F.response(s) == "y" and isinstance(F.likelihood(s), F.Gaussian)
    assert F.formula(s) == F.SqExp("x", 1)
    # README.md:101 uses a comma before the keyword: Julia passes l as a keyword there too
    assert F.formula(F.gp_spec("y ~| SqExp(:x, l=2)")) == F.SqExp("x", 2)
    assert F.formula(F.gp_spec("y ~| Linear(:x; c=0.5)")) == F.Linear("x", 0.5)


def test_invalid_specs():
    with pytest.raises(F.ArgumentError):
        F.gp_spec("y | SqExp(:x)")
    with pytest.raises(F.ArgumentError):
        F.gp_spec("y ~ SqExp(:x)")
    with pytest.raises(F.UndefVarError):
        F.gp_spec("y ~| Periodic(:x)")
    # the docstring's positional lengthscale has no constructor method
    with pytest.raises(F.MethodError):
        F.gp_spec("y ~| SqExp(:x, 1.5)")


def test_varnames_one_per_term_left_to_right():
    f = F.formula(F.gp_spec("y ~| SqExp(:t) + OU(:t; l=3) + Cat(:subject)"))
    assert F.varnames(f) == ["t", "t", "subject"]


# --- lowering (src/abstractgp_translations.jl:45-71) -------------------------------
def test_single_term_has_no_select():
    k, v = K.kernel(F.formula(F.gp_spec("y ~| SqExp(:x; l=2)")))
    assert isinstance(k, K.TransformedKernel) and isinstance(k.transform, K.ScaleTransform)
    assert K.lower(k) == [(SQEXP, 0, 2.0, 0)] and v == ["x"]
    k, _ = K.kernel(F.formula(F.gp_spec("y ~| OU(:x)")))
    assert k == K.ExponentialKernel()  # l == 1: no ScaleTransform (makekernel :9)


def test_sum_lowering_positions_and_params():
    f = F.formula(F.gp_spec("y ~| SqExp(:t; l=1.5) + OU(:t; l=3) + Linear(:x; c=2) + Cat(:g)"))
    k, v = K.kernel(f)
    assert isinstance(k, K.KernelSum) and len(k.kernels) == 4
    assert K.lower(k) == [(SQEXP, 0, 1.5, 0), (OU, 1, 3.0, 1), (LINEAR, 2, 2.0, 2), (CAT, 3, 0.0, 3)]
    assert v == ["t", "t", "x", "g"]


def test_q1_toplevel_product_becomes_sum_and_nested_product_errors():
    k, v = K.kernel(F.formula(F.gp_spec("y ~| SqExp(:a) * Cat(:b)")))
    assert K.lower(k) == [(SQEXP, 0, 1.0, 0), (CAT, 1, 0.0, 1)]  # summed, as the reference
    with pytest.raises(RuntimeError):
        K.kernel(F.formula(F.gp_spec("y ~| SqExp(:a) * Cat(:b) + Linear(:c)")))
    # extension: true products
    d, v = K.lower_formula(F.formula(F.gp_spec("y ~| SqExp(:a) * Cat(:b) + Linear(:c)")), products=True)
    assert d == [(SQEXP, 0, 1.0, 0), (CAT, 1, 0.0, 0), (LINEAR, 2, 0.0, 1)]


def test_q4_cat_hyperparameter_is_method_error_and_q6_shared_l():
    f = F.formula(F.gp_spec("y ~| SqExp(:x; l=1.5) + OU(:t; l=2)"))
    d, _ = K.lower_formula(f, {"x": 4.0})  # mcmc.jl:33 infers l for :x only
    assert d == [(SQEXP, 0, 4.0, 0), (OU, 1, 2.0, 1)]
    d, _ = K.lower_formula(F.formula(F.gp_spec("y ~| Linear(:x)")), {"x": 0.25})
    assert d == [(LINEAR, 0, 0.25, 0)]  # Linear's "hyperparameter" is the intercept
    with pytest.raises(F.MethodError):
        K.kernel(F.formula(F.gp_spec("y ~| Cat(:g) + SqExp(:x)")), {"g": 2.0})


def test_noise_extension_and_make_gp_check():
    gp, v = make_gp(F.gp_spec("y ~| SqExp(:t) + Noise"))
    assert v == ["t"]
    assert K.lower(gp.kernel) == [(SQEXP, 0, 1.0, 0), (NOISE, -1, 1.0, 1)]
    gp, _ = make_gp(F.gp_spec("y ~| Cat(:g) + Noise(0.3)"))
    assert K.lower(gp.kernel)[-1] == (NOISE, -1, 0.3, 1)


def test_linear_negative_intercept_rejected():
    with pytest.raises(F.ArgumentError):
        K.lower_formula(F.formula(F.gp_spec("y ~| Linear(:x; c=-1)")))


def test_finitegp_design_matrix_rowvecs():
    table = {"t": np.arange(5.0), "g": np.array([1, 1, 2, 2, 3.0]), "y": np.zeros(5)}
    gp, v = make_gp(F.gp_spec("y ~| SqExp(:t) + Cat(:g)"))
    X = design_matrix(table, v)
    fx = FiniteGP(gp, X, 0.1)
    assert fx.x.shape == (5, 2) and fx.x.flags.f_contiguous and fx.noise == 0.1
    assert fx.terms == [(SQEXP, 0, 1.0, 0), (CAT, 1, 0.0, 1)]
    fx2 = FiniteGP(gp, X.T, 0.1, obsdim=2)
    assert np.array_equal(fx2.x, fx.x)
