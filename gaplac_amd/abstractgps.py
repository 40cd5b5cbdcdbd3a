"""AbstractGPs-shaped front end over the HIP backend (the drop-in boundary).

In the reference the hot path is the generic function
`Distributions.logpdf(::AbstractGPs.FiniteGP, ::AbstractVector)` (AbstractGPs 0.5.12),
reached from CLI/src/mcmc.jl:35 (`fx ~ FiniteGP(GP(k), RowVecs(X), 0.1)`) and
CLI/src/select.jl:43-50 (`logpdf(FiniteGP(gp, x, 0.1, obsdim=1), y)`). This module
mirrors that surface: GP(kernel), FiniteGP(gp, X, noise), logpdf(fx, v) — and routes the
evaluation through libgaplac_hip.so. There is no CPU fallback.

The switch: the Julia glue gates its overloads on a flag that
__init__ sets from GAPLAC_HIP at every package load; here the same variable is read at
EVERY call (hip_enabled). Off, the Julia host falls through to AbstractGPs' own method;
this twin has no such method (no CPU path in the product), so it raises BackendDisabled.
Default on here, since nothing else could answer.
"""
from __future__ import annotations

import os

import numpy as np

from . import backend
from . import formula as F
from . import kernels as K


class BackendDisabled(RuntimeError):
    """GAPLAC_HIP=0: the HIP backend is switched off (the Julia host would use AbstractGPs)."""


def hip_enabled() -> bool:
    """GAPLAC_HIP, read now (not at import): "0" turns the backend off."""
    return os.environ.get("GAPLAC_HIP", "1") != "0"


def _gate():
    if not hip_enabled():
        raise BackendDisabled("GAPLAC_HIP=0: HIP backend disabled; the Julia host falls back to AbstractGPs")


class GP:
    """Zero-mean GP with a kernel from GaPLAC.kernel (AbstractGPs.GP(k))."""

    def __init__(self, kern):
        self.kernel = kern

    def __call__(self, x, noise=0.0, obsdim=1):
        return FiniteGP(self, x, noise, obsdim=obsdim)


class FiniteGP:
    """AbstractGPs.FiniteGP(f, x, Σy): f at the rows of x (RowVecs / obsdim=1) with
    i.i.d. observation noise Σy = Diagonal(Fill(noise, N))."""

    def __init__(self, f: GP, x, noise=0.0, obsdim=1):
        X = np.asarray(x, dtype=np.float64)
        if X.ndim == 1:
            X = X[:, None]
        if obsdim == 2:
            X = X.T
        elif obsdim != 1:
            raise F.ArgumentError("obsdim must be 1 or 2")
        self.f = f
        self.x = np.asfortranarray(X)
        self.noise = float(noise)
        self.terms = K.lower(f.kernel)

    def __len__(self):
        return self.x.shape[0]


def logpdf(fx: FiniteGP, y, ctx: backend.Context | None = None, full: bool = False):
    """-(N log 2pi + logdet(C) + ||U^-T y||^2) / 2 on the GPU; raises
    backend.PosDefException(info) when C is not positive definite (cholesky check=true)."""
    _gate()
    ctx = ctx or backend.default_context()
    y = np.asarray(y, dtype=np.float64)
    if y.shape[0] != len(fx):
        raise F.ArgumentError("DimensionMismatch: length of y does not match the FiniteGP")
    return ctx.logpdf(fx.x, fx.terms, fx.noise, y, full=full)


def logpdf_and_gradient(fx: FiniteGP, y, ctx: backend.Context | None = None):
    """(logpdf, dlogpdf/dy, dlogpdf/dparam per lowered term, dlogpdf/dnoise) on the GPU:
    what ForwardDiff computes through AbstractGPs.logpdf in the reference's mcmc
    (CLI/src/mcmc.jl:31-41), as one analytic evaluation (gaplac_logpdf_grad)."""
    _gate()
    ctx = ctx or backend.default_context()
    y = np.asarray(y, dtype=np.float64)
    if y.shape[0] != len(fx):
        raise F.ArgumentError("DimensionMismatch: length of y does not match the FiniteGP")
    return ctx.logpdf_grad(fx.x, fx.terms, fx.noise, y)


class PosteriorGP:
    """AbstractGPs.posterior(fx, y): the GP conditioned on observations y at fx's inputs.
    Evaluation happens per query (mean_and_var at test inputs), one gaplac_posterior_mean_var
    call each."""

    def __init__(self, fx: FiniteGP, y, ctx: backend.Context | None = None):
        y = np.asarray(y, dtype=np.float64)
        if y.shape[0] != len(fx):
            raise F.ArgumentError("DimensionMismatch: length of y does not match the FiniteGP")
        self.prior = fx
        self.y = y
        self.ctx = ctx

    def _xs(self, x):
        X = np.asarray(x, dtype=np.float64)
        if X.ndim == 1:
            X = X[:, None]
        return X

    def mean_and_var(self, x):
        """AbstractGPs.mean_and_var(f::PosteriorGP, x): posterior mean and marginal variance
        (latent: no observation noise) at the rows of x."""
        _gate()
        ctx = self.ctx or backend.default_context()
        return ctx.posterior_mean_var(self.prior.x, self.prior.terms, self.prior.noise, self.y, self._xs(x))

    def mean(self, x):
        return self.mean_and_var(x)[0]

    def var(self, x):
        return self.mean_and_var(x)[1]


def posterior(fx: FiniteGP, y, ctx: backend.Context | None = None) -> PosteriorGP:
    """AbstractGPs.posterior(fx, y) (CLI/src/select.jl:51-52, src/plotting.jl:8)."""
    return PosteriorGP(fx, y, ctx)


def mean_and_var(f: PosteriorGP, x):
    """AbstractGPs.mean_and_var(pgp, xtest) (src/plotting.jl:12)."""
    return f.mean_and_var(x)


def rand(fx: FiniteGP, z=None, rng=None, ctx: backend.Context | None = None):
    """rand(rng, fx) = cholesky(C).U' * randn(rng, N) for the zero-mean FiniteGP
    (CLI/src/sample.jl:25). The standard-normal draws stay on the host: pass z, or an rng
    (numpy Generator) to draw it."""
    _gate()
    ctx = ctx or backend.default_context()
    if z is None:
        rng = rng if rng is not None else np.random.default_rng()
        z = rng.standard_normal(len(fx))
    return ctx.rand(fx.x, fx.terms, fx.noise, z)


def make_gp(spec: F.Spec, hyperparams=None):
    """src/interface.jl:36-41 — (GP(kern), vars), checking #vars == #kernels."""
    kern, vars_ = K.kernel(F.formula(spec), hyperparams)
    kernels = K._walk_kernel(kern)
    n_noise = sum(isinstance(k, K.IndexNoiseKernel) for k in kernels)
    if len(vars_) != len(kernels) - n_noise:
        raise RuntimeError("Something went wrong with equation parsing, number of variables should == number of kernels")
    return GP(kern), vars_


def design_matrix(table, vars_) -> np.ndarray:
    """`Matrix(df[!, vars])`: one column per formula term (duplicates allowed here; the
    reference's DataFrames selection rejects duplicates)."""
    cols = [np.asarray(table[v], dtype=np.float64) for v in vars_]
    if not cols:
        n = len(next(iter(table.values()))) if isinstance(table, dict) else len(table)
        return np.zeros((n, 0))
    return np.column_stack(cols)


def select_formulae(f1: str, f2: str, table, noise: float = 0.1, ctx: backend.Context | None = None):
    """CLI/src/select.jl:21-54 (`select --formulae`): logpdf of two formulas on the same
    data and the printed "Log2 Bayes" value, which is lp1 - lp2. Both models
    run through one batched call."""
    _gate()
    ctx = ctx or backend.default_context()
    specs = [F.gp_spec(f1), F.gp_spec(f2)]
    if F.response(specs[0]) != F.response(specs[1]):
        # the reference reads each response separately; keep the same data flow
        pass
    lps = []
    for s in specs:
        gp, vars_ = make_gp(s)
        X = design_matrix(table, vars_)
        y = np.asarray(table[F.response(s)], dtype=np.float64)
        lps.append(logpdf(FiniteGP(gp, X, noise), y, ctx=ctx))
    lp1, lp2 = lps
    return lp1 - lp2, lp1, lp2
