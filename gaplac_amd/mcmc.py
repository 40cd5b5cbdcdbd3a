"""The per-step log density of GaPLAC's `mcmc` model and its gradient — what NUTS calls.

The reference (CLI/src/mcmc.jl:12-41) builds a Turing model

    @model function inference_engine(Y, X, eq, inferable)
        ℓ ~ Uniform(0, 20)
        gp, = GaPLAC.kernel(eq; hyperparams=Dict(v => ℓ for v in inferable))
        fx ~ AbstractGPs.FiniteGP(GP(gp), RowVecs(X), 0.1)
        Y .~ Normal.(fx, 1)
    end

and samples it with NUTS(0.65), which evaluates the log joint and its gradient (ForwardDiff
Duals through the Gram matrix and the Cholesky) once per leapfrog step. This module is the
host-side mirror of that model: `logdensity_and_gradient(ℓ, fx)` returns the same log joint
(in the constrained space; the sampler's Bijectors transform of ℓ and its log-Jacobian stay
on the sampler's side) and its gradient, with the GP term evaluated in one
gaplac_logpdf_grad call on the GPU. Turing/NUTS itself is out of scope.

Semantics mirrored from the reference:
  * every formula term whose variable is in `infer` gets ℓ (SqExp/OU lengthscale, Linear
    intercept; a Cat term raises MethodError, src/abstractgp_translations.jl:13-15,33);
  * makekernel(::SqExp/::OU, l) drops the transform when l == 1 (:13-14), so at ℓ == 1
    exactly those terms do not depend on ℓ and ForwardDiff's dℓ gets no contribution from
    them; the gradient here reproduces that;
  * Y .~ Normal.(fx, 1): Σ_i -(log(2π) + (Y_i - fx_i)^2) / 2.
"""
from __future__ import annotations

import math

import numpy as np

from . import abstractgps as AG
from . import backend
from . import formula as F
from . import kernels as K
from ._native import LINEAR, NOISE, OU, SQEXP

LOG2PI = 1.8378770664093453
ELL_LO, ELL_HI = 0.0, 20.0  # ℓ ~ Uniform(0, 20)
NOISE_VAR = 0.1             # FiniteGP(GP(gp), RowVecs(X), 0.1)


class GradMemo:
    """The last gaplac_logpdf_grad result, keyed on the primal inputs.

    ForwardDiff evaluates the log density of a NUTS step in ceil((N+1)/chunk) chunked Dual
    passes whose primal values (ℓ and fx) are identical; only the seeded partials differ.
    The Julia glue answers every pass from ONE library call through
    this memo; this is its Python mirror. `calls` counts library calls."""

    def __init__(self):
        self.key = None
        self.X = None
        self.v = None
        self.val = None
        self.calls = 0

    def __call__(self, ctx, X, terms, noise: float, v):
        # keyed on the VALUES of X and v (copies kept and compared), never on a buffer
        # address: an X modified in place, or a new X in a reused buffer, misses the memo
        X = np.ascontiguousarray(X, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        key = (X.shape, tuple(map(tuple, terms)), float(noise))
        hit = (key == self.key and self.v is not None and np.array_equal(v, self.v)
               and np.array_equal(X, self.X))
        if not hit:
            self.val = ctx.logpdf_grad(X, terms, noise, v)
            self.key, self.X, self.v = key, X.copy(), v.copy()
            self.calls += 1
        return self.val


class MCMCModel:
    """inference_engine(y, x, formula, inferable) of CLI/src/mcmc.jl:31-39 on a table."""

    def __init__(self, formula: str, table, infer, ctx: backend.Context | None = None):
        spec = F.gp_spec(formula)                       # mcmc.jl:14
        self.formula = F.formula(spec)
        _, vars_ = AG.make_gp(spec)                     # mcmc.jl:19
        self.vars = list(vars_)
        self.infer = [str(v).lstrip(":") for v in infer]  # mcmc.jl:20 Symbol.(args["infer"])
        self.y = np.asarray(table[F.response(spec)], dtype=np.float64)  # mcmc.jl:25
        self.X = AG.design_matrix(table, vars_)         # mcmc.jl:26 Matrix(df[!, vars])
        self.ctx = ctx
        self.memo = GradMemo()

    @property
    def N(self) -> int:
        return self.X.shape[0]

    def terms(self, ell: float):
        """Lowered kernel of GaPLAC.kernel(eq; hyperparams=Dict(v => ℓ for v in inferable))."""
        hyper = {v: ell for v in self.infer}
        k, _ = K.kernel(self.formula, hyper)
        return K.lower(k)

    def tied(self, terms, ell: float):
        """Indices of the lowered terms whose value depends on ℓ."""
        out = []
        for t, (kind, col, _param, _group) in enumerate(terms):
            if kind == NOISE or self.vars[col] not in self.infer:
                continue
            if kind in (SQEXP, OU) and ell == 1:
                continue  # makekernel(::SqExp/::OU, 1): no ScaleTransform, no ℓ dependence
            if kind in (SQEXP, OU, LINEAR):
                out.append(t)
        return out

    def logdensity_and_gradient(self, ell: float, fx):
        """(log joint, d/dℓ, d/dfx). Outside ℓ's support: (-inf, nan, nan vector)."""
        fx = np.asarray(fx, dtype=np.float64)
        if fx.shape != (self.N,):
            raise F.ArgumentError("DimensionMismatch: fx must have one entry per observation")
        if not (ELL_LO <= ell <= ELL_HI):
            return -math.inf, math.nan, np.full(self.N, math.nan)
        terms = self.terms(ell)
        ctx = self.ctx or backend.default_context()
        lp_gp, dv, dparam, _ = self.memo(ctx, self.X, terms, NOISE_VAR, fx)
        r = self.y - fx
        lik = float(np.sum(-(LOG2PI + r * r) / 2))
        prior = -math.log(ELL_HI - ELL_LO)
        dell = float(sum(dparam[t] for t in self.tied(terms, ell)))
        return prior + lp_gp + lik, dell, dv + r

    def logdensity(self, ell: float, fx) -> float:
        """The log joint alone (one gaplac_logpdf call)."""
        fx = np.asarray(fx, dtype=np.float64)
        if not (ELL_LO <= ell <= ELL_HI):
            return -math.inf
        ctx = self.ctx or backend.default_context()
        lp_gp = ctx.logpdf(self.X, self.terms(ell), NOISE_VAR, fx)
        r = self.y - fx
        return -math.log(ELL_HI - ELL_LO) + lp_gp + float(np.sum(-(LOG2PI + r * r) / 2))

    def dual_pass(self, ell: float, fx, d_ell, d_fx):
        """One ForwardDiff chunk pass of the log joint: the value and its directional
        derivatives along the seeded partials (d_ell: (k,), d_fx: (N, k)) — what the Julia
        Dual method of INTEGRATION.md §1b returns, T(lp, ∂) with
        ∂ = Σ_i dv_i ∂fx_i + Σ_t dparam_t ∂θ_t (+ the Normal likelihood's (y - fx)·∂fx).
        Every pass at the same primal point reuses one library call (GradMemo)."""
        lp, dell, dfx = self.logdensity_and_gradient(ell, fx)
        d_ell = np.asarray(d_ell, dtype=np.float64)
        d_fx = np.asarray(d_fx, dtype=np.float64)
        return lp, dell * d_ell + dfx @ d_fx

    def gradient_chunked(self, ell: float, fx, chunk: int = 12):
        """ForwardDiff's chunked gradient over θ = (ℓ, fx) (Turing 0.21's default AD): one
        dual_pass per chunk of `chunk` seeded inputs. Returns (lp, dℓ, dfx, passes)."""
        fx = np.asarray(fx, dtype=np.float64)
        n = self.N + 1
        g = np.empty(n)
        lp = None
        passes = 0
        for c0 in range(0, n, chunk):
            k = min(chunk, n - c0)
            seeds = np.zeros((n, k))
            seeds[c0 + np.arange(k), np.arange(k)] = 1.0
            lp, part = self.dual_pass(ell, fx, seeds[0], seeds[1:])
            g[c0:c0 + k] = part
            passes += 1
        return lp, float(g[0]), g[1:], passes
