"""CPU restatement of GaPLAC's log-marginal-likelihood path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline — never as the product path.

PARITY STATUS: **parity unpinned** by the reference. The reference (Julia 1.8.5 +
KernelFunctions 0.10.38 + AbstractGPs 0.5.12 + OpenBLAS 0.3.20) cannot run in this
container or on the GPU box (no `julia` binary, no depot, no network),
and its own tests pin no numbers on this path (they cover formula parsing only,
/root/reference/src/interface.jl:68-100). This restatement follows the documented
definitions of the pinned packages and is cross-checked (tests/test_oracle.py) against
scikit-learn's independent GaussianProcessRegressor.log_marginal_likelihood (RBF and
Matern(nu=1/2) kernels) to ~1e-15 relative, and against a Distances.jl-style
(`|a|^2+|b|^2-2ab`, clamped) distance computation to <=1e-9 relative logpdf.

What it restates, with the reference lines it follows:
  * term kernels — src/gp_parts.jl:11-13 (CategoricalKernel: kappa(d) = d > 0 ? 0 : 1 on
    Euclidean), :21-47 (SqExp/Linear/OU/Cat structs), src/abstractgp_translations.jl:8-15
    (makekernel: SqExponentialKernel / ExponentialKernel with_lengthscale(l) =
    k ∘ ScaleTransform(1/l), LinearKernel(c), CategoricalKernel);
  * term combination — src/abstractgp_translations.jl:45-69 (each term applied to its own
    column through SelectTransform, terms summed: KernelSum = left fold);
  * covariance + likelihood — CLI/src/select.jl:43-50 and CLI/src/mcmc.jl:35
    (FiniteGP(GP(k), RowVecs(X), 0.1): C = K + 0.1 I, zero mean) and AbstractGPs'
    logpdf = -(N log 2pi + logdet(C) + ||U^-T v||^2) / 2 with U = cholesky(Symmetric(C)).U
    (LAPACK dpotrf('U'), here scipy's dpotrf) and U' \\ v (dtrtrs/dtrsv).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg
from scipy.linalg import lapack

SQEXP, OU, LINEAR, CAT, NOISE = 1, 2, 3, 4, 5
LOG2PI = 1.8378770664093453  # Julia's log2π as Float64


class PosDefException(Exception):
    """Mirror of LinearAlgebra.PosDefException(info)."""

    def __init__(self, info: int):
        super().__init__(f"PosDefException: matrix is not positive definite; Cholesky factorization failed (info={info})")
        self.info = info


def _pair(a: np.ndarray, kind: str, distances: str) -> np.ndarray:
    """Pairwise squared-euclidean ('sq') or euclidean ('eu') distance of a 1-D coordinate.

    distances='direct': (a_i - a_j)^2 — the mathematical definition.
    distances='gemm'  : max(a_i^2 + a_j^2 - 2 a_i a_j, 0) — the BLAS form Distances.jl
                        0.10.7 uses for pairwise(SqEuclidean/Euclidean, X; dims=1)
                        [unverified-in-container, SURVEY.md §2].
    """
    if distances == "direct":
        d = a[:, None] - a[None, :]
        d2 = d * d
    elif distances == "gemm":
        sa = a * a
        d2 = np.maximum(sa[:, None] + sa[None, :] - 2.0 * np.outer(a, a), 0.0)
        np.fill_diagonal(d2, 0.0)
    else:
        raise ValueError(distances)
    return d2 if kind == "sq" else np.sqrt(d2)


def term_matrix(X: np.ndarray, kind: int, col: int, param: float, distances: str = "direct") -> np.ndarray:
    """K_t for one term (KernelFunctions kernelmatrix of the term's kernel on its column)."""
    N = X.shape[0]
    if kind == NOISE:
        return param * np.eye(N)
    x = np.ascontiguousarray(X[:, col], dtype=np.float64)
    if kind == SQEXP:
        if not (param > 0) or not math.isfinite(param):
            raise ValueError("lengthscale must be > 0")
        s = 1.0 / param  # ScaleTransform(inv(l))
        d2 = _pair(s * x, "sq", distances)
        return np.exp(-d2 * 0.5)  # SqExponentialKernel: kappa(d2) = exp(-d2/2)
    if kind == OU:
        if not (param > 0) or not math.isfinite(param):
            raise ValueError("lengthscale must be > 0")
        s = 1.0 / param
        d = _pair(s * x, "eu", distances)
        return np.exp(-d)  # ExponentialKernel: kappa(d) = exp(-d)
    if kind == LINEAR:
        if not (param >= 0):
            raise ValueError("LinearKernel: c >= 0 required")
        return np.outer(x, x) + param  # kappa(xᵀy) = xᵀy + c
    if kind == CAT:
        if distances == "direct":
            return (x[:, None] == x[None, :]).astype(np.float64)
        d = _pair(x, "eu", distances)
        return np.where(d > 0, 0.0, 1.0)
    raise ValueError(f"unknown term kind {kind}")


def gram(X: np.ndarray, terms, noise: float = 0.0, distances: str = "direct") -> np.ndarray:
    """C = sum over groups of (product over the group's terms) + noise I.

    terms: sequence of (kind, col, param, group); groups contiguous, summed in order.
    """
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    N = X.shape[0]
    total = np.zeros((N, N))
    prod = None
    terms = list(terms)
    for t, (kind, col, param, group) in enumerate(terms):
        K = term_matrix(X, kind, col, param, distances)
        prod = K if prod is None else prod * K
        last = t == len(terms) - 1 or terms[t + 1][3] != group
        if last:
            total = total + prod
            prod = None
    if noise:
        total[np.diag_indices(N)] += noise
    return total


def logpdf_from_cov(C: np.ndarray, v: np.ndarray):
    """AbstractGPs logpdf for zero mean: returns (logpdf, logdet, quad).

    Raises PosDefException(info) like cholesky(check=true)."""
    N = C.shape[0]
    if N == 0:
        return -0.0, 0.0, 0.0
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=0)
    if info > 0:
        raise PosDefException(int(info))
    if info < 0:
        raise ValueError(f"dpotrf argument error {info}")
    z = scipy.linalg.solve_triangular(U, v, trans="T", lower=False, check_finite=False)
    dd = 0.0
    for u in np.diag(U):  # logdet(::Cholesky): sequential sum of log diag, then dd + dd
        dd += math.log(u)
    logdet = dd + dd
    quad = float(np.sum(z * z))
    lp = -((N * LOG2PI + logdet) + quad) / 2
    return float(lp), float(logdet), quad


def logpdf(X, terms, noise: float, v, distances: str = "direct"):
    """Whole path: (logpdf, logdet, quad)."""
    C = gram(X, terms, noise, distances)
    return logpdf_from_cov(C, np.asarray(v, dtype=np.float64))


def cholesky_lower(X, terms, noise: float):
    """L = U^T and z = U^-T v-ready factor for small parity checks."""
    C = gram(X, terms, noise)
    U, info = lapack.dpotrf(C, lower=0, clean=1)
    if info > 0:
        raise PosDefException(int(info))
    return U.T.copy()


# ---------------------------------------------------------------------------------------
# Gradient of the log-marginal-likelihood (what NUTS in
# CLI/src/mcmc.jl:31-41 differentiates through logpdf(FiniteGP, fx) with ForwardDiff).
#   d logp / d v      = -alpha,  alpha = C^-1 v
#   d logp / d theta  = 1/2 * sum_ij (alpha_i alpha_j - (C^-1)_ij) dC_ij/dtheta
# per term parameter theta (l of SqExp/OU, c of Linear, variance of a Noise term; Cat
# has none -> 0) and for the FiniteGP observation variance (dC/dnoise = I).
# Term derivatives of the KernelFunctions kernels built at
# src/abstractgp_translations.jl:8-15 (u = x_i/l - x_j/l, the ScaleTransform(1/l) form):
#   SqExp  k = exp(-u^2/2)  dk/dl = k u^2 / l
#   OU     k = exp(-|u|)    dk/dl = k |u| / l
#   Linear k = x_i x_j + c  dk/dc = 1
# A term inside a product group (extension) is multiplied by the group's other terms.
# ---------------------------------------------------------------------------------------
def term_derivative(X: np.ndarray, kind: int, col: int, param: float) -> np.ndarray:
    """dK_t/dparam_t for one term (zeros for Cat)."""
    N = X.shape[0]
    if kind == NOISE:
        return np.eye(N)
    if kind == CAT:
        return np.zeros((N, N))
    x = np.ascontiguousarray(X[:, col], dtype=np.float64)
    if kind == LINEAR:
        return np.ones((N, N))
    s = 1.0 / param
    sx = s * x
    u = sx[:, None] - sx[None, :]
    if kind == SQEXP:
        return np.exp(-(u * u) * 0.5) * (u * u) / param
    if kind == OU:
        a = np.abs(u)
        return np.exp(-a) * a / param
    raise ValueError(f"unknown term kind {kind}")


def logpdf_grad(X, terms, noise: float, v):
    """(logpdf, dv, dparam[T], dnoise) with the definitions above.

    Raises PosDefException(info) like logpdf."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    v = np.asarray(v, dtype=np.float64)
    terms = list(terms)
    N = X.shape[0]
    if N == 0:
        return -0.0, np.zeros(0), np.zeros(len(terms)), 0.0
    C = gram(X, terms, noise)
    lp, _, _ = logpdf_from_cov(C, v)
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=0)
    alpha = scipy.linalg.cho_solve((U, False), v, check_finite=False)
    Cinv = scipy.linalg.cho_solve((U, False), np.eye(N), check_finite=False)
    W = np.outer(alpha, alpha) - Cinv
    dparam = np.zeros(len(terms))
    for t, (kind, col, param, group) in enumerate(terms):
        dK = term_derivative(X, kind, col, param)
        for s, (k2, c2, p2, g2) in enumerate(terms):
            if s != t and g2 == group:
                dK = dK * term_matrix(X, k2, c2, p2)
        dparam[t] = 0.5 * float(np.sum(W * dK))
    dnoise = 0.5 * float(np.trace(W))
    return float(lp), -alpha, dparam, dnoise


def logpdf_grad_scale(X, terms, noise: float, v):
    """Per-parameter magnitude 1/2 sum_ij |alpha_i alpha_j - Cinv_ij| |dC_ij| (and the same
    for the observation variance): the size of the terms the gradient sums, used to state
    the parity tolerance of a gradient entry that cancels to near zero."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    terms = list(terms)
    N = X.shape[0]
    C = gram(X, terms, noise)
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=0)
    if info:
        raise PosDefException(int(info))
    alpha = scipy.linalg.cho_solve((U, False), np.asarray(v, dtype=np.float64), check_finite=False)
    Cinv = scipy.linalg.cho_solve((U, False), np.eye(N), check_finite=False)
    A = np.abs(np.outer(alpha, alpha)) + np.abs(Cinv)
    out = np.zeros(len(terms))
    for t, (kind, col, param, group) in enumerate(terms):
        dK = term_derivative(X, kind, col, param)
        for s2, (k2, c2, p2, g2) in enumerate(terms):
            if s2 != t and g2 == group:
                dK = dK * term_matrix(X, k2, c2, p2)
        out[t] = 0.5 * float(np.sum(A * np.abs(dK)))
    return out, 0.5 * float(np.trace(A))


def logpdf_grad_potri(X, terms, noise: float, v):
    """Same result as logpdf_grad with C^{-1} from LAPACK dpotri on the dpotrf factor (what a
    CPU port of the gradient would call; used as bench.py's timed CPU baseline for the
    gradient). Returns (logpdf, dv, dparam, dnoise)."""
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    v = np.asarray(v, dtype=np.float64)
    terms = list(terms)
    C = gram(X, terms, noise)
    lp, _, _ = logpdf_from_cov(C, v)
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=1)
    del C
    alpha = scipy.linalg.cho_solve((U, False), v, check_finite=False)
    Cinv, info = lapack.dpotri(U, lower=0, overwrite_c=1)
    del U
    Cinv = np.triu(Cinv) + np.triu(Cinv, 1).T
    W = np.outer(alpha, alpha)
    W -= Cinv
    del Cinv
    dparam = np.zeros(len(terms))
    for t, (kind, col, param, group) in enumerate(terms):
        dK = term_derivative(X, kind, col, param)
        for s2, (k2, c2, p2, g2) in enumerate(terms):
            if s2 != t and g2 == group:
                dK *= term_matrix(X, k2, c2, p2)
        dparam[t] = 0.5 * float(np.vdot(W, dK))
        del dK
    return float(lp), -alpha, dparam, 0.5 * float(np.trace(W))


# ---------------------------------------------------------------------------------------
# Posterior mean / variance and rand (rank 3), AbstractGPs 0.5.12:
#   posterior(fx, y): C = cov(fx) (K + noise I), alpha = C^-1 (y - 0)
#   mean_and_var(post, xs): m = K(xs, X) alpha,
#                           v = kernelmatrix_diag(k, xs) - colsum((U' \ K(X, xs)).^2)
#     (diag_Xt_invA_X(C::Cholesky, X) = sum(abs2, C.U' \ X; dims=1)); reached from
#     src/plotting.jl:8-12 and CLI/src/select.jl:51-52.
#   rand(rng, fx) = mean(fx) + cholesky(C).U' * randn(rng, N), CLI/src/sample.jl:25.
# The index-noise extension couples a point with itself only: 0 across point sets, its
# variance on kernelmatrix_diag.
# ---------------------------------------------------------------------------------------
def cross_term_matrix(Xa: np.ndarray, Xb: np.ndarray, kind: int, col: int, param: float) -> np.ndarray:
    """K_t(Xa rows, Xb rows) for one term (len(Xa) x len(Xb))."""
    if kind == NOISE:
        return np.zeros((Xa.shape[0], Xb.shape[0]))
    a = np.ascontiguousarray(Xa[:, col], dtype=np.float64)
    b = np.ascontiguousarray(Xb[:, col], dtype=np.float64)
    if kind in (SQEXP, OU):
        s = 1.0 / param
        d = (s * a)[:, None] - (s * b)[None, :]
        return np.exp(-(d * d) * 0.5) if kind == SQEXP else np.exp(-np.abs(d))
    if kind == LINEAR:
        return np.outer(a, b) + param
    if kind == CAT:
        return (a[:, None] == b[None, :]).astype(np.float64)
    raise ValueError(f"unknown term kind {kind}")


def cross_gram(Xa, Xb, terms) -> np.ndarray:
    total = np.zeros((Xa.shape[0], Xb.shape[0]))
    prod = None
    terms = list(terms)
    for t, (kind, col, param, group) in enumerate(terms):
        K = cross_term_matrix(Xa, Xb, kind, col, param)
        prod = K if prod is None else prod * K
        if t == len(terms) - 1 or terms[t + 1][3] != group:
            total = total + prod
            prod = None
    return total


def kernel_diag(Xs, terms) -> np.ndarray:
    """kernelmatrix_diag(k, xs) (no observation noise)."""
    M = Xs.shape[0]
    total = np.zeros(M)
    prod = None
    terms = list(terms)
    for t, (kind, col, param, group) in enumerate(terms):
        if kind == NOISE:
            K = np.full(M, float(param))
        elif kind == LINEAR:
            x = Xs[:, col]
            K = x * x + param
        else:
            K = np.ones(M)
        prod = K if prod is None else prod * K
        if t == len(terms) - 1 or terms[t + 1][3] != group:
            total = total + prod
            prod = None
    return total


def posterior_mean_var(X, terms, noise: float, y, Xs):
    X = np.asarray(X, dtype=np.float64)
    X = X[:, None] if X.ndim == 1 else X
    Xs = np.asarray(Xs, dtype=np.float64)
    Xs = Xs[:, None] if Xs.ndim == 1 else Xs
    terms = list(terms)
    C = gram(X, terms, noise)
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=0)
    if info > 0:
        raise PosDefException(int(info))
    alpha = scipy.linalg.cho_solve((U, False), np.asarray(y, dtype=np.float64), check_finite=False)
    Kxs = cross_gram(X, Xs, terms)  # N x M
    mean = Kxs.T @ alpha
    V = scipy.linalg.solve_triangular(U, Kxs, trans="T", lower=False, check_finite=False)
    var = kernel_diag(Xs, terms) - np.sum(V * V, axis=0)
    return mean, var


def rand_from(X, terms, noise: float, z):
    """cholesky(C).U' * z for a given standard-normal vector z (zero mean)."""
    C = gram(X, terms, noise)
    U, info = lapack.dpotrf(C, lower=0, clean=1, overwrite_a=0)
    if info > 0:
        raise PosDefException(int(info))
    return U.T @ np.asarray(z, dtype=np.float64)
