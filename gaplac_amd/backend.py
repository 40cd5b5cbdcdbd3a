"""Python handle on the HIP backend: a device context and the logpdf entry points.

This is the Python mirror of the `ccall` glue a GaPLAC maintainer would add in Julia
(INTEGRATION.md); numpy arrays stand in for Julia's GC-owned column-major buffers.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_double, c_int32, c_int64, c_void_p

import numpy as np

from . import _native
from ._native import Term, term_array


class GaplacError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gaplac error {code}: {msg}")
        self.code = code


class PosDefException(ArithmeticError):
    """Mirror of Julia's LinearAlgebra.PosDefException(info) (cholesky check=true)."""

    def __init__(self, info: int):
        super().__init__(f"PosDefException: matrix is not positive definite; Cholesky factorization failed (info={info})")
        self.info = info


class ArgumentError(ValueError):
    """Mirror of Julia's ArgumentError for invalid kernel parameters / arguments."""


def _colmajor(X: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    return np.asfortranarray(X)


class Context:
    """One device, one persistent workspace (gaplac_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = _native.load()
        h = c_void_p()
        rc = self.lib.gaplac_ctx_create(int(device), byref(h))
        if rc != 0:
            raise GaplacError(rc, f"gaplac_ctx_create(device={device}) failed")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self.lib.gaplac_ctx_destroy(self.h)
            self.h = None

    def release(self):
        """Free the large device workspaces (gaplac_ctx_release); the next call re-allocates."""
        self._check(self.lib.gaplac_ctx_release(self.h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ helpers
    def _check(self, rc: int):
        if rc == 0:
            return
        if rc > 0:
            raise PosDefException(rc)
        msg = self.lib.gaplac_last_error(self.h)
        msg = msg.decode() if msg else ""
        if rc in (_native.E_PARAM, _native.E_KIND, _native.E_COL, _native.E_ARG):
            raise ArgumentError(f"gaplac error {rc}: {msg}")
        raise GaplacError(rc, msg)

    # ------------------------------------------------------------------ entries
    def logpdf(self, X, terms, noise: float, v, full: bool = False):
        """logpdf of the zero-mean FiniteGP; full=True returns (logpdf, logdet, quad)."""
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        if v.shape[0] != N:
            raise ArgumentError(f"length of v ({v.shape[0]}) != N ({N})")
        terms = list(terms)  # one pass: a generator must not reach the library as T = 0
        ta = term_array(terms)
        lp, ld, q = c_double(), c_double(), c_double()
        rc = self.lib.gaplac_logpdf(
            self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta, float(noise),
            v.ctypes.data_as(c_void_p), byref(lp), byref(ld), byref(q),
        )
        self._check(rc)
        return (lp.value, ld.value, q.value) if full else lp.value

    def logpdf_device(self, N: int, D: int, dX_ptr: int, ldx: int, terms, noise: float, dv_ptr: int, full=False):
        terms = list(terms)
        ta = term_array(terms)
        lp, ld, q = c_double(), c_double(), c_double()
        rc = self.lib.gaplac_logpdf_device(
            self.h, N, D, c_void_p(dX_ptr), ldx, len(terms), ta, float(noise), c_void_p(dv_ptr),
            byref(lp), byref(ld), byref(q),
        )
        self._check(rc)
        return (lp.value, ld.value, q.value) if full else lp.value

    def logpdf_batch(self, X, models, noise: float, v):
        """models: list of term lists. Returns (logpdf array, info array)."""
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        offs = [0]
        flat = []
        models = [list(m) for m in models]
        for m in models:
            flat.extend(m)
            offs.append(len(flat))
        ta = term_array(flat)
        off_arr = (c_int32 * len(offs))(*offs)
        out = np.empty(len(models), dtype=np.float64)
        info = np.zeros(len(models), dtype=np.int64)
        rc = self.lib.gaplac_logpdf_batch(
            self.h, len(models), N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), off_arr, ta, float(noise),
            v.ctypes.data_as(c_void_p), out.ctypes.data_as(ctypes.POINTER(c_double)),
            info.ctypes.data_as(ctypes.POINTER(c_int64)),
        )
        self._check(rc)
        return out, info

    def logpdf_grad(self, X, terms, noise: float, v):
        """(logpdf, dv, dparam, dnoise): logpdf and its gradient with respect to v, to each
        term's parameter (l / c / variance; 0 for Cat) and to the observation variance
        (gaplac_logpdf_grad)."""
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        if v.shape[0] != N:
            raise ArgumentError(f"length of v ({v.shape[0]}) != N ({N})")
        terms = list(terms)
        ta = term_array(terms)
        lp, dn = c_double(), c_double()
        dv = np.empty(N, dtype=np.float64)
        dp = np.empty(max(1, len(terms)), dtype=np.float64)
        rc = self.lib.gaplac_logpdf_grad(
            self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta, float(noise),
            v.ctypes.data_as(c_void_p), byref(lp), dv.ctypes.data_as(c_void_p), dp.ctypes.data_as(c_void_p),
            byref(dn),
        )
        self._check(rc)
        return lp.value, dv, dp[: len(terms)].copy(), dn.value

    def logpdf_grad_device(self, N: int, D: int, dX_ptr: int, ldx: int, terms, noise: float, dv_ptr: int,
                           want_dv: bool = True):
        """Device-resident inputs; returns (logpdf, dv or None, dparam, dnoise)."""
        terms = list(terms)
        ta = term_array(terms)
        lp, dn = c_double(), c_double()
        dv = np.empty(N, dtype=np.float64) if want_dv else None
        dp = np.empty(max(1, len(terms)), dtype=np.float64)
        rc = self.lib.gaplac_logpdf_grad_device(
            self.h, N, D, c_void_p(dX_ptr), ldx, len(terms), ta, float(noise), c_void_p(dv_ptr), byref(lp),
            dv.ctypes.data_as(c_void_p) if want_dv else None, dp.ctypes.data_as(c_void_p), byref(dn),
        )
        self._check(rc)
        return lp.value, dv, dp[: len(terms)].copy(), dn.value

    def posterior_mean_var(self, X, terms, noise: float, y, Xs):
        """(mean, var) of the posterior of the zero-mean FiniteGP given y, at the rows of Xs
        (gaplac_posterior_mean_var)."""
        Xc = _colmajor(X)
        y = np.ascontiguousarray(y, dtype=np.float64)
        N, D = Xc.shape
        if y.shape[0] != N:
            raise ArgumentError(f"length of y ({y.shape[0]}) != N ({N})")
        Xsc = _colmajor(Xs)
        M = Xsc.shape[0]
        if Xsc.shape[1] != D:
            raise ArgumentError(f"test inputs have {Xsc.shape[1]} columns, training inputs {D}")
        terms = list(terms)
        ta = term_array(terms)
        mean = np.empty(M, dtype=np.float64)
        var = np.empty(M, dtype=np.float64)
        rc = self.lib.gaplac_posterior_mean_var(
            self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta, float(noise),
            y.ctypes.data_as(c_void_p), M, Xsc.ctypes.data_as(c_void_p), max(M, 1),
            mean.ctypes.data_as(c_void_p), var.ctypes.data_as(c_void_p),
        )
        self._check(rc)
        return mean, var

    def rand(self, X, terms, noise: float, z):
        """L z with C = K(X) + noise I = L L^T (gaplac_rand): one draw of the FiniteGP for the
        standard-normal vector z."""
        Xc = _colmajor(X)
        z = np.ascontiguousarray(z, dtype=np.float64)
        N, D = Xc.shape
        if z.shape[0] != N:
            raise ArgumentError(f"length of z ({z.shape[0]}) != N ({N})")
        terms = list(terms)
        ta = term_array(terms)
        out = np.empty(N, dtype=np.float64)
        rc = self.lib.gaplac_rand(self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta,
                                  float(noise), z.ctypes.data_as(c_void_p), out.ctypes.data_as(c_void_p))
        self._check(rc)
        return out

    def gram(self, X, terms, noise: float = 0.0) -> np.ndarray:
        Xc = _colmajor(X)
        N, D = Xc.shape
        out = np.empty((N, N), dtype=np.float64, order="F")
        terms = list(terms)
        ta = term_array(terms)
        rc = self.lib.gaplac_gram(self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta,
                                  float(noise), out.ctypes.data_as(c_void_p), max(N, 1))
        self._check(rc)
        return out

    def gram_time(self, X, terms, noise: float, v, reps: int = 5):
        """(best_ms, bytes): one plain-grid Gram launch into the workspace, timed with
        hipEvents (best of reps), and its algorithmic HBM bytes (bench.py extra.gram)."""
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        terms = list(terms)
        ta = term_array(terms)
        ms, nbytes = c_double(0.0), c_double(0.0)
        rc = self.lib.gaplac_gram_time(self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta,
                                       float(noise), v.ctypes.data_as(c_void_p), int(reps), byref(ms), byref(nbytes))
        self._check(rc)
        return ms.value, nbytes.value

    def factor(self, X, terms, noise: float, v):
        """(L, z): lower Cholesky factor of C and z = L^{-1} v."""
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        L = np.empty((N, N), dtype=np.float64, order="F")
        z = np.empty(N, dtype=np.float64)
        terms = list(terms)
        ta = term_array(terms)
        rc = self.lib.gaplac_factor(self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta,
                                    float(noise), v.ctypes.data_as(c_void_p), L.ctypes.data_as(c_void_p),
                                    max(N, 1), z.ctypes.data_as(c_void_p))
        self._check(rc)
        return L, z

    def set_profiling(self, mode):
        """0/False off, 1/True per-launch device timestamps, 2 hipEvents around the bulk
        trailing-update launches (production schedule)."""
        self.lib.gaplac_set_profiling(self.h, int(mode))

    def stats(self) -> dict:
        s = _native.Stats()
        self.lib.gaplac_get_stats(self.h, byref(s))
        return {name: getattr(s, name) for name, _ in _native.Stats._fields_}

    def reset_stats(self):
        self.lib.gaplac_reset_stats(self.h)


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx
