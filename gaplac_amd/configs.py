"""Synthetic inputs of the BASELINE.json configurations, seeded.

One definition shared by bench.py and the GPU tests, so that the benchmarked workloads
are exactly the ones the parity tests cover:

  configs[1]  SqExp(:x), N = 4096, x ~ U(-5, 5), seed 1; v ~ N(0, 1); l swept over
              {0.5, 1, 1.5, 3} to emulate MCMC proposals
  configs[2]  SqExp(:t; l) + OU(:t; l=3) + Cat(:subject) + Noise, N = 16384, t ~ U(0, 10),
              subject = randint(0, N/3), seed 2 (the headline metric)
  configs[3]  SqExp(:x; l=1.5), N = 65536, x ~ U(-5, 5), seed 3 (one evaluation over the
              GPUs of a node)
  configs[4]  select over 64 candidate formulas (16 structures over the columns x, t,
              subject x lengthscales {0.5, 1, 2, 4}), N = 8192, seed 4

Term tuples are the lowered descriptors (kind, column, param, group) of kernels.lower.
"""
from __future__ import annotations

import numpy as np

from ._native import CAT, LINEAR, NOISE, OU, SQEXP

N1, N2, N3, N4 = 4096, 16384, 65536, 8192
LENGTHSCALES_1 = (0.5, 1.0, 1.5, 3.0)
LENGTHSCALES_2 = (1.0, 1.5, 2.0, 3.0)
NOISE_VAR = 0.1  # FiniteGP(..., 0.1): CLI/src/mcmc.jl:35, CLI/src/select.jl:43,47


def config1_inputs(N: int = N1, seed: int = 1):
    """configs[1]: x (N,) and v (N,)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-5.0, 5.0, N)
    v = rng.standard_normal(N)
    return x, v


def config1_terms(l: float):
    return [(SQEXP, 0, float(l), 0)]


def config2_inputs(N: int = N2, seed: int = 2):
    """configs[2]: X (N x 2: t, subject) and v (N,)."""
    rng = np.random.default_rng(seed)
    t = rng.uniform(0.0, 10.0, N)
    subject = rng.integers(0, max(1, N // 3), N).astype(np.float64)
    v = rng.standard_normal(N)
    return np.column_stack([t, subject]), v


def config2_terms(l_sqexp: float):
    """SqExp(:t; l) + OU(:t; l=3) + Cat(:subject) + Noise, each term its own group."""
    return [(SQEXP, 0, float(l_sqexp), 0), (OU, 0, 3.0, 1), (CAT, 1, 0.0, 2), (NOISE, -1, 1.0, 3)]


def config3_inputs(N: int = N3, seed: int = 3):
    """configs[3]: x (N,) and v (N,)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-5.0, 5.0, N)
    v = rng.standard_normal(N)
    return x, v


CONFIG3_TERMS = [(SQEXP, 0, 1.5, 0)]


def config4_inputs(N: int = N4, seed: int = 4):
    """configs[4]: X (N x 3: x, t, subject) and y (N,)."""
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.uniform(-5, 5, N), rng.uniform(0, 10, N),
                         rng.integers(0, max(1, N // 3), N).astype(np.float64)])
    y = rng.standard_normal(N)
    return X, y


def select_models():
    """configs[4]: the 64 candidate formulas, lowered. Columns: 0 x, 1 t, 2 subject; every
    term is its own group (GaPLAC formulas lower to sums)."""
    x, t, g = 0, 1, 2
    structures = [
        lambda l: [(SQEXP, x, l)], lambda l: [(OU, x, l)], lambda l: [(SQEXP, t, l)], lambda l: [(OU, t, l)],
        lambda l: [(SQEXP, x, l), (CAT, g, 0.0)], lambda l: [(OU, t, l), (CAT, g, 0.0)],
        lambda l: [(SQEXP, x, l), (OU, t, 2 * l)], lambda l: [(SQEXP, t, l), (LINEAR, x, 0.5)],
        lambda l: [(SQEXP, x, l), (SQEXP, t, l)], lambda l: [(OU, x, l), (CAT, g, 0.0)],
        lambda l: [(SQEXP, t, l), (OU, t, 3.0), (CAT, g, 0.0)], lambda l: [(LINEAR, x, l), (CAT, g, 0.0)],
        lambda l: [(SQEXP, x, l), (OU, x, l), (CAT, g, 0.0)], lambda l: [(OU, t, l), (LINEAR, t, 1.0)],
        lambda l: [(SQEXP, x, l), (SQEXP, t, 2 * l), (CAT, g, 0.0)],
        lambda l: [(SQEXP, t, l), (OU, x, l), (LINEAR, x, 0.0), (CAT, g, 0.0)],
    ]
    models = []
    for mk in structures:
        for l in (0.5, 1.0, 2.0, 4.0):
            models.append([(k, c, p, i) for i, (k, c, p) in enumerate(mk(l))])
    return models
