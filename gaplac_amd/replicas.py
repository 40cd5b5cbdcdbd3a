"""Multi-GPU execution of independent evaluations ("replicas").

The path does not need a collective for independent units: MCMC chains, hyperparameter
points and `select` candidates (BASELINE configs[4]: 64 formulas x N=8192) are sharded
over ranks, one process per GPU, and only the scalar results are gathered. There is no
data-path collective; the gather of a handful of doubles at the end is the only
communication (torch.distributed: RCCL on GPUs, gloo on CPU in the tests).

    rank r of W owns units r, r+W, r+2W, ...   (round-robin: balances mixed formula costs)
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import numpy as np


def shard(n_units: int, rank: int, world: int) -> List[int]:
    """Units owned by `rank` (round-robin)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return list(range(rank, n_units, world))


def gather_results(local_idx: Sequence[int], local_vals: Sequence[float], n_units: int,
                   group=None, device=None) -> np.ndarray:
    """All-gather (index, value) pairs so every rank holds the full result vector."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    per = (n_units + world - 1) // world
    buf = torch.full((per, 2), float("nan"), dtype=torch.float64, device=device)
    for s, (i, v) in enumerate(zip(local_idx, local_vals)):
        buf[s, 0] = float(i)
        buf[s, 1] = float(v)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    res = np.full(n_units, np.nan)
    for o in outs:
        for i, v in o.cpu().numpy():
            if not np.isnan(i):
                res[int(i)] = v
    return res


def run_sharded(evaluate: Callable[[int], float], n_units: int, group=None, device=None) -> np.ndarray:
    """Evaluate units round-robin over the ranks of `group`; return all results on every rank.

    `evaluate(u)` computes unit u on this rank's GPU (e.g. a gaplac Context logpdf).
    """
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mine = shard(n_units, rank, world)
    vals = [evaluate(u) for u in mine]
    return gather_results(mine, vals, n_units, group=group, device=device)


def select_batch(ctx, X, models, noise: float, v, group=None, device=None, raise_posdef: bool = True):
    """Batched `select` over many formulas, sharded across ranks (BASELINE configs[4]).

    models: list of term lists (lowered descriptors). Each rank runs its share through one
    gaplac_logpdf_batch call; the values and the per-model potrf info are all-gathered.
    Like the reference (CLI/src/select.jl:49-50: logpdf -> cholesky(check=true)), a
    formula whose covariance is not positive definite raises PosDefException(info) — the
    first such model's, on every rank. raise_posdef=False instead returns
    (values, info) with NaN values where info > 0."""
    import torch.distributed as dist
    from .backend import PosDefException
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    mine = shard(len(models), rank, world)
    if mine:
        out, info = ctx.logpdf_batch(X, [models[u] for u in mine], noise, v)
    else:
        out, info = [], []
    vals = gather_results(mine, list(out), len(models), group=group, device=device)
    infos = gather_results(mine, [float(i) for i in info], len(models), group=group, device=device)
    infos = np.nan_to_num(infos, nan=0.0).astype(np.int64)
    if raise_posdef:
        bad = np.nonzero(infos > 0)[0]
        if bad.size:
            raise PosDefException(int(infos[bad[0]]))
        return vals
    return vals, infos
