"""N>1 host path on CPU: world_size-2 gloo process groups (no GPU needed).

The GPU path shards independent evaluations over ranks (replicas); here
the per-unit evaluator is the CPU oracle so the sharding/gather logic and the batched
select aggregation are exercised end to end.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gaplac_amd import replicas
from gaplac_amd.backend import PosDefException


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_round_robin_covers_everything_once():
    for n in (0, 1, 5, 64):
        for w in (1, 2, 3, 8):
            got = sorted(u for r in range(w) for u in replicas.shard(n, r, w))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        replicas.shard(4, 2, 2)


class _OracleCtx:
    """Stands in for gaplac_amd.backend.Context in the CPU test (same batch signature)."""

    def logpdf_batch(self, X, models, noise, v):
        from oracle import restatement as R
        out, info = [], []
        for m in models:
            try:
                out.append(R.logpdf(X, m, noise, v)[0])
                info.append(0)
            except R.PosDefException as e:
                out.append(float("nan"))
                info.append(e.info)
        return np.array(out), np.array(info)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(4)
        N = 200
        X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 30, N).astype(float)])
        v = rng.standard_normal(N)
        models = [[(1, 0, l, 0)] for l in (0.5, 1.0, 2.0, 4.0)] + [[(2, 0, 1.0, 0), (4, 1, 0.0, 1)],
                                                                 [(4, 1, 0.0, 0)], [(3, 0, 0.5, 0)]]
        res = replicas.select_batch(_OracleCtx(), X, models, 0.1, v)
        vals = replicas.run_sharded(lambda u: float(u) * 10 + rank * 0, 5)
        # a non-PD candidate (Cat only, no observation noise): PosDefException on every
        # rank, as select.jl's logpdf would raise; or NaN + info with raise_posdef=False
        bad = [m + [(5, -1, 0.1, 1)] for m in models[:3]] + [[(4, 1, 0.0, 0)]]  # Noise terms keep 0..2 PD
        try:
            replicas.select_batch(_OracleCtx(), X, bad, 0.0, v)
            raised = None
        except PosDefException as e:
            raised = e.info
        bv, binfo = replicas.select_batch(_OracleCtx(), X, bad, 0.0, v, raise_posdef=False)
        q.put((rank, res.tolist(), vals.tolist(), raised, binfo.tolist(), bool(np.isnan(bv[3]))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_select_batch_matches_single_process():
    from oracle import restatement as R
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(4)
    N = 200
    X = np.column_stack([rng.uniform(0, 10, N), rng.integers(0, 30, N).astype(float)])
    v = rng.standard_normal(N)
    models = [[(1, 0, l, 0)] for l in (0.5, 1.0, 2.0, 4.0)] + [[(2, 0, 1.0, 0), (4, 1, 0.0, 1)],
                                                             [(4, 1, 0.0, 0)], [(3, 0, 0.5, 0)]]
    expect = [R.logpdf(X, m, 0.1, v)[0] for m in models]
    with pytest.raises(R.PosDefException) as ref:
        R.logpdf(X, [(4, 1, 0.0, 0)], 0.0, v)
    for rank, res, vals, raised, binfo, isnan in got:
        assert np.allclose(res, expect, rtol=1e-12, atol=0)
        assert vals == [0.0, 10.0, 20.0, 30.0, 40.0]
        assert raised == ref.value.info
        assert binfo[:3] == [0, 0, 0] and binfo[3] == ref.value.info and isnan
