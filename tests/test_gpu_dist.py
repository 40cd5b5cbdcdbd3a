"""Distributed evaluation through the C-ABI (gaplac_dist_*) on the GPU.

* LoopbackTransport: every rank of a 1..8-rank job in this process on cuda:0 — the real
  HIP steps on the 1-D block-column cyclic layout, with the broadcast as D2D copies.
* TorchTransport over a world_size-2 gloo group: two processes sharing cuda:0 (RCCL
  refuses two ranks on one GPU; the driver's 8-GPU node runs the nccl backend).
Bar: the north_star's <= 1e-9 relative logpdf against the oracle (observed ~1e-15); the
1-rank distributed path also agrees with the single-GPU gaplac_logpdf to 1e-12.
"""
import os
import socket

import numpy as np
import pytest

from gaplac_amd import distributed as DI
from gaplac_amd.backend import Context, PosDefException
from oracle import restatement as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu
RTOL = 1e-9


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def _case(N, seed=0):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0, 10, N)
    g = rng.integers(0, max(1, N // 3), N).astype(float)
    v = rng.standard_normal(N)
    X = np.column_stack([t, g])
    terms = [(1, 0, 1.5, 0), (2, 0, 3.0, 1), (4, 1, 0.0, 2), (5, -1, 1.0, 3)]
    return X, terms, v


def _ranks(world, spw):
    return [DI.DistRank(0, world, r, spw=spw) for r in range(world)]


@pytest.mark.parametrize("world,spw,N", [
    (1, 4, 1000), (2, 1, 1000), (2, 4, 3000), (3, 1, 129), (3, 2, 1500), (4, 1, 700),
    (4, 2, 2100), (8, 1, 1100), (8, 1, 300), (2, 2, 1), (3, 1, 127), (3, 1, 128),
])
@pytest.mark.parametrize("snake", [0, 1])
def test_loopback_matches_oracle(world, spw, N, snake):
    X, terms, v = _case(N, seed=world * 7 + spw)
    ranks = [DI.DistRank(0, world, r, spw=spw, snake=snake) for r in range(world)]
    lp, ld, q = DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.1, v, full=True)
    rl, rd, rq = R.logpdf(X, terms, 0.1, v)
    assert abs(lp - rl) <= RTOL * abs(rl)
    assert abs(lp - rl) <= 1e-12 * max(1.0, abs(rl))
    assert abs(ld - rd) <= 1e-9 * max(1.0, abs(rd))
    assert abs(q - rq) <= 1e-9 * max(1.0, abs(rq))


@pytest.mark.parametrize("snake", [0, 1])
def test_loopback_factor_columns_match_oracle(snake):
    """Each rank's stored columns are the owned columns of L (and z in row N), in the
    round-robin and the snake layout."""
    N, world, spw = 900, 3, 1
    X, terms, v = _case(N, seed=2)
    ranks = [DI.DistRank(0, world, r, spw=spw, snake=snake) for r in range(world)]
    DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.1, v)
    C = R.gram(X, terms, 0.1)
    L = np.linalg.cholesky(C)
    z = np.linalg.solve(L, v)
    for r in ranks:
        loc = r.local(N)
        g = r.geometry(N)
        for lj in range(g["nloc"]):
            bj = r.global_col(lj)
            if not snake:
                assert bj == ((lj // spw) * world + r.rank) * spw + lj % spw
            for e in range(128):
                j = bj * 128 + e
                if j >= N:
                    continue
                col = loc[:, lj * 128 + e]
                assert np.allclose(col[j:N], L[j:, j], rtol=1e-11, atol=1e-12)
                assert abs(col[N] - z[j]) <= 1e-10 * max(1.0, abs(z[j]))


def test_one_rank_matches_single_gpu_path():
    N = 4096
    rng = np.random.default_rng(1)
    x = rng.uniform(-5, 5, N)
    v = rng.standard_normal(N)
    terms = [(1, 0, 1.5, 0)]
    with Context(0) as ctx:
        ref = ctx.logpdf(x, terms, 0.1, v)
    got = DI.logpdf_dist(_ranks(1, 4), DI.LoopbackTransport(), x, terms, 0.1, v)
    assert abs(got - ref) <= 1e-12 * abs(ref)


@pytest.mark.parametrize("world,spw,N", [(1, 4, 16384), (2, 1, 8192), (4, 2, 12000)])
def test_loopback_large_matches_single_gpu(world, spw, N):
    """Sizes whose bulk updates run the 128x128 tile kernel on the distributed layout
    (> 512 tiles per launch) and long enough to expose stream-ordering races; checked
    against the single-GPU path (itself parity-tested against the oracle)."""
    X, terms, v = _case(N, seed=N)
    with Context(0) as ctx:
        ref = ctx.logpdf(X, terms, 0.1, v)
    ranks = _ranks(world, spw)
    for _ in range(2):
        got = DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.1, v)
        assert abs(got - ref) <= 1e-11 * abs(ref)


@pytest.mark.parametrize("world,spw,N,depth,chunk", [
    (2, 2, 12000, 4, 1), (4, 2, 12000, 8, 2), (3, 4, 14000, 3, 1), (8, 2, 12000, 2, 1), (2, 4, 10000, 1, 2),
    (5, 3, 9000, 4, 3)])
def test_loopback_depth_and_chunks_match_single_gpu(world, spw, N, depth, chunk):
    """Deferral groups of `depth` panels (K up to depth x 128 spw per bulk update) and
    broadcast chunks of `chunk` tile columns (per-chunk packs, events and lookahead
    launches) at sizes where the deferral and the tile kernel run; against the single-GPU
    path and the oracle, twice through the same workspaces."""
    X, terms, v = _case(N, seed=N + depth)
    with Context(0) as ctx:
        ref = ctx.logpdf(X, terms, 0.1, v)
    ranks = [DI.DistRank(0, world, r, spw=spw, depth=depth, chunk=chunk) for r in range(world)]
    for _ in range(2):
        got = DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.1, v)
        assert abs(got - ref) <= 1e-11 * abs(ref)
    for r in ranks:
        r.close()


def test_loopback_non_pd_info():
    rng = np.random.default_rng(5)
    N = 700
    X = rng.integers(0, 40, N).astype(float)[:, None]
    v = rng.standard_normal(N)
    terms = [(4, 0, 0.0, 0)]
    with pytest.raises(R.PosDefException) as ref:
        R.logpdf(X, terms, 0.0, v)
    with pytest.raises(PosDefException) as got:
        DI.logpdf_dist(_ranks(3, 1), DI.LoopbackTransport(), X, terms, 0.0, v)
    assert got.value.info == ref.value.info


def test_loopback_repeated_evals_reuse_workspace():
    X, terms, v = _case(1500, seed=9)
    ranks = _ranks(4, 1)
    tr = DI.LoopbackTransport()
    for l in (0.7, 1.5, 3.0):
        tt = [(1, 0, l, 0)] + terms[1:]
        lp = DI.logpdf_dist(ranks, tr, X, tt, 0.1, v)
        rl = R.logpdf(X, tt, 0.1, v)[0]
        assert abs(lp - rl) <= 1e-12 * abs(rl)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, tail=-1):
    try:
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        X, terms, v = _case(2500, seed=21)
        r = DI.DistRank(0, world, rank, spw=2, tail=tail, tail_root=world - 1)
        lp = DI.logpdf_dist([r], DI.TorchTransport(), X, terms, 0.1, v)
        r.close()
        dist.destroy_process_group()
        q.put((rank, lp, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("tail", [0, 12])
def test_gloo_world2_processes_share_one_gpu(tail):
    """tail 12: the tail gather through TorchTransport.gather_tail (gloo: host copies of the
    segments), onto rank 1."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, tail)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, lp, err in got:
        assert err is None, err
    X, terms, v = _case(2500, seed=21)
    rl = R.logpdf(X, terms, 0.1, v)[0]
    for rank, lp, err in got:
        assert abs(lp - rl) <= 1e-12 * abs(rl)


@pytest.mark.parametrize("world,spw,N,big,snake", [(4, 2, 12000, 1, 0), (4, 2, 12000, 0, 0), (8, 2, 9000, 1, 0),
                                                    (8, 2, 9000, 1, 1), (3, 4, 14000, 1, 1)])
def test_loopback_multirank_defaults_match_single_gpu(world, spw, N, big, snake):
    """the P > 1 defaults (chain alone with held post-mark ops, depth 2, chunk 2,
    the per-rank bulk kernel choice) across ranks that really exchange panels: every rank
    keeps its options (LoopbackTransport(keep_options=True)); against the single-GPU path
    at 1e-11, twice through the same workspaces."""
    X, terms, v = _case(N, seed=N + world)
    with Context(0) as ctx:
        ref = ctx.logpdf(X, terms, 0.1, v)
    ranks = [DI.DistRank(0, world, r, spw=spw, depth=2, chunk=2, big=big, alone=1, snake=snake) for r in range(world)]
    tr = DI.LoopbackTransport(keep_options=True)
    for _ in range(2):
        got = DI.logpdf_dist(ranks, tr, X, terms, 0.1, v)
        assert abs(got - ref) <= 1e-11 * abs(ref)
    for r in ranks:
        r.close()


# ---- tail gather ----

@pytest.mark.parametrize("world,spw,N,tail,root", [
    (1, 4, 3000, 8, 0), (2, 1, 1000, 3, 1), (3, 2, 1500, 5, 2), (4, 2, 2100, 10, 0), (8, 1, 1100, 4, 5),
    (3, 1, 700, 5, 1)])
def test_loopback_tail_gather_matches_oracle(world, spw, N, tail, root):
    """The super-panels of the last `tail` tile columns are gathered onto `root` and factored
    by the persistent tail there; against the oracle at 1e-12."""
    X, terms, v = _case(N, seed=world * 11 + tail)
    ranks = [DI.DistRank(0, world, r, spw=spw, tail=tail, tail_root=root) for r in range(world)]
    assert ranks[0].tail_geometry(N)["nseg"] > 0
    lp, ld, q = DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.1, v, full=True)
    rl, rd, rq = R.logpdf(X, terms, 0.1, v)
    assert abs(lp - rl) <= 1e-12 * max(1.0, abs(rl))
    assert abs(ld - rd) <= 1e-9 * max(1.0, abs(rd))
    assert abs(q - rq) <= 1e-9 * max(1.0, abs(rq))
    for r in ranks:
        r.close()


@pytest.mark.parametrize("world,spw,N,tail,root,snake", [
    (4, 4, 16384, 80, 0, 0), (8, 2, 12000, 40, 7, 1), (2, 4, 14000, 128, 1, 0), (8, 4, 20000, 77, 3, 1)])
def test_loopback_tail_gather_large_matches_single_gpu(world, spw, N, tail, root, snake):
    """At the P > 1 defaults (chain alone, held ops, chunks of 2, per-rank bulk kernel: every
    rank keeps its options) with the gathered tail up to its 128-column maximum; against the
    single-GPU path at 1e-11, twice through the same workspaces."""
    X, terms, v = _case(N, seed=N + tail)
    with Context(0) as ctx:
        ref = ctx.logpdf(X, terms, 0.1, v)
    ranks = [DI.DistRank(0, world, r, spw=spw, depth=2, chunk=2, big=1, alone=1, tail=tail, tail_root=root,
                         snake=snake) for r in range(world)]
    tr = DI.LoopbackTransport(keep_options=True)
    for _ in range(2):
        got = DI.logpdf_dist(ranks, tr, X, terms, 0.1, v)
        assert abs(got - ref) <= 1e-11 * abs(ref)
    for r in ranks:
        r.close()


def test_loopback_tail_gather_non_pd_info_in_the_tail():
    """A first failing pivot inside the gathered matrix (a repeated category at j = 400, tile
    column 3 of 6, the tail = columns 3..5) comes back as its global j + 1."""
    N = 700
    rng = np.random.default_rng(3)
    cats = np.concatenate([np.arange(400), rng.integers(0, 400, N - 400)]).astype(float)
    X = cats[:, None]
    v = rng.standard_normal(N)
    terms = [(4, 0, 0.0, 0)]
    with pytest.raises(R.PosDefException) as ref:
        R.logpdf(X, terms, 0.0, v)
    assert ref.value.info == 401
    ranks = [DI.DistRank(0, 3, r, spw=1, tail=3, tail_root=2) for r in range(3)]
    assert ranks[0].tail_geometry(N)["nsteps"] == 3
    with pytest.raises(PosDefException) as got:
        DI.logpdf_dist(ranks, DI.LoopbackTransport(), X, terms, 0.0, v)
    assert got.value.info == 401


def test_tail_gather_options_and_reuse():
    """set_tail validation; the gather toggled between evaluations on the same contexts."""
    from gaplac_amd.backend import ArgumentError
    r = DI.DistRank(0, 2, 0, spw=2)
    with pytest.raises(ArgumentError):
        r.set_tail(129)
    with pytest.raises(ArgumentError):
        r.set_tail(8, root=2)
    r.close()
    X, terms, v = _case(2600, seed=4)
    rl = R.logpdf(X, terms, 0.1, v)[0]
    ranks = _ranks(3, 2)
    tr = DI.LoopbackTransport()
    for tail in (0, 6, 0, 10, 20):
        for r in ranks:
            r.set_tail(tail, 1)
        lp = DI.logpdf_dist(ranks, tr, X, terms, 0.1, v)
        assert abs(lp - rl) <= 1e-12 * abs(rl), tail
