"""The distributed evaluation over a real RCCL communicator (torch.distributed "nccl").

RCCL refuses two ranks on one GPU, so the multi-rank nccl job is the driver's 8-GPU run
(bench.py --gpus N: extra.dist). This test runs the same code path at world_size 1 in a
child process: TorchTransport issues every panel broadcast with dist.broadcast on the
library's comm stream (torch.cuda.ExternalStream), with the hipEvent timing bench.py
uses, and the (logdet, quad) allreduce and info MIN on the rank's own device. Checked
against the oracle (bar 1e-9 relative, observed ~1e-15) and against the in-process
loopback schedule.
"""
import os
import socket

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(N, seed):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0, 10, N)
    g = rng.integers(0, max(1, N // 3), N).astype(float)
    v = rng.standard_normal(N)
    return np.column_stack([t, g]), [(1, 0, 1.5, 0), (2, 0, 3.0, 1), (4, 1, 0.0, 2), (5, -1, 1.0, 3)], v


def _worker(port, q):
    try:
        import datetime

        import torch
        import torch.distributed as dist
        from gaplac_amd import distributed as DI
        from gaplac_amd.backend import PosDefException
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                                timeout=datetime.timedelta(seconds=60))
        out = {}
        for N, spw in ((3000, 1), (9000, 4)):
            X, terms, v = _case(N, seed=N)
            r = DI.DistRank(0, 1, 0, spw=spw)
            tr = DI.TorchTransport(device=torch.device("cuda", 0), timing=True)
            lp = DI.logpdf_dist([r], tr, X, terms, 0.1, v, full=True)
            out[N] = (lp, tr.bcast_ms(), len(tr._ev))
            r.close()
        # a non-positive-definite input: info travels through the MIN allreduce
        rng = np.random.default_rng(5)
        Xc = rng.integers(0, 40, 700).astype(float)[:, None]
        r = DI.DistRank(0, 1, 0, spw=1)
        try:
            DI.logpdf_dist([r], DI.TorchTransport(), Xc, [(4, 0, 0.0, 0)], 0.0, rng.standard_normal(700))
            out["info"] = 0
        except PosDefException as e:
            out["info"] = e.info
        r.close()
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((None, repr(e)))


def test_nccl_world1_broadcast_path_matches_oracle():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    from oracle import restatement as R
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    out, err = q.get(timeout=110)
    p.join(timeout=30)
    assert err is None, err
    for N in (3000, 9000):
        X, terms, v = _case(N, seed=N)
        (lp, ld, qd), bc_ms, nbc = out[N]
        rl, rd, rq = R.logpdf(X, terms, 0.1, v)
        assert abs(lp - rl) <= 1e-9 * abs(rl)
        assert abs(ld - rd) <= 1e-9 * abs(rl) and abs(qd - rq) <= 1e-9 * abs(rl)
        assert nbc >= 2 and bc_ms >= 0.0  # every super-panel went through dist.broadcast
    rng = np.random.default_rng(5)
    Xc = rng.integers(0, 40, 700).astype(float)[:, None]
    with pytest.raises(R.PosDefException) as ref:
        R.logpdf(Xc, [(4, 0, 0.0, 0)], 0.0, rng.standard_normal(700))
    assert out["info"] == ref.value.info
