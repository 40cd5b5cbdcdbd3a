"""bench.py's configs[3] leg end to end at world size 2 (gloo, both ranks on cuda:0: RCCL
refuses two ranks on one GPU; the driver's 8-GPU node runs the nccl backend through the
same functions). Each rank runs bench.measure_config3_dist inside bench.bounded_leg -- the
worker thread, its device selection, DistRank + TorchTransport, the max-over-ranks timing,
and on rank 0 the single-GPU reference and parity_vs_single -- at N = 12000 (configs[3]'s
SqExp workload at a smaller order). The line must come back without error and match the
single-GPU evaluation to the bench's 1e-9 bar."""
import os
import socket
import sys

import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import datetime

        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        import bench
        from gaplac_amd import configs as CF
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
        inputs = CF.config3_inputs(12000)
        line, expired = bench.bounded_leg(
            rank, lambda: bench.measure_config3_dist(rank, world, 0, torch, dist, steps=1, inputs=inputs), 120.0,
            device=0)
        q.put((rank, line, expired))
        if not expired:
            dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}, False))


def test_bench_dist_leg_world2_gloo():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        rank, line, expired = q.get(timeout=180)
        got[rank] = (line, expired)
    for p in procs:
        p.join(timeout=60)
    line, expired = got[0]
    assert not expired and "error" not in line, line
    assert line["ranks_seen"] == 2 and line["parity_ok"], line
    assert line["parity_vs_single"] <= 1e-9
    assert "error" not in got[1][0], got[1]
