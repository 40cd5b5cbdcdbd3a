"""The one-GPU replay of one rank of a distributed job (gaplac_amd/dist_replay.py,
DESIGN.md §7.3): the replayed rank's arithmetic is the job's (its partial logdet / quad
sums equal the loopback run's for the same rank), the modelled transfers are released no
earlier than the model says, and the model's inputs are measured."""
import numpy as np
import pytest

from gaplac_amd import distributed as DI
from gaplac_amd import dist_replay as RP
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("world,rank,depth,chunk,big,alone,tail,snake", [
    (4, 1, 2, 1, 1, 1, 0, 0), (4, 3, 4, 2, 1, 0, 0, 0), (3, 0, 1, 4, 0, 1, 0, 0), (3, 2, 2, 2, 1, 1, 0, 1),
    (4, 0, 2, 2, 1, 1, 24, 1), (4, 2, 2, 2, 1, 1, 24, 0)])
def test_replay_rank_matches_loopback(world, rank, depth, chunk, big, alone, tail, snake):
    """tail > 0: the tail gather onto rank 0, replayed: the root's partial
    sums (its columns and the gathered tail) equal the loopback run's, and the gathered
    segments arrive no earlier than the model says."""
    import torch
    N = 9000
    rng = np.random.default_rng(17)
    x = rng.uniform(-5, 5, N)
    v = rng.standard_normal(N)
    terms = [(1, 0, 1.5, 0)]
    dx = torch.from_numpy(x).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    owners = [DI.DistRank(0, world, r, spw=4, tail=tail, snake=snake) for r in range(world)]
    DI.logpdf_dist_device(owners, DI.LoopbackTransport(), N, 1, dx.data_ptr(), N, terms, 0.1, dv.data_ptr())
    ld0, q0, info0 = owners[rank].finish()
    rep = DI.DistRank(0, world, rank, spw=4, depth=depth, chunk=chunk, big=big, alone=alone, tail=tail, snake=snake)
    model = RP.ReplayModel(bw_GBps=50.0, lat_us=20.0)
    F = band = None
    for _ in range(2):
        res = RP.replay_rank(owners, rep, N, 1, dx.data_ptr(), terms, 0.1, dv.data_ptr(), model, F=F, band=band)
        assert abs(res["logdet_part"] - ld0) <= 1e-13 * abs(ld0)
        assert abs(res["quad_part"] - q0) <= 1e-13 * max(1.0, abs(q0))
        assert res["info"] == info0 == 0
        # every remote chunk left no earlier than its model time after the owner's inputs
        st, maxc, nch = res["stamps"], res["maxc"], res["nch"]
        recv = st[:, 3 + maxc:3 + 2 * maxc]
        lat = model.lat_ticks()
        for s in range(1, res["nsp"]):
            if rep.owns(s):
                continue
            for c in range(nch[s]):
                fs = (F[s][c] if F else 50000 * (c + 1))
                assert recv[s, c] >= res["last_recv"][s - 1] + fs + lat - 2, (s, c)
        assert res["f_meas"] and all(v[-1] > 0 for v in res["f_meas"].values())
        if tail:
            t = res["tail"]
            g = rep.geometry(N)
            nsteps = res["nsp"]
            tNt = g["Np"] - nsteps * 4 * 128
            sent = {}
            for i, sp in enumerate(range(nsteps, g["nsp"])):
                o = rep.owner(sp)
                if o:
                    sent[o] = sent.get(o, 0) + min(4, g["nt"] - sp * 4) * 128 * (tNt - i * 512) * 8
            need = (model.lat + max(sent.values()) / (model.gbw * 1e9) * 1e6) if rank == 0 else model.lat
            # both stamps are rounded to 0.1 us and the modelled link time to 10 ns ticks
            assert t["arrive_us"] >= t["steps_end_us"] + need - 0.15, (t, need)
            if rank == 0:
                assert t["tail_end_us"] > t["arrive_us"] and t["tail_ms"] > 0
        else:
            assert res["tail"] is None
        F, band = RP.next_inputs(res)
    rep.close()
    for r in owners:
        r.close()
