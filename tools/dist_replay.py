"""Predict configs[3] (N = 65536 over P GPUs) per-rank evaluation time on ONE GPU by
replaying one rank's schedule against a modelled link (gaplac_amd/dist_replay.py,
DESIGN.md §7.3).

    python tools/dist_replay.py --N 65536 --ranks 8 --local 0 7 --bw 100 200 300 \
        --depth 2 4 --chunk 1 4 --tail 0 80 --out gpurun_out/r05_dist_replay.jsonl

--tail: the tail gather's tile columns (0 = off), onto rank 0; each value
gets its own loopback run (the owners' segment buffers hold that gather's segments).
--job: replay every rank (the gather's root last, its gather released after the latest
sender's last update from the other replays) and emit the job's prediction (the max over
ranks) per tail length, with the first value of every option list.

First an in-process loopback run of the whole job factors every rank's columns (the
panels the replayed rank receives), then for every option set the replayed rank runs
--iters evaluations (F and band re-measured each time); the last one is the prediction.
One JSON line per replay: options, the predicted ms per evaluation, the inputs, parity of
the replayed rank's partial sums with the loopback's, and a per-step summary.
"""
import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--local", type=int, nargs="+", default=[0])
    ap.add_argument("--bw", type=float, nargs="+", default=[200.0])
    ap.add_argument("--lat", type=float, default=15.0)
    ap.add_argument("--depth", type=int, nargs="+", default=[2])
    ap.add_argument("--chunk", type=int, nargs="+", default=[4])
    ap.add_argument("--big", type=int, nargs="+", default=[1])
    ap.add_argument("--alone", type=int, nargs="+", default=[0])
    ap.add_argument("--tail", type=int, nargs="+", default=[0])
    ap.add_argument("--snake", type=int, nargs="+", default=[-1], help="layout (-1: the library's default)")
    ap.add_argument("--gbw", type=float, nargs="+", default=[50.0], help="gather GB/s per sender link")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--steps", action="store_true", help="include the per-step table")
    ap.add_argument("--job", action="store_true", help="every rank, and the job's prediction")
    ap.add_argument("--single", action="store_true", help="also time the single-GPU path on the input")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import numpy as np
    import torch
    from gaplac_amd import configs as CF
    from gaplac_amd import distributed as DI
    from gaplac_amd import dist_replay as RP

    x, v = CF.config3_inputs(a.N)
    N = a.N
    dx = torch.from_numpy(x).to("cuda")
    dv = torch.from_numpy(v).to("cuda")
    terms = CF.CONFIG3_TERMS
    out = open(a.out, "a") if a.out else None

    def emit(d):
        s = json.dumps(d)
        print(s[:2000], flush=True)
        if out:
            out.write(s + "\n")
            out.flush()

    single_ms = None
    if a.single:
        from gaplac_amd.backend import Context
        with Context(0) as ctx:
            ctx.logpdf_device(N, 1, dx.data_ptr(), N, terms, CF.NOISE_VAR, dv.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lp_single = ctx.logpdf_device(N, 1, dx.data_ptr(), N, terms, CF.NOISE_VAR, dv.data_ptr())
            torch.cuda.synchronize()
            single_ms = (time.perf_counter() - t0) * 1e3
        emit(dict(kind="single", N=N, ms=single_ms, logpdf=lp_single))

    for tail, snake in itertools.product(a.tail, a.snake):
        a.cur_snake = snake
        # the loopback job: every rank's factored columns (the owners of the replayed panels)
        t0 = time.perf_counter()
        owners = [DI.DistRank(0, a.ranks, r, spw=4, tail=tail, snake=snake) for r in range(a.ranks)]
        lp_loop = DI.logpdf_dist_device(owners, DI.LoopbackTransport(), N, 1, dx.data_ptr(), N, terms, CF.NOISE_VAR,
                                        dv.data_ptr())
        parts = {r.rank: r.finish() for r in owners}
        emit(dict(kind="loopback", N=N, ranks=a.ranks, tail=tail, snake=snake, logpdf=lp_loop, s=time.perf_counter() - t0))
        if a.job:
            job(a, owners, parts, tail, N, dx, dv, terms, emit)
        else:
            replays(a, owners, parts, tail, N, dx, dv, terms, single_ms, emit)
        for r in owners:
            r.close()


def _replay(a, owners, rank, tail, N, dx, dv, terms, model, senders_end_us=0.0):
    from gaplac_amd import configs as CF
    from gaplac_amd import distributed as DI
    from gaplac_amd import dist_replay as RP
    rep = DI.DistRank(0, a.ranks, rank, spw=4, depth=a.depth[0], chunk=a.chunk[0], big=a.big[0], alone=a.alone[0],
                      tail=tail, snake=a.cur_snake)
    F = band = None
    copy = tcopy = 0
    hist = []
    for it in range(a.iters):
        res = RP.replay_rank(owners, rep, N, 1, dx.data_ptr(), terms, CF.NOISE_VAR, dv.data_ptr(), model, F=F,
                             band=band, copy_ticks=copy, tail_copy_ticks=tcopy, senders_end_us=senders_end_us)
        hist.append(round(res["wall_s"] * 1e3, 2))
        F, band = RP.next_inputs(res)
        copy = int(res["copy_mean"])
        tcopy = int(res["tail_copy"])
    rows = RP.step_table(res, a.ranks, rank, rep.owner)
    rep.close()
    return res, hist, rows


def job(a, owners, parts, tail, N, dx, dv, terms, emit):
    """Every rank replayed; the root (rank 0) last, its gather released after the latest
    sender's last update."""
    from gaplac_amd import dist_replay as RP
    model = RP.ReplayModel(bw_GBps=a.bw[0], lat_us=a.lat, gather_bw_GBps=a.gbw[0])
    ranks = list(range(1, a.ranks)) + [0]
    per = {}
    senders_end = 0.0
    for rank in ranks:
        res, hist, rows = _replay(a, owners, rank, tail, N, dx, dv, terms, model,
                                  senders_end_us=senders_end if rank == 0 else 0.0)
        ld0, q0, _ = parts[rank]
        per[rank] = dict(predicted_ms=hist[-1], iters_ms=hist, steps_end_ms=round(rows[-1]["upd_end_us"] / 1e3, 3),
                         parts_equal=bool(res["logdet_part"] == ld0 and res["quad_part"] == q0), tail=res["tail"])
        if rank != 0 and tail:
            senders_end = max(senders_end, res["tail"]["steps_end_us"])
    pred = max(v["predicted_ms"] for v in per.values())
    emit(dict(kind="job", N=N, ranks=a.ranks, tail=tail, snake=a.cur_snake, bw_GBps=a.bw[0], gather_bw_GBps=a.gbw[0] if tail else None,
              depth=a.depth[0], chunk=a.chunk[0], big=a.big[0], alone=a.alone[0], predicted_ms=pred,
              slowest=max(per, key=lambda r: per[r]["predicted_ms"]), senders_end_ms=round(senders_end / 1e3, 3),
              per_rank=per))


def replays(a, owners, parts, tail, N, dx, dv, terms, single_ms, emit):
    from gaplac_amd import configs as CF
    from gaplac_amd import distributed as DI
    from gaplac_amd import dist_replay as RP
    for rank, depth, chunk, big, alone in itertools.product(a.local, a.depth, a.chunk, a.big, a.alone):
        rep = DI.DistRank(0, a.ranks, rank, spw=4, depth=depth, chunk=chunk, big=big, alone=alone, tail=tail,
                          snake=a.cur_snake)
        for bw, gbw in itertools.product(a.bw, a.gbw if tail else a.gbw[:1]):
            model = RP.ReplayModel(bw_GBps=bw, lat_us=a.lat, gather_bw_GBps=gbw)
            F = band = None
            copy = tcopy = 0
            hist = []
            res = None
            for it in range(a.iters):
                res = RP.replay_rank(owners, rep, N, 1, dx.data_ptr(), terms, CF.NOISE_VAR, dv.data_ptr(), model,
                                     F=F, band=band, copy_ticks=copy, tail_copy_ticks=tcopy)
                hist.append(round(res["wall_s"] * 1e3, 2))
                F, band = RP.next_inputs(res)
                copy = int(res["copy_mean"])
                tcopy = int(res["tail_copy"])
            ld0, q0, _ = parts[rank]
            rows = RP.step_table(res, a.ranks, rank, rep.owner)
            idle = [r["main_idle_us"] for r in rows]
            f_own = {s: [round(t * 0.01, 1) for t in v] for s, v in res["f_meas"].items()}
            d = dict(kind="replay", N=N, ranks=a.ranks, rank=rank, depth=depth, chunk=chunk, big=big, alone=alone, bw_GBps=bw,
                     lat_us=a.lat, tail=tail, gather_bw_GBps=gbw if tail else None, tail_stamps=res["tail"],
                     iters_ms=hist, predicted_ms=hist[-1],
                     speedup_vs_single=(single_ms / hist[-1]) if single_ms else None,
                     logdet_part_equal=res["logdet_part"] == ld0, quad_part_equal=res["quad_part"] == q0,
                     logdet_part_rel=abs(res["logdet_part"] - ld0) / max(1e-300, abs(ld0)),
                     copy_us=round(res["copy_mean"] * 0.01, 2),
                     steps_main_waited=sum(1 for b in idle if b > 5),
                     main_idle_ms=round(sum(idle) / 1e3, 3),
                     main_end_ms=round(rows[-1]["upd_end_us"] / 1e3, 3),
                     chain_ms_own=f_own)
            if a.steps:
                d["steps"] = rows
            emit(d)
        rep.close()


if __name__ == "__main__":
    main()
