"""Replay of one rank of an N-GPU distributed evaluation on ONE GPU.

BASELINE configs[3] (N = 65536 over 8 MI355X) needs an 8-GPU node, which this project's
GPU pool does not provide. This module predicts one rank's evaluation time on such a
node from a run of that rank's real work on one GPU:

* every kernel the rank runs on a real node runs here for real, on its own GPU-sized
  share: its Gram tiles, its factor() chains (lookahead, diagonal blocks, TRSMs, packs),
  its 1/P-width bulk updates, with the same streams, events and kernel choices
  (gaplac_dist_configure's per-rank big-kernel policy);
* the other ranks' panels arrive as device-to-device copies of their columns, factored
  beforehand by an in-process loopback run of the whole job, released on the rank's comm
  stream by a spinning kernel at the time the model gives (gaplac_dist_replay_chunk):
      owner ready(s) = max(arrival(s-1), UPD(s-2) + band(s))
      arrival(s, c)  = max(owner ready(s) + F(s, c), arrival(s, c-1)) + lat + bytes(s, c) / BW
  where UPD(s-2) is when this rank's own update(s-2) started (every rank's s_main runs the
  same steps at the same time, up to the 1/P shares), band(s) and F(s, c) (the owner's time
  from its inputs to chunk c packed) are MEASURED on this rank's own super-panels (every
  P-th) in the previous iteration and interpolated in s, and lat, BW model the link;
* this rank's own panels leave at PACK(s, c) + lat + bytes / BW (its sends);
* with the tail gather every sender's segments leave when its last update
  ends (taken as this rank's own END) over its own link at gather_bw, so the root's
  receives arrive at END(last) + lat + (the largest sender's bytes) / gather_bw, as copies
  from the owners' segment buffers (gaplac_dist_replay_tail); the root then runs the tail.

Iterated a few times (F and band from the previous run), the rank's evaluation time is
the prediction; the per-step stamps show whether a step waited for the panel (comm/chain
bound) or for its own bulk update. Everything this rank computes is checked against the
loopback run's storage for the same rank (bitwise: the same kernels on the same inputs).
"""
from __future__ import annotations

import time
from ctypes import c_int32, c_int64, c_uint64, c_void_p, byref

import numpy as np

from . import distributed as DI

TICK_S = 1e-8  # s_memrealtime: 100 MHz


class ReplayModel:
    """Link model: per broadcast chunk lat_us + bytes / (bw_GBps * 1e9); the tail gather's
    point-to-point sends over one xGMI link each at gather_bw_GBps."""

    def __init__(self, bw_GBps: float = 200.0, lat_us: float = 15.0, gather_bw_GBps: float = 50.0):
        self.bw, self.lat, self.gbw = float(bw_GBps), float(lat_us), float(gather_bw_GBps)

    def gather_ticks_per_byte(self) -> float:
        return 1.0 / (self.gbw * 1e9) / TICK_S

    def xfer_ticks(self, nbytes: int) -> int:
        return int(round(nbytes / (self.bw * 1e9) / TICK_S))

    def lat_ticks(self) -> int:
        return int(round(self.lat * 1e-6 / TICK_S))


ST_EXTRA = 4  # gaplac_dist.hip: Gram end, gather arrival, tail end, gather copies end


def _stamps(r: DI.DistRank, nsp: int):
    per, maxc = c_int32(), c_int32()
    nb = c_int64()
    r._check(r.lib.gaplac_dist_replay_info(r.h, 0, 0, byref(nb), byref(per), byref(maxc)))
    n = nsp * per.value + ST_EXTRA
    out = (c_uint64 * n)()
    r._check(r.lib.gaplac_dist_replay_stamps(r.h, out, n))
    a = np.frombuffer(out, dtype=np.uint64).astype(np.int64)
    return a[:-ST_EXTRA].reshape(nsp, per.value), maxc.value, [int(x) for x in a[-ST_EXTRA:]]


def _interp(samples: dict, nsp: int, default: float) -> np.ndarray:
    """Linear interpolation in s of {s: value}, clamped at the ends."""
    if not samples:
        return np.full(nsp, default)
    xs = np.array(sorted(samples))
    ys = np.array([samples[x] for x in xs], dtype=float)
    return np.interp(np.arange(nsp), xs, ys)


def replay_rank(owners, rep: DI.DistRank, N: int, D: int, dX_ptr: int, terms, noise: float, dv_ptr: int,
                model: ReplayModel, F=None, band=None, copy_ticks: int = 0, tail_copy_ticks: int = 0,
                senders_end_us: float = 0.0):
    """One replayed evaluation of rank rep.rank. owners[q]: the factored loopback context of
    rank q (a loopback run with the same tail gather). F[s][c], band[s]: model inputs in
    ticks (None: a first guess). senders_end_us: the root's gather waits for the latest
    sender's last update, from that rank's replay (its tail["steps_end_us"]; 0: this rank's
    own). Returns a dict of the time, the stamps and the measured inputs for the next
    iteration."""
    import torch
    rep._check(rep.lib.gaplac_dist_replay_enable(rep.h, int(N)))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nsp = rep.begin_device(N, D, dX_ptr, N, terms, noise, dv_ptr)  # the distributed steps
    nsp_all = rep.geometry(N)["nsp"]
    P = rep.nranks
    nch = [rep.chunks(s) for s in range(nsp)]
    if F is None:  # first guess: 0.5 ms per chunk of chain
        F = [[50000 * (c + 1) for c in range(nch[s])] for s in range(nsp)]
    if band is None:
        band = [0] * nsp
    lat = model.lat_ticks()

    def release(s):
        for c in range(nch[s]):
            nbytes = c_int64()
            rep._check(rep.lib.gaplac_dist_replay_info(rep.h, s, c, byref(nbytes), None, None))
            src = owners[rep.owner(s)].h if not rep.owns(s) else None
            rep._check(rep.lib.gaplac_dist_replay_chunk(rep.h, src, s, c, int(F[s][c]), int(band[s]), lat,
                                                        model.xfer_ticks(nbytes.value), int(copy_ticks)))

    # begin enqueued the Gram; the schedule of distributed.run_schedule with the
    # modelled transfers in place of the broadcasts
    if rep.owns(0):
        rep.factor(0)
    release(0)
    for s in range(nsp):
        if s + 1 < nsp and rep.owns(s + 1):
            rep.factor(s + 1)
        rep.update(s)
        if s + 1 < nsp:
            release(s + 1)
    gathered = rep.tail_segments() > 0
    if gathered:
        arr = (c_void_p * P)(*[o.h.value for o in owners])
        rep._check(rep.lib.gaplac_dist_replay_tail(rep.h, arr, P, lat, model.gather_ticks_per_byte(),
                                                   int(tail_copy_ticks), int(round(senders_end_us * 100))))
    ld, q, info = rep.finish()
    wall = time.perf_counter() - t0
    st, maxc, extra = _stamps(rep, nsp_all)
    gram_done, t_arrive, t_tail_end, t_copied = extra
    st = st[:nsp]
    rep._check(rep.lib.gaplac_dist_replay_enable(rep.h, 0))
    UPD, BAND = st[:, 0], st[:, 1]
    PACK = st[:, 3:3 + maxc]
    RECV = st[:, 3 + maxc:3 + 2 * maxc]
    last = [RECV[s, nch[s] - 1] for s in range(nsp)]
    # measured on this rank's own super-panels: band(s) = its band in update(s-2); F(s, c)
    # from the later of its inputs (panel s-1 in, SP s up to date) to chunk c packed
    f_meas, b_meas = {}, {}
    for s in range(nsp):
        if not rep.owns(s):
            continue
        if s >= 2:
            b_meas[s] = float(BAND[s - 2] - UPD[s - 2])
        ready = max(last[s - 1] if s >= 1 else gram_done, BAND[s - 2] if s >= 2 else 0)
        f_meas[s] = [float(PACK[s, c] - ready) for c in range(nch[s])]
    copies = [float(PACK[s, c] - RECV[s, c]) for s in range(nsp) if not rep.owns(s) for c in range(nch[s])]
    t_first = gram_done
    tail = None
    root = gathered and rep.rank == rep.tail_root
    if gathered:
        end_last = int(st[nsp - 1, 2])
        tail = dict(steps_end_us=round((end_last - t_first) * 0.01, 1), arrive_us=round((t_arrive - t_first) * 0.01, 1))
        if root:
            tail.update(copies_us=round(max(0, t_copied - t_arrive) * 0.01, 1),
                        tail_end_us=round((t_tail_end - t_first) * 0.01, 1),
                        tail_ms=round((t_tail_end - max(t_copied, t_arrive)) * 1e-5, 3))
    return dict(wall_s=wall, nsp=nsp, nch=nch, stamps=st, maxc=maxc, f_meas=f_meas, b_meas=b_meas,
                copy_mean=float(np.mean(copies)) if copies else 0.0, logdet_part=ld, quad_part=q, info=info,
                last_recv=last, t_first=t_first, tail=tail,
                tail_copy=max(0, t_copied - t_arrive) if root else 0)


def next_inputs(res: dict, prev_F=None, prev_band=None):
    """F[s][c] and band[s] for the next iteration from this rank's measured super-panels
    (the first guess where none is measured yet)."""
    nsp, nch = res["nsp"], res["nch"]
    maxch = max(nch)
    F = [[0] * nch[s] for s in range(nsp)]
    for c in range(maxch):
        samp = {s: v[c] for s, v in res["f_meas"].items() if c < len(v)}
        if not samp:
            samp = {s: v[-1] for s, v in res["f_meas"].items()}
        col = _interp(samp, nsp, 50000.0 * (c + 1))
        for s in range(nsp):
            if c < nch[s]:
                F[s][c] = int(max(0.0, col[s]))
    band = [int(max(0.0, b)) for b in _interp(res["b_meas"], nsp, 0.0)]
    return F, band


def step_table(res: dict, P: int, rank: int, owner=None):
    """Per step: the panel's arrival (last chunk), this rank's update start and end, and
    how long its s_main sat idle waiting for the panel (> 0: the step was chain / link
    bound on this rank; 0: the panel was there before the stream got to it)."""
    st = res["stamps"]
    t0 = res["t_first"]
    rows = []
    prev_end = t0
    for s in range(res["nsp"]):
        arr = int(res["last_recv"][s]) - t0
        upd, end = int(st[s, 0]) - t0, int(st[s, 2]) - t0
        o = owner(s) if owner else s % P
        rows.append(dict(s=s, owner=o, own=(o == rank), arrival_us=arr * 0.01, upd_start_us=upd * 0.01,
                         upd_end_us=end * 0.01, main_idle_us=max(0, upd - (prev_end - t0 if s else 0)) * 0.01))
        prev_end = end + t0
    return rows
