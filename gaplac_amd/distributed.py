"""Distributed log-marginal-likelihood: 1-D block-column cyclic Cholesky over ranks.

BASELINE configs[3] (N = 65536 over the GPUs of one node) / SURVEY.md §8e. One process
per GPU (torch.distributed: backend "nccl" = RCCL over xGMI). Each rank owns the
super-panels s with s % world == rank (W = 4 tile columns of 128 each by default), builds
only its own Gram tiles, and the only data-path exchange is one broadcast of each factored
super-panel from its owner; the result needs one allreduce of (logdet, quad) and a min of
the failing-pivot index. The compute lives in libgaplac_hip.so (gaplac_dist_* in
include/gaplac.h); this module sequences the steps and issues the collectives.

With the snake layout (set_layout) SP s belongs to rank world-1-s%world in
odd rounds of world super-panels; owner(s) asks the library.

Reference semantics are those of gaplac_logpdf (AbstractGPs.logpdf(FiniteGP, v) at
CLI/src/mcmc.jl:35 and CLI/src/select.jl:49-50): the same value to <= 1e-9 relative,
PosDefException(info) on a non-positive pivot.

Transports:
  TorchTransport(group)  one rank per process; broadcasts with torch.distributed on the
                         library's comm stream (RCCL on GPUs; gloo in CPU/1-GPU tests)
  LoopbackTransport()    every rank of the job in this process on one device: the
                         broadcast is a device-to-device copy (tests of the multi-rank
                         schedule at any rank count on a single GPU)

Schedule (per rank; every library call only enqueues work except finish):
    begin -> nsteps; factor(0) [owner]; bcast(0)
    for s in 0..nsteps-1: factor(s+1) [owner of s+1, s+1 < nsteps]; update(s); bcast(s+1)
    [tail gather: tail_begin; send / receive the segments; tail_end]
    finish -> partial (logdet, quad, info); combine across ranks
bcast(s) is one broadcast per chunk of panel s (a run of its tile columns): the owner packs
a chunk as soon as its last column is final, and the next owner's lookahead consumes it as
it arrives. With the tail gather (set_tail) the last
super-panels are not stepped: every rank sends its columns of the trailing matrix to the
root, which factors it with the single-GPU persistent tail (nsteps < nsp).
"""
from __future__ import annotations

import ctypes
import math
from ctypes import byref, c_double, c_int32, c_int64, c_void_p
from typing import List, Optional, Sequence

import numpy as np

from . import _native
from ._native import term_array
from .backend import ArgumentError, GaplacError, PosDefException, _colmajor

LOG2PI = 1.8378770664093453  # Julia's log2π (AbstractGPs logpdf)
DEFAULT_SPW = 4


class DistRank:
    """One rank's state (a gaplac_dist context) on `device`."""

    def __init__(self, device: int, nranks: int, rank: int, spw: int = DEFAULT_SPW, depth: int = -1,
                 chunk: int = -1, big: int = -1, big_min: int = -1, alone: int = -1, tail: int = -1,
                 tail_root: int = 0, snake: int = -1):
        self.lib = _native.load()
        h = c_void_p()
        rc = self.lib.gaplac_dist_create(int(device), int(nranks), int(rank), int(spw), byref(h))
        if rc != 0:
            raise GaplacError(rc, f"gaplac_dist_create(device={device}, nranks={nranks}, rank={rank}) failed")
        self.h = h
        self.device, self.nranks, self.rank, self.spw = device, nranks, rank, spw
        self._bufs = None  # torch tensors backing the panel buffers (kept alive here)
        self._tbuf = None  # torch tensor backing the tail-gather segment buffer
        self._nseg = 0
        self.tail_root = 0
        self.configure(depth, chunk, big, big_min, alone)
        if tail >= 0:
            self.set_tail(tail, tail_root)
        if snake >= 0:
            self.set_layout(snake)

    def set_layout(self, snake: int):
        """gaplac_dist_set_layout: 1 = snake (boustrophedon) dealing of the super-panels."""
        self._check(self.lib.gaplac_dist_set_layout(self.h, int(snake)))

    def owner(self, s: int) -> int:
        r = c_int32()
        self._check(self.lib.gaplac_dist_owner(self.h, int(s), byref(r)))
        return r.value

    def global_col(self, lj: int) -> int:
        """Global tile column of local tile column lj (ColMap::global)."""
        u, e = divmod(lj, self.spw)
        s = next(u * self.nranks + k for k in range(self.nranks) if self.owner(u * self.nranks + k) == self.rank)
        return s * self.spw + e

    def set_tail(self, cols: int, root: int = 0):
        """Tail gather (gaplac_dist_set_tail): the super-panels in the last `cols` tile
        columns are factored on rank `root` by the persistent tail; 0 = off."""
        self._check(self.lib.gaplac_dist_set_tail(self.h, int(cols), int(root)))
        self.tail_root = int(root)

    def tail_geometry(self, N: int):
        nseg, elems, nsteps = c_int32(), c_int64(), c_int32()
        self._check(self.lib.gaplac_dist_tail_geometry(self.h, int(N), byref(nseg), byref(elems), byref(nsteps)))
        return dict(nseg=nseg.value, elems=elems.value, nsteps=nsteps.value)

    def configure(self, depth: int = -1, chunk: int = -1, big: int = -1, big_min: int = -1, alone: int = -1):
        """Schedule options (gaplac_dist_configure; -1 keeps the current value): deferral
        depth, tile columns per broadcast chunk, bulk kernel choice (2 for ranks sharing one
        device, as LoopbackTransport's do), chain alone (the bulk update waits while this
        rank factors the next super-panel; 0 for ranks sharing one device)."""
        if self._bufs is not None and depth != -1:
            raise ArgumentError("configure the depth before the panel buffers are set")
        self._check(self.lib.gaplac_dist_configure(self.h, int(depth), int(chunk), int(big), int(big_min),
                                                   int(alone)))

    def close(self):
        if getattr(self, "h", None):
            self.lib.gaplac_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc == 0:
            return
        msg = self.lib.gaplac_dist_last_error(self.h)
        msg = msg.decode() if msg else ""
        if rc in (_native.E_PARAM, _native.E_KIND, _native.E_COL, _native.E_ARG):
            raise ArgumentError(f"gaplac error {rc}: {msg}")
        raise GaplacError(rc, msg)

    def owns(self, s: int) -> bool:
        return self.owner(s) == self.rank

    def geometry(self, N: int):
        Np, pel = c_int64(), c_int64()
        nt, nsp, nloc = c_int32(), c_int32(), c_int32()
        self._check(self.lib.gaplac_dist_geometry(self.h, int(N), byref(Np), byref(nt), byref(nsp), byref(nloc),
                                                  byref(pel)))
        return dict(Np=Np.value, nt=nt.value, nsp=nsp.value, nloc=nloc.value, panel_elems=pel.value)

    def use_torch_panel_buffers(self, N: int):
        """Back the two panel buffers (and the tail gather's segment buffer) with torch
        tensors on this rank's device (so the collective library moves torch tensors)."""
        import torch
        dev = torch.device("cuda", self.device)
        need = self.geometry(N)["panel_elems"]
        if self._bufs is None or self._bufs[0].numel() < need:
            self._bufs = [torch.empty(need, dtype=torch.float64, device=dev) for _ in range(2)]
            self._check(self.lib.gaplac_dist_set_panel_buffers(
                self.h, c_void_p(self._bufs[0].data_ptr()), c_void_p(self._bufs[1].data_ptr()), need))
        tneed = self.tail_geometry(N)["elems"]
        if tneed > 0 and (self._tbuf is None or self._tbuf.numel() < tneed):
            self._tbuf = torch.empty(tneed, dtype=torch.float64, device=dev)
            self._check(self.lib.gaplac_dist_set_tail_buffer(self.h, c_void_p(self._tbuf.data_ptr()), tneed))

    def panel_tensor(self, s: int, count: int, ptr: int = None):
        """The torch view of panel s (count doubles at ptr, inside one of the two pair
        buffers: gaplac_dist_panel)."""
        if ptr is None:
            ptr = self.panel(s)[0]
        for b in self._bufs:
            off = (ptr - b.data_ptr()) // 8
            if 0 <= off and off + count <= b.numel():
                return b[off:off + count]
        raise GaplacError(_native.E_ARG, f"panel {s} is outside the panel buffers")

    # ---- steps
    def begin(self, X: np.ndarray, terms, noise: float, v: np.ndarray) -> int:
        Xc = _colmajor(X)
        v = np.ascontiguousarray(v, dtype=np.float64)
        N, D = Xc.shape
        if v.shape[0] != N:
            raise ArgumentError(f"length of v ({v.shape[0]}) != N ({N})")
        terms = list(terms)
        ta = term_array(terms)
        nsp = c_int32()
        self._check(self.lib.gaplac_dist_begin(self.h, N, D, Xc.ctypes.data_as(c_void_p), max(N, 1), len(terms), ta,
                                               float(noise), v.ctypes.data_as(c_void_p), 0, byref(nsp)))
        self._nseg = self.tail_geometry(N)["nseg"]
        return nsp.value

    def begin_device(self, N: int, D: int, dX_ptr: int, ldx: int, terms, noise: float, dv_ptr: int) -> int:
        terms = list(terms)
        nsp = c_int32()
        self._check(self.lib.gaplac_dist_begin(self.h, N, D, c_void_p(dX_ptr), ldx, len(terms), term_array(terms),
                                               float(noise), c_void_p(dv_ptr), 1, byref(nsp)))
        self._nseg = self.tail_geometry(N)["nseg"]
        return nsp.value

    def factor(self, s: int):
        self._check(self.lib.gaplac_dist_factor(self.h, int(s)))

    def panel(self, s: int):
        ptr, count, root = c_void_p(), c_int64(), c_int32()
        self._check(self.lib.gaplac_dist_panel(self.h, int(s), byref(ptr), byref(count), byref(root)))
        return ptr.value, count.value, root.value

    def comm_begin(self, s: int) -> int:
        st = c_void_p()
        self._check(self.lib.gaplac_dist_comm_begin(self.h, int(s), byref(st)))
        return st.value or 0

    def comm_end(self, s: int):
        self._check(self.lib.gaplac_dist_comm_end(self.h, int(s)))

    def chunks(self, s: int) -> int:
        n = c_int32()
        self._check(self.lib.gaplac_dist_chunks(self.h, int(s), byref(n)))
        return n.value

    def panel_chunk(self, s: int, c: int):
        ptr, count, root = c_void_p(), c_int64(), c_int32()
        self._check(self.lib.gaplac_dist_panel_chunk(self.h, int(s), int(c), byref(ptr), byref(count), byref(root)))
        return ptr.value, count.value, root.value

    def chunk_tensor(self, s: int, c: int):
        ptr, count, _root = self.panel_chunk(s, c)
        return self.panel_tensor(s, count, ptr)

    def comm_begin_chunk(self, s: int, c: int) -> int:
        st = c_void_p()
        self._check(self.lib.gaplac_dist_comm_begin_chunk(self.h, int(s), int(c), byref(st)))
        return st.value or 0

    def comm_end_chunk(self, s: int, c: int):
        self._check(self.lib.gaplac_dist_comm_end_chunk(self.h, int(s), int(c)))

    def update(self, s: int):
        self._check(self.lib.gaplac_dist_update(self.h, int(s)))

    # ---- tail gather
    def tail_segments(self) -> int:
        """Segments of this evaluation's gather (0: none)."""
        return self._nseg

    def tail_segment(self, i: int):
        ptr, count, src = c_void_p(), c_int64(), c_int32()
        self._check(self.lib.gaplac_dist_tail_segment(self.h, int(i), byref(ptr), byref(count), byref(src)))
        return ptr.value, count.value, src.value

    def segment_tensor(self, i: int):
        """The torch view of segment i in this rank's segment buffer."""
        ptr, count, _src = self.tail_segment(i)
        if not ptr or self._tbuf is None:
            raise GaplacError(_native.E_ARG, f"tail segment {i} is not on rank {self.rank}")
        off = (ptr - self._tbuf.data_ptr()) // 8
        if off < 0 or off + count > self._tbuf.numel():
            raise GaplacError(_native.E_ARG, f"tail segment {i} is outside the segment buffer")
        return self._tbuf[off:off + count]

    def tail_begin(self) -> int:
        st = c_void_p()
        self._check(self.lib.gaplac_dist_tail_begin(self.h, byref(st)))
        return st.value or 0

    def tail_end(self):
        self._check(self.lib.gaplac_dist_tail_end(self.h))

    def finish(self):
        ld, q, info = c_double(), c_double(), c_int64()
        self._check(self.lib.gaplac_dist_finish(self.h, byref(ld), byref(q), byref(info)))
        return ld.value, q.value, info.value

    def local(self, N: int) -> np.ndarray:
        g = self.geometry(N)
        out = np.zeros((g["Np"], g["nloc"] * 128), dtype=np.float64, order="F")
        if g["nloc"]:
            self._check(self.lib.gaplac_dist_local(self.h, out.ctypes.data_as(c_void_p), g["Np"]))
        return out


class TorchTransport:
    """One rank per process; torch.distributed collectives on the rank's comm stream.

    device: where the 3-number allreduce runs (default: the rank's own GPU, DistRank.device,
    for the nccl backend — not torch's current device, which a process-per-GPU caller may
    not have set — and the CPU otherwise).
    timing: record hipEvents on the comm stream around every broadcast (bcast_ms())."""

    def __init__(self, group=None, device=None, timing: bool = False):
        self.group = group
        self.device = device
        self.rank_device = None
        self.timing = timing
        self._ev = []

    def prepare(self, ranks: Sequence, N: int):
        (r,) = ranks
        r.use_torch_panel_buffers(N)
        self.rank_device = r.device

    def reset_timing(self):
        self._ev = []

    def bcast_ms(self) -> float:
        """Sum of the recorded broadcasts' durations on the comm stream (synchronises)."""
        tot = 0.0
        for a, b in self._ev:
            b.synchronize()
            tot += a.elapsed_time(b)
        return tot

    def bcast(self, ranks: Sequence, s: int):
        """One broadcast per chunk of panel s, each on the library's comm stream."""
        import torch
        import torch.distributed as dist
        (r,) = ranks
        for c in range(r.chunks(s)):
            _ptr, _count, root = r.panel_chunk(s, c)
            stream = r.comm_begin_chunk(s, c)
            buf = r.chunk_tensor(s, c)
            src = dist.get_global_rank(self.group, root) if self.group is not None else root
            if stream and buf.is_cuda:
                st = torch.cuda.ExternalStream(stream, device=buf.device)
                with torch.cuda.stream(st):
                    if self.timing:
                        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                        ev[0].record(st)
                    dist.broadcast(buf, src=src, group=self.group, async_op=True).wait()
                    if self.timing:
                        ev[1].record(st)
                        self._ev.append(ev)
            else:
                dist.broadcast(buf, src=src, group=self.group)
            r.comm_end_chunk(s, c)

    def gather_tail(self, ranks: Sequence):
        """The tail gather: this rank's segments to the root, or the root's receives, as one
        batch of point-to-point ops on the library's comm stream (RCCL send / recv over
        xGMI with the nccl backend: every sender's link runs at once). gloo's point-to-point
        ops take host tensors, so with gloo a device segment goes through a host copy."""
        import torch
        import torch.distributed as dist
        (r,) = ranks
        n = r.tail_segments()
        stream = r.tail_begin()
        root = r.tail_root
        ops = []
        for i in range(n):
            _ptr, _count, src = r.tail_segment(i)
            if src == root or r.rank not in (src, root):
                continue
            peer = root if r.rank == src else src
            gpeer = dist.get_global_rank(self.group, peer) if self.group is not None else peer
            ops.append((dist.isend if r.rank == src else dist.irecv, r.segment_tensor(i), gpeer))
        if ops:
            t0 = ops[0][1]
            st = torch.cuda.ExternalStream(stream, device=t0.device) if (stream and t0.is_cuda) else None
            if st is not None and dist.get_backend(self.group) == "nccl":
                with torch.cuda.stream(st):
                    reqs = dist.batch_isend_irecv([dist.P2POp(op, t, peer, group=self.group) for op, t, peer in ops])
                    for q in reqs:
                        q.wait()
            else:
                if st is not None:
                    st.synchronize()  # the packs
                host = [t.cpu() if op is dist.isend else torch.empty(t.shape, dtype=t.dtype) for op, t, _ in ops]
                reqs = [op(h, peer, group=self.group) for (op, _t, peer), h in zip(ops, host)]
                for q in reqs:
                    q.wait()
                for (op, t, _), h in zip(ops, host):
                    if op is dist.irecv:
                        if st is not None:
                            with torch.cuda.stream(st):
                                t.copy_(h, non_blocking=False)
                        else:
                            t.copy_(h)
        r.tail_end()

    def combine(self, parts: Sequence, device=None):
        import torch
        import torch.distributed as dist
        (ld, q, info), = parts
        dev = device if device is not None else self.device
        if dev is None:
            if dist.get_backend(self.group) == "nccl":
                dev = torch.device("cuda", self.rank_device if self.rank_device is not None
                                   else torch.cuda.current_device())
            else:
                dev = "cpu"
        sums = torch.tensor([ld, q], dtype=torch.float64, device=dev)
        imin = torch.tensor([info if info > 0 else np.iinfo(np.int64).max], dtype=torch.int64, device=dev)
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group)
        dist.all_reduce(imin, op=dist.ReduceOp.MIN, group=self.group)
        info = int(imin.item())
        return float(sums[0].item()), float(sums[1].item()), 0 if info == np.iinfo(np.int64).max else info


class LoopbackTransport:
    """All ranks of the job in this process, on one device: broadcast = D2D copies on the
    receivers' comm streams, ordered after the root's pack; the root's comm stream then
    waits for every copy, so its buffer is not re-packed before the copies have read it.

    keep_options: leave each rank's schedule options as configured (the multi-rank
    defaults: chain alone, per-rank bulk kernel) instead of the single-GPU choices the
    shared device would favour; for correctness checks of those options across ranks that
    exchange panels (they only add waits inside a rank, so they are valid on one device)."""

    def __init__(self, keep_options: bool = False):
        self.keep_options = keep_options

    def prepare(self, ranks: Sequence, N: int):
        for r in ranks:
            if len(ranks) > 1 and hasattr(r, "configure") and not self.keep_options:
                r.configure(big=2, alone=0)  # the ranks share one device: the single-GPU choices
            r.use_torch_panel_buffers(N)

    def bcast(self, ranks: Sequence, s: int):
        import torch
        root = ranks[0].panel_chunk(s, 0)[2]
        rootr = next(r for r in ranks if r.rank == root)
        for c in range(rootr.chunks(s)):
            streams = {r.rank: torch.cuda.ExternalStream(r.comm_begin_chunk(s, c), device=torch.device("cuda", r.device))
                       for r in ranks}
            src = rootr.chunk_tensor(s, c)
            for r in ranks:
                if r.rank == root:
                    continue
                st = streams[r.rank]
                st.wait_stream(streams[root])
                with torch.cuda.stream(st):
                    r.chunk_tensor(s, c).copy_(src, non_blocking=True)
                streams[root].wait_stream(st)
            for r in ranks:
                r.comm_end_chunk(s, c)

    def gather_tail(self, ranks: Sequence):
        """Every sender's segments copied into the root's buffer on the root's comm stream
        (after the sender's packs; the sender's stream then waits for the copy, so its buffer
        is not re-packed before the copy has read it)."""
        import torch
        root = ranks[0].tail_root
        rootr = next(r for r in ranks if r.rank == root)
        streams = {r.rank: torch.cuda.ExternalStream(r.tail_begin(), device=torch.device("cuda", r.device))
                   for r in ranks}
        by_rank = {r.rank: r for r in ranks}
        for i in range(rootr.tail_segments()):
            _ptr, _count, src = rootr.tail_segment(i)
            if src == root:
                continue
            st = streams[root]
            st.wait_stream(streams[src])
            with torch.cuda.stream(st):
                rootr.segment_tensor(i).copy_(by_rank[src].segment_tensor(i), non_blocking=True)
            streams[src].wait_stream(st)
        for r in ranks:
            r.tail_end()

    def combine(self, parts: Sequence, device=None):
        ld = sum(p[0] for p in parts)
        q = sum(p[1] for p in parts)
        infos = [p[2] for p in parts if p[2] > 0]
        return ld, q, (min(infos) if infos else 0)


def plan(nt: int, spw: int, depth: int, pair_m: int = 40, tail: int = 0):
    """The library's step plan (gaplac_dist_plan_tail, host-only): a list per step of
    (kind, sp, first panel, last panel), kind 0 = that SP, 1 = every SP from it on, 2 = the
    step's event once SP step+2 is up to date. tail: the tail gather's tile columns (the
    plan then has fewer steps than super-panels)."""
    lib = _native.load()
    n = c_int64()
    rc = lib.gaplac_dist_plan_tail(int(nt), int(spw), int(depth), int(pair_m), int(tail), None, 0, byref(n))
    if rc != 0:
        raise ArgumentError(f"gaplac_dist_plan({nt}, {spw}, {depth}, tail={tail}) failed: {rc}")
    buf = (c_int32 * (5 * max(1, n.value)))()
    lib.gaplac_dist_plan_tail(int(nt), int(spw), int(depth), int(pair_m), int(tail), buf, 5 * n.value, byref(n))
    nsteps = max((buf[5 * i] for i in range(n.value)), default=-1) + 1
    steps = [[] for _ in range(nsteps)]
    for i in range(n.value):
        p, kind, g, pf, pl = buf[5 * i:5 * i + 5]
        steps[p].append((kind, g, pf, pl))
    return steps


def plan_check(nt: int, spw: int, depth: int, pair_m: int = 40, tail: int = 0):
    """gaplac_dist_plan_check_tail: (ok, op count, message)."""
    lib = _native.load()
    ops = c_int64()
    msg = ctypes.create_string_buffer(256)
    rc = lib.gaplac_dist_plan_check_tail(int(nt), int(spw), int(depth), int(pair_m), int(tail), byref(ops), msg, 256)
    return rc == 0, ops.value, msg.value.decode()


def run_schedule(ranks: Sequence, transport, nsteps: int):
    """Enqueue one evaluation's factorisation on the local ranks (begin already called and
    returned nsteps): the distributed steps, then the tail gather when there is one."""
    for r in ranks:
        if r.owns(0):
            r.factor(0)
    transport.bcast(ranks, 0)
    for s in range(nsteps):
        if s + 1 < nsteps:
            for r in ranks:
                if r.owns(s + 1):
                    r.factor(s + 1)
        for r in ranks:
            r.update(s)
        if s + 1 < nsteps:
            transport.bcast(ranks, s + 1)
    if ranks[0].tail_segments() > 0:
        transport.gather_tail(ranks)


def finish(ranks: Sequence, transport, N: int, device=None, full: bool = False):
    parts = [r.finish() for r in ranks]
    ld, q, info = transport.combine(parts, device=device)
    if info > 0:
        raise PosDefException(info)
    lp = -((N * LOG2PI + ld) + q) / 2.0
    return (lp, ld, q) if full else lp


def logpdf_dist(ranks: Sequence[DistRank], transport, X, terms, noise: float, v, full: bool = False,
                device=None):
    """logpdf of the zero-mean FiniteGP with the factorisation spread over the job's ranks.

    ranks: the DistRank(s) this process drives ([one] with TorchTransport, all of them
    with LoopbackTransport). Returns the same value on every rank."""
    X = _colmajor(X)
    N = X.shape[0]
    if N == 0:
        return (-0.0, 0.0, 0.0) if full else -0.0
    transport.prepare(ranks, N)
    nsps = [r.begin(X, terms, noise, v) for r in ranks]
    run_schedule(ranks, transport, nsps[0])
    return finish(ranks, transport, N, device=device, full=full)


def logpdf_dist_device(ranks: Sequence[DistRank], transport, N: int, D: int, dX_ptr: int, ldx: int, terms,
                       noise: float, dv_ptr: int, full: bool = False, device=None):
    """As logpdf_dist with X (N x D column-major, leading dim ldx) and v already on the
    device (the benchmark's entry)."""
    transport.prepare(ranks, N)
    nsps = [r.begin_device(N, D, dX_ptr, ldx, terms, noise, dv_ptr) for r in ranks]
    run_schedule(ranks, transport, nsps[0])
    return finish(ranks, transport, N, device=device, full=full)
