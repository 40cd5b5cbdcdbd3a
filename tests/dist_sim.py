"""CPU test double of one distributed rank (the gaplac_dist_* step contract), in numpy.

It implements the same per-rank contract as gaplac_amd.distributed.DistRank (ownership,
local column storage, group panel buffers of `depth` panels with their geometry and
parity, broadcast chunks of `chunk` tile columns, the lookahead in factor(s+1), and the
bulk updates of the library's own step plan, gaplac_dist_plan_tail, and the tail gather's
segments) with a smaller tile edge, so the orchestration in
gaplac_amd/distributed.py (schedule order, per-chunk broadcast roots and counts, the gather,
the combine) runs end to end under a gloo process group on CPU. Test infrastructure only;
the Gram comes from the oracle restatement, the root's tail is a dense numpy Cholesky.
"""
import numpy as np

from gaplac_amd import distributed as DI
from oracle import restatement as R


class SimRank:
    def __init__(self, nranks: int, rank: int, spw: int = 2, nb: int = 16, depth: int = 2, chunk: int = None,
                 pair_m: int = 2, tail: int = 0, tail_root: int = 0, snake: int = 0):
        self.nranks, self.rank, self.spw, self.nb = nranks, rank, spw, nb
        self.depth, self.cw, self.pair_m = depth, (chunk or spw), pair_m
        self.tail, self.tail_root, self.snake = tail, tail_root, snake
        self.device = None
        self._bufs = None
        self._tbuf = None
        self.applied = None  # per local tile column: panels applied, in order (checked by tests)
        self.tail_part = None  # the root's (logdet, quad, info) of the gathered trailing matrix

    def owner(self, s):  # gaplac_dist.hip owner()
        r = s % self.nranks
        return self.nranks - 1 - r if self.snake and (s // self.nranks) % 2 else r

    def owns(self, s):
        return self.owner(s) == self.rank

    def geometry(self, N):
        nb, W = self.nb, self.spw
        Np = (N + 1 + nb - 1) // nb * nb
        nt = Np // nb
        nsp = (nt + W - 1) // W
        nloc = sum(min(W, nt - s * W) for s in range(nsp) if self.owner(s) == self.rank)
        return dict(Np=Np, nt=nt, nsp=nsp, nloc=nloc, panel_elems=Np * min(self.depth * W, nt) * nb)

    def use_torch_panel_buffers(self, N):
        import torch
        need = self.geometry(N)["panel_elems"]
        self._bufs = [torch.zeros(need, dtype=torch.float64) for _ in range(2)]
        self._tail_layout(N)
        self._tbuf = torch.zeros(max(1, self._telems), dtype=torch.float64)

    # ---- tail gather (gaplac_dist.hip: tail_stop_of / tail_geom)
    def _tail_layout(self, N):
        g = self.geometry(N)
        nt, nsp, W, nb = g["nt"], g["nsp"], self.spw, self.nb
        stop = -1
        if self.tail > 0 and nt > self.tail:
            stop = (nt - self.tail + W - 1) // W
            if not (1 <= stop < nsp):
                stop = -1
        self.tstop = stop
        self._tseg = []  # (offset, count) per segment, count 0 when not on this rank
        self._telems = 0
        if stop < 0:
            return
        self.tN0 = stop * W * nb
        self.tNt = g["Np"] - self.tN0
        for sp in range(stop, nsp):
            i = sp - stop
            here = self.rank == self.tail_root or self.owns(sp)
            c = min(W, nt - sp * W) * nb * (self.tNt - i * W * nb)
            self._tseg.append((self._telems, c) if here else (0, 0))
            if here:
                self._telems += c

    def tail_segments(self):
        return len(self._tseg) if self.tstop >= 0 else 0

    def tail_segment(self, i):
        off, c = self._tseg[i]
        return None, c, self.owner(self.tstop + i)

    def segment_tensor(self, i):
        off, c = self._tseg[i]
        assert c > 0, (self.rank, i)
        return self._tbuf[off:off + c]

    def tail_begin(self):
        W, nb = self.spw, self.nb
        for i, (off, c) in enumerate(self._tseg):
            sp = self.tstop + i
            if not self.owns(sp):
                continue
            lc0 = (sp // self.nranks) * W
            w = self._width(sp)
            r0 = sp * W * nb
            rows = self.tNt - i * W * nb
            seg = self.C[r0:, lc0 * nb:(lc0 + w) * nb]  # rows x w*nb
            self._tbuf[off:off + c] = __import__("torch").from_numpy(np.asfortranarray(seg).reshape(-1, order="F"))
            assert seg.shape[0] == rows
        return 0

    def tail_end(self):
        if self.rank != self.tail_root:
            return
        W, nb, N = self.spw, self.nb, self.N
        Nt, N0 = self.tNt, self.tN0
        T = np.zeros((Nt, Nt))
        buf = self._tbuf.numpy()
        for i, (off, c) in enumerate(self._tseg):
            rows = Nt - i * W * nb
            cols = c // rows
            r0 = i * W * nb
            T[r0:, r0:r0 + cols] = buf[off:off + c].reshape(cols, rows).T
        info, ld, q = 0, 0.0, 0.0
        for jj in range(Nt):
            j = N0 + jj
            piv = T[jj, jj]
            if j >= N:
                piv = 1.0
            elif not piv > 0 and info == 0:
                info = j + 1
            d = np.sqrt(piv) if piv > 0 else np.nan
            T[jj, jj] = d
            T[jj + 1:, jj] /= d
            T[jj + 1:, jj + 1:] -= np.outer(T[jj + 1:, jj], T[jj + 1:, jj])
            if j < N:
                ld += np.log(d)
                q += T[N - N0, jj] ** 2
        self.tail_part = (2 * ld, q, info)

    # ---- panel geometry (gaplac_dist.hip: group_* / chunk_*)
    def _width(self, s):
        return min(self.spw, self.nt - s * self.spw)

    def _group(self, s):
        g0 = s // self.depth * self.depth
        origin = g0 * self.spw * self.nb
        return g0, origin, self.Np - origin

    def _group_view(self, s):
        """Column-major view of panel s's group buffer: [row - origin, panel column]."""
        g0, origin, ld = self._group(s)
        buf = self._bufs[(s // self.depth) & 1]
        ncol = buf.numel() // ld
        return buf[:ld * ncol].numpy().reshape(ncol, ld).T, g0, origin

    def chunks(self, s):
        return (self._width(s) + self.cw - 1) // self.cw

    def _chunk_range(self, s, c):
        """(offset, count) of chunk c of panel s in its group buffer."""
        g0, origin, ld = self._group(s)
        r0 = s * self.spw * self.nb
        col0 = (s - g0) * self.spw * self.nb + c * self.cw * self.nb
        ncols = min(self.cw, self._width(s) - c * self.cw) * self.nb
        return col0 * ld + (r0 - origin), ncols * ld - (r0 - origin)

    def panel_chunk(self, s, c):
        return None, self._chunk_range(s, c)[1], self.owner(s)

    def chunk_tensor(self, s, c):
        off, count = self._chunk_range(s, c)
        return self._bufs[(s // self.depth) & 1][off:off + count]

    def panel_tensor(self, s, count, ptr=None):
        raise AssertionError("the transports address panels by chunk")

    def comm_begin_chunk(self, s, c):
        return 0

    def comm_end_chunk(self, s, c):
        pass

    # global tile column of local tile column lj (ColMap::global)
    def gcol(self, lj):
        W, P = self.spw, self.nranks
        u = lj // W
        r = P - 1 - self.rank if self.snake and u % 2 else self.rank
        return (u * P + r) * W + lj % W

    def begin(self, X, terms, noise, v):
        g = self.geometry(len(v))
        self.N, self.Np, self.nt, self.nsp, self.nloc = len(v), g["Np"], g["nt"], g["nsp"], g["nloc"]
        N, Np, nb = self.N, self.Np, self.nb
        A = np.zeros((Np, Np))
        A[:N, :N] = R.gram(np.asarray(X, dtype=float).reshape(N, -1), terms, noise)
        A[N, :N] = v
        self.C = np.zeros((Np, self.nloc * nb))
        for lj in range(self.nloc):
            bj = self.gcol(lj)
            self.C[:, lj * nb:(lj + 1) * nb] = A[:, bj * nb:(bj + 1) * nb]
        self.info = 0
        self.plan = DI.plan(self.nt, self.spw, self.depth, self.pair_m, self.tail)
        self._tail_layout(N)
        assert len(self.plan) == (self.tstop if self.tstop >= 0 else self.nsp)
        self.applied = [[] for _ in range(self.nloc)]
        self.tail_part = None
        return len(self.plan)

    def _apply(self, q, lj0, ncols):
        """C[:, local tile cols lj0..lj0+ncols) -= panel q's contributions (rows >= column)."""
        P, g0, origin = self._group_view(q)
        nb, W = self.nb, self.spw
        c0 = (q - g0) * W * nb
        Pq = P[:, c0:c0 + self._width(q) * nb]
        for lj in range(lj0, lj0 + ncols):
            g = self.gcol(lj) * nb
            rows = slice(g, self.Np)
            self.C[rows, lj * nb:(lj + 1) * nb] -= Pq[g - origin:, :] @ Pq[g - origin:g - origin + nb, :].T
            self.applied[lj].append(q)

    def _apply_sp(self, sp, pf, pl):
        W = self.spw
        u = sp // self.nranks
        for q in range(pf, pl + 1):
            self._apply(q, u * W, min(W, self.nloc - u * W))

    def factor(self, s):
        assert self.owns(s)
        W, nb, N = self.spw, self.nb, self.N
        c0 = s * W
        w = self._width(s)
        lc0 = (s // self.nranks) * W
        if s > 0:
            self._apply(s - 1, lc0, w)
        r0 = c0 * nb
        B = self.C[r0:, lc0 * nb:(lc0 + w) * nb]  # view
        for jj in range(w * nb):
            j = r0 + jj
            piv = B[jj, jj]
            if j >= N:
                piv = 1.0
            elif not piv > 0 and self.info == 0:
                self.info = j + 1
            d = np.sqrt(piv) if piv > 0 else np.nan
            B[jj, jj] = d
            B[jj + 1:, jj] /= d
            B[jj + 1:, jj + 1:] -= np.outer(B[jj + 1:, jj], B[jj + 1:w * nb, jj])
        P, g0, origin = self._group_view(s)
        col0 = (s - g0) * W * nb
        P[r0 - origin:, col0:col0 + w * nb] = B

    def update(self, s):
        W = self.spw
        for kind, g, pf, pl in self.plan[s]:
            if kind == 0:
                if g < self.nsp and self.owns(g):
                    self._apply_sp(g, pf, pl)
            elif kind == 1:
                for u in range((self.nloc + W - 1) // W):
                    sg = self.gcol(u * W) // W
                    if sg >= g:
                        self._apply_sp(sg, pf, pl)

    def finish(self):
        nb, N = self.nb, self.N
        stop = self.tstop if self.tstop >= 0 else self.nsp
        # every local column got every earlier panel exactly once, in order (a gathered SP:
        # every distributed panel)
        for lj in range(self.nloc):
            sp = self.gcol(lj) // self.spw
            assert self.applied[lj] == list(range(min(sp, stop))), (lj, self.applied[lj])
        ld = q = 0.0
        info = self.info
        if self.tstop >= 0 and self.rank == self.tail_root:
            assert self.tail_part is not None, "the gather was not completed"
            ld, q, ti = self.tail_part[0] / 2, self.tail_part[1], self.tail_part[2]
            if ti and (info == 0 or ti < info):
                info = ti
        for lj in range(self.nloc):
            if self.gcol(lj) // self.spw >= stop:
                continue
            for e in range(nb):
                j = self.gcol(lj) * nb + e
                if j < N:
                    ld += np.log(self.C[j, lj * nb + e])
                    q += self.C[N, lj * nb + e] ** 2
        return 2 * ld, q, info
