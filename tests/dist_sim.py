"""CPU test double of one distributed rank (the gaplac_dist_* step contract), in numpy.

It implements the same per-rank contract as gaplac_amd.distributed.DistRank (ownership,
local column storage, panel buffer geometry and parity, lookahead in factor(s+1), bulk
update of super-panels > s+1) with a smaller tile edge, so the orchestration in
gaplac_amd/distributed.py (schedule order, broadcast roots and counts, the combine) runs
end to end under a gloo process group on CPU. Test infrastructure only; the Gram comes
from the oracle restatement.
"""
import numpy as np

from oracle import restatement as R


class SimRank:
    def __init__(self, nranks: int, rank: int, spw: int = 2, nb: int = 16):
        self.nranks, self.rank, self.spw, self.nb = nranks, rank, spw, nb
        self.device = None
        self._bufs = None

    def owns(self, s):
        return s % self.nranks == self.rank

    def geometry(self, N):
        nb, W = self.nb, self.spw
        Np = (N + 1 + nb - 1) // nb * nb
        nt = Np // nb
        nsp = (nt + W - 1) // W
        nloc = sum(min(W, nt - s * W) for s in range(self.rank, nsp, self.nranks))
        return dict(Np=Np, nt=nt, nsp=nsp, nloc=nloc, panel_elems=Np * min(W, nt) * nb)

    def use_torch_panel_buffers(self, N):
        import torch
        need = self.geometry(N)["panel_elems"]
        self._bufs = [torch.zeros(need, dtype=torch.float64) for _ in range(2)]

    def panel_tensor(self, s, count, ptr=None):
        return self._bufs[s & 1][:count]

    # global tile column of local tile column lj (ColMap::global)
    def gcol(self, lj):
        W = self.spw
        return ((lj // W) * self.nranks + self.rank) * W + lj % W

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
        return self.nsp

    def _panel(self, s):
        W, nb = self.spw, self.nb
        w = min(W, self.nt - s * W)
        r0 = s * W * nb
        ldp = self.Np - r0
        P = self._bufs[s & 1][:ldp * w * nb].numpy().reshape(w * nb, ldp).T  # column-major view
        return P, r0

    def _apply(self, s, lj0, ncols):
        """C[:, local tile cols lj0..lj0+ncols) -= panel s contributions (rows >= column)."""
        P, r0 = self._panel(s)
        nb = self.nb
        for lj in range(lj0, lj0 + ncols):
            g0 = self.gcol(lj) * nb
            rows = slice(g0, self.Np)
            self.C[rows, lj * nb:(lj + 1) * nb] -= P[g0 - r0:, :] @ P[g0 - r0:g0 - r0 + nb, :].T

    def factor(self, s):
        assert self.owns(s)
        W, nb, N = self.spw, self.nb, self.N
        c0 = s * W
        w = min(W, self.nt - c0)
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
        ldp = self.Np - r0
        self._bufs[s & 1][:ldp * w * nb] = __import__("torch").from_numpy(np.asfortranarray(B).T.reshape(-1).copy())

    def panel(self, s):
        W, nb = self.spw, self.nb
        w = min(W, self.nt - s * W)
        return None, (self.Np - s * W * nb) * w * nb, s % self.nranks

    def comm_begin(self, s):
        return 0

    def comm_end(self, s):
        pass

    def update(self, s):
        W = self.spw
        for u in range((self.nloc + W - 1) // W):
            sg = u * self.nranks + self.rank
            if sg > s + 1:
                self._apply(s, u * W, min(W, self.nloc - u * W))

    def finish(self):
        nb, N = self.nb, self.N
        ld = q = 0.0
        for lj in range(self.nloc):
            for e in range(nb):
                j = self.gcol(lj) * nb + e
                if j < N:
                    ld += np.log(self.C[j, lj * nb + e])
                    q += self.C[N, lj * nb + e] ** 2
        return 2 * ld, q, self.info
