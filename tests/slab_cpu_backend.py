"""CPU backend of the slab decomposition (TEST INFRASTRUCTURE ONLY).

It implements GpuSlabBackend's interface with numpy and the oracle's phase functions, so
SlabRunner's orchestration (cuts, exchange protocol, canonical [left | own | right] order,
ghost columns, interior/boundary split) runs over gloo on CPU and can be compared with the
single-domain oracle. It uses the oracle's global grid; the GPU uses a local column window of
the same grid, which changes neither the column of any particle nor the sorted order.
"""
from __future__ import annotations

import numpy as np
import torch


class CpuSlabBackend:
    def __init__(self, O, op, sc, cut, jitter_frac=0.01):
        self.O, self.op = O, op
        self.cx_lo, self.cx_hi = cut
        G = op.grid.G
        self.G = (int(G[0]), int(G[1]), int(G[2]))
        self.gyz = int(op.grid.xsub) * self.G[1] * self.G[2]   # keys per column (x sub-columns)
        self.nk = self.G[0] * self.gyz
        self.has_left = self.cx_lo > 0
        self.has_right = self.cx_hi < self.G[0]
        x = O.lattice(sc.dim, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=jitter_frac)
        keys = O.grid_keys(op, x)
        col = keys // self.gyz
        own = (col >= self.cx_lo) & (col < self.cx_hi)
        self.pos = x[own].copy()
        self.vel = np.zeros_like(self.pos)
        self.id = np.nonzero(own)[0].astype(np.int32)
        self.o0, self.o1 = 0, len(self.pos)
        self.rng = [0] * 10
        self.t = 0.0
        self.rp = np.zeros((0, 2), np.float32)

    # interface -------------------------------------------------------------
    def bind_stream(self, handle):
        pass

    def empty(self, n, width):
        return torch.empty((max(n, 1), width), dtype=torch.float32)

    def _cols(self):
        keys = self.O.grid_keys(self.op, self.pos[self.o0:self.o1])
        return keys // self.gyz

    def count_sends(self):
        col = self._cols()
        nl = int((col <= self.cx_lo).sum()) if self.has_left else 0
        nr = int((col >= self.cx_hi - 1).sum()) if self.has_right else 0
        return nl, nr

    def count_sends_into(self, counts):
        nl, nr = self.count_sends()
        counts[0], counts[1] = nl, nr

    def send_capacity(self):
        return max(self.o1 - self.o0, 1)

    def pack_send(self, side, buf, n):
        col = self._cols()
        sel = (col <= self.cx_lo) if side == 0 else (col >= self.cx_hi - 1)
        idx = np.nonzero(sel)[0] + self.o0
        rec = np.zeros((len(idx), 8), np.float32)
        rec[:, 0:3] = self.pos[idx]
        rec[:, 3] = self.id[idx].view(np.float32)
        rec[:, 4:7] = self.vel[idx]
        assert len(rec) <= n, "send buffer smaller than the records"
        buf[:len(rec)] = torch.from_numpy(rec)

    def assemble(self, left, nl, right, nr):
        L = left[:nl].numpy() if nl else np.zeros((0, 8), np.float32)
        R = right[:nr].numpy() if nr else np.zeros((0, 8), np.float32)
        own = slice(self.o0, self.o1)
        pos = np.concatenate([L[:, 0:3], self.pos[own], R[:, 0:3]]).astype(np.float32)
        vel = np.concatenate([L[:, 4:7], self.vel[own], R[:, 4:7]]).astype(np.float32)
        ids = np.concatenate([L[:, 3].view(np.int32), self.id[own], R[:, 3].view(np.int32)]).astype(np.int32)
        keys = self.O.grid_keys(self.op, pos)
        perm = self.O.stable_sort(keys, self.nk)
        self.pos, self.vel, self.id = pos[perm].copy(), vel[perm].copy(), ids[perm].copy()
        self.sk = keys[perm].copy()
        self.cs = self.O.cell_start(self.sk, self.nk)
        cs, g = self.cs, self.gyz
        lo, hi = self.cx_lo, self.cx_hi
        c = lambda col: int(cs[min(max(col, 0), self.G[0]) * g])   # noqa: E731
        gl = (c(lo - 1), c(lo)) if self.has_left else (c(lo), c(lo))
        gr = (c(hi), c(hi + 1)) if self.has_right else (c(hi), c(hi))
        self.rng = [gl[0], gl[1], c(lo), c(hi), gr[0], gr[1], c(lo), c(lo + 1), c(hi - 1), c(hi)]
        self.o0, self.o1 = self.rng[2], self.rng[3]
        self.rp = np.zeros((len(self.pos), 2), np.float32)

    def ranges(self):
        return list(self.rng)

    def density(self):
        rho = np.zeros(len(self.pos), np.float32)
        prho = np.zeros(len(self.pos), np.float32)
        self.O.density_range(self.op, self.pos, self.sk, self.cs, self.o0, self.o1, rho, prho)
        self.rp[self.o0:self.o1, 0] = rho[self.o0:self.o1]
        self.rp[self.o0:self.o1, 1] = prho[self.o0:self.o1]

    def pack_rho(self, side, buf, n):
        b, e = self.rng[6 + 2 * side], self.rng[7 + 2 * side]
        assert e - b == n
        buf[:n] = torch.from_numpy(self.rp[b:e].copy())

    def unpack_rho(self, side, buf, n):
        b, e = self.rng[4 * side], self.rng[4 * side + 1]
        assert e - b == n, (side, e - b, n)
        if n:
            self.rp[b:e] = buf[:n].numpy()

    def force(self, dt, part):
        if not hasattr(self, "pos_out") or len(self.pos_out) != len(self.pos):
            self.pos_out = self.pos.copy()
            self.vel_out = self.vel.copy()
        r = self.rng
        ib = r[7] if self.has_left else r[2]
        ie = r[8] if self.has_right else r[3]
        if part == 1:
            spans = [(ib, max(ib, ie))]
        elif ie < ib:
            spans = [(r[2], r[3])]
        else:
            spans = [(r[2], ib), (ie, r[3])]
        rho = np.ascontiguousarray(self.rp[:, 0])
        prho = np.ascontiguousarray(self.rp[:, 1])
        for b, e in spans:
            if e > b:
                self.O.force_range(self.op, self.pos, self.vel, rho, prho, self.sk, self.cs, b, e, dt,
                                   np.float32(self.t), self.pos_out, self.vel_out)

    def finish(self, dt):
        self.pos, self.vel = self.pos_out, self.vel_out
        del self.pos_out, self.vel_out
        self.t += dt

    def column_counts(self, ncols):
        out = np.zeros(ncols, np.int64)
        cs, g = self.cs, self.gyz
        for c in range(self.cx_lo, self.cx_hi):
            out[c] = int(cs[(c + 1) * g]) - int(cs[c * g])
        return out

    def recut(self, cut):
        self.cx_lo, self.cx_hi = cut
        self.has_left = self.cx_lo > 0
        self.has_right = self.cx_hi < self.G[0]

    def read_owned(self):
        s = slice(self.o0, self.o1)
        rec = np.zeros((self.o1 - self.o0, 8), np.float32)
        rec[:, 0:3] = self.pos[s]
        rec[:, 3:6] = self.vel[s]
        rec[:, 6] = self.id[s].view(np.float32)
        rec[:, 7] = self.rp[s, 0]
        return rec

    def reset_stats(self):
        pass

    def kernel_stats(self):
        return {}

    def close(self):
        pass
