"""Multi-GPU slab decomposition of the Model S step (SPEC_SPH.md §3).

There is one process per GPU. Rank r owns the global cell columns [cx_lo, cx_hi) of the
x-slowest grid and holds one halo column on each side. Particles move between ranks, and
halos are exchanged, over `torch.distributed` point-to-point ops. With the "nccl" backend
that is RCCL over xGMI, ordered on the same HIP stream as libsphhip's kernels. Per step:

  1. count_sends / pack_send: owned particles now in column <= cx_lo go left, those in
     column >= cx_hi-1 go right (ballot/scan compaction, order preserved) — one exchange
     carries both the migrants and the position/velocity halo. The counts stay on the device
     until one host read of all four (sent and received);
  2. assemble: [from left | own | from right] -> keys -> radix sort -> cell start; the slot
     ranges are copied back asynchronously;
  3. density on the owned slots (range read on the device), then the ranges on the host;
  4. ρ, P/ρ² of the two boundary columns -> neighbours' ghost columns, in flight while the
     interior columns' force pass runs; then the boundary columns' force pass;
  5. finish_step.

The backend is libsphhip.so (GpuSlabBackend). The tests drive the same SlabRunner with a CPU
backend over gloo to check the decomposition against the single-domain oracle.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from typing import List, Optional, Tuple

import numpy as np

from . import _abi as A
from .context import Context, make_scenario, scenario_params

REC_FLOATS = A.SPH_SLAB_RECORD_BYTES // 4     # 8 floats per particle record


def weak_scenario(config: str, world: int, dx: float = 0.01, seed: int = 1234) -> A.SphScenario:
    """Weak-scaling scenario: `config`'s fluid column and tank stretched ×world along x
    (the slab axis), so every rank owns the same number of particles as one C-config GPU."""
    from .controllers import CONFIGS
    kind, dim, nx, ny, nz, tx, ty, tz = CONFIGS[config]
    return make_scenario(kind, dim, nx * world, ny, nz, tx * world, ty, tz, dx=dx, seed=seed)


def global_columns(params: A.SphParams) -> int:
    """Cell columns of the global grid along x (cells 2h, SPEC_SPH.md §0)."""
    cell = np.float32(2.0) * np.float32(params.h)
    return int(np.floor(np.float32(params.box[0]) / cell)) + 1


def balanced_cuts(sc: A.SphScenario, params: A.SphParams, world: int) -> List[Tuple[int, int]]:
    """Column cuts with equal initial particle counts (the lattice is uniform in y and z, so
    counts per column come from the x lattice index alone; jitter is ignored, cuts only need
    to be identical on every rank)."""
    cell = np.float32(2.0) * np.float32(params.h)
    inv = np.float32(1.0) / cell
    G = global_columns(params)
    x = (np.arange(sc.nx, dtype=np.float32) + np.float32(0.5)) * np.float32(sc.dx)
    col = np.clip(np.floor(x * inv).astype(np.int64), 0, G - 1)
    per_col = np.bincount(col, minlength=G).astype(np.float64)
    cum = np.cumsum(per_col)
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, total * r / world, side="left")) + 1
        c = max(c, cuts[-1] + 1)
        c = min(c, G - (world - r))
        cuts.append(c)
    cuts.append(G)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def column_counts(sc: A.SphScenario, params: A.SphParams) -> np.ndarray:
    """Initial particles per global column (lattice, jitter ignored)."""
    cell = np.float32(2.0) * np.float32(params.h)
    inv = np.float32(1.0) / cell
    G = global_columns(params)
    x = (np.arange(sc.nx, dtype=np.float32) + np.float32(0.5)) * np.float32(sc.dx)
    col = np.clip(np.floor(x * inv).astype(np.int64), 0, G - 1)
    per_x = sc.ny * (sc.nz if sc.dim == 3 else 1)
    return np.bincount(col, minlength=G).astype(np.int64) * per_x


def rebalance_cuts(cuts: List[Tuple[int, int]], hist: np.ndarray, max_move: int = 1,
                   min_width: int = 2) -> List[Tuple[int, int]]:
    """New cuts from the global per-column particle histogram: every inner
    cut moves toward the equal-count position by at most max_move columns, and a move is dropped
    when it would leave a slab narrower than min_width. With max_move = 1 every particle changes
    owner only between neighbouring ranks, which the step's exchange already handles. A pure
    function of its inputs, so every rank computes the same cuts."""
    world = len(cuts)
    b = [c[0] for c in cuts] + [cuts[-1][1]]
    cum = np.cumsum(np.asarray(hist, dtype=np.float64))
    total = cum[-1] if len(cum) else 0.0
    nb = list(b)
    if total > 0:
        for r in range(1, world):
            ideal = int(np.searchsorted(cum, total * r / world, side="left")) + 1
            nb[r] = b[r] + max(-max_move, min(max_move, ideal - b[r]))
    changed = True
    while changed:                       # drop moves that squeeze a slab (terminates: moves only revert)
        changed = False
        for r in range(1, world):
            if nb[r] != b[r] and (nb[r] - nb[r - 1] < min_width or nb[r + 1] - nb[r] < min_width):
                nb[r] = b[r]
                changed = True
    return [(nb[r], nb[r + 1]) for r in range(world)]


class GpuSlabBackend:
    """One rank's libsphhip.so context in slab mode."""

    def __init__(self, sc: A.SphScenario, params: A.SphParams, cut: Tuple[int, int], capacity: int,
                 device: int = 0, profile: bool = False):
        import torch
        self.torch = torch
        self.device = torch.device("cuda", device)
        self.ctx = Context(A.SPH_MODEL_WCSPH, sc.dim, capacity, device=device, profile=profile)
        # the counts, records and ρ halos the library writes are handed to torch p2p / .cpu(): the library
        # and torch share one stream by default (torch's current one; a new one if that is the legacy
        # null stream, which sph_set_stream cannot name). SlabRunner.step runs on it; bind_stream rebinds.
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream == 0:
            cur = torch.cuda.Stream(self.device)
        self.stream = cur
        self.ctx.set_stream(cur.cuda_stream)
        self.ctx.set_params(params)
        L, h = self.ctx._L, self.ctx.handle
        A.check("sph_slab_set", L.sph_slab_set(h, C.byref(A.SphSlab(cut[0], cut[1]))), h)
        A.check("sph_slab_init_scenario", L.sph_slab_init_scenario(h, C.byref(sc)), h)
        self._L, self._h = L, h

    def _chk(self, fn, st):
        A.check(fn, st, self._h)

    def bind_stream(self, handle: int) -> None:
        self.ctx.set_stream(handle)
        self.stream = self.torch.cuda.ExternalStream(handle, device=self.device)

    def empty(self, n: int, width: int):
        return self.torch.empty((max(n, 1), width), dtype=self.torch.float32, device=self.device)

    def count_sends(self) -> Tuple[int, int]:
        c = (C.c_int32 * 2)()
        self._chk("sph_slab_count_sends", self._L.sph_slab_count_sends(self._h, c))
        return int(c[0]), int(c[1])

    def count_sends_into(self, counts) -> None:
        """(left, right) send counts into a device int64[2] tensor, without a host sync."""
        self._chk("sph_slab_count_sends_async",
                  self._L.sph_slab_count_sends_async(self._h, A.ptr(counts.data_ptr())))

    def send_capacity(self) -> int:
        c = C.c_int32()
        self._chk("sph_slab_send_capacity", self._L.sph_slab_send_capacity(self._h, C.byref(c)))
        return int(c.value)

    def pack_send(self, side: int, buf, capacity: int) -> None:
        self._chk("sph_slab_pack_send", self._L.sph_slab_pack_send(self._h, side, A.ptr(buf.data_ptr()), capacity))

    def assemble(self, left, nl: int, right, nr: int) -> None:
        self._chk("sph_slab_assemble", self._L.sph_slab_assemble(self._h, A.ptr(left.data_ptr() if nl else 0), nl,
                                                                 A.ptr(right.data_ptr() if nr else 0), nr))

    def ranges(self) -> List[int]:
        r = (C.c_int32 * 10)()
        self._chk("sph_slab_ranges", self._L.sph_slab_ranges(self._h, r))
        return list(r)

    def density(self) -> None:
        self._chk("sph_slab_density", self._L.sph_slab_density(self._h))

    def pack_rho(self, side: int, buf, n: int) -> None:
        self._chk("sph_slab_pack_rho", self._L.sph_slab_pack_rho(self._h, side, A.ptr(buf.data_ptr()), n))

    def unpack_rho(self, side: int, buf, n: int) -> None:
        self._chk("sph_slab_unpack_rho", self._L.sph_slab_unpack_rho(self._h, side, A.ptr(buf.data_ptr() if n else 0), n))

    def force(self, dt: float, part: int) -> None:
        self._chk("sph_slab_force", self._L.sph_slab_force(self._h, dt, part))

    def finish(self, dt: float) -> None:
        self._chk("sph_slab_finish_step", self._L.sph_slab_finish_step(self._h, dt))

    def column_counts(self, ncols: int) -> np.ndarray:
        """Owned particles per global column (zero outside the owned columns)."""
        out = np.zeros(ncols, np.int64)
        self._chk("sph_slab_column_counts", self._L.sph_slab_column_counts(self._h, A.ptr(out), ncols))
        return out

    def recut(self, cut: Tuple[int, int]) -> None:
        self._chk("sph_slab_recut", self._L.sph_slab_recut(self._h, C.byref(A.SphSlab(cut[0], cut[1]))))

    def read_owned(self) -> np.ndarray:
        """(n, 8) records: x, y, z, u, v, w, id (as int32 bits), ρ."""
        cap = self.ctx.capacity
        out = np.empty((cap, 8), np.float32)
        n = C.c_int32()
        self._chk("sph_slab_read_owned", self._L.sph_slab_read_owned(self._h, A.ptr(out), cap, C.byref(n)))
        return out[: n.value].copy()

    def kernel_stats(self) -> dict:
        return self.ctx.kernel_stats()

    def reset_stats(self) -> None:
        self.ctx.reset_kernel_stats()

    def close(self) -> None:
        self.ctx.close()


class _StagedWork:
    """gloo transport of device tensors through host copies (one-GPU test boxes)."""

    def __init__(self, dist, sends, recvs):
        self.recvs = recvs
        self.host = [t.new_empty(t.shape, device="cpu") for t, _ in recvs]
        ops = [dist.P2POp(dist.isend, t.cpu(), p) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, h, p) for h, (_, p) in zip(self.host, recvs)]
        self.works = dist.batch_isend_irecv(ops)

    def wait(self):
        for w in self.works:
            w.wait()
        for h, (t, _) in zip(self.host, self.recvs):
            t.copy_(h)


class SlabRunner:
    """Drives one rank's backend through the decomposed step (see module doc)."""

    def __init__(self, config: str, rank: int, world: int, device: int = 0, profile: bool = False,
                 backend=None, scenario: Optional[A.SphScenario] = None, capacity_factor: float = 1.5,
                 cuts: Optional[List[Tuple[int, int]]] = None, rebalance_every: int = 0):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.config, self.rank, self.world = config, rank, world
        self.scenario = scenario if scenario is not None else weak_scenario(config, world)
        self.params, self.dt = scenario_params(self.scenario)
        self.cuts = [tuple(c) for c in cuts] if cuts is not None else balanced_cuts(self.scenario, self.params, world)
        self.rebalance_every = rebalance_every
        self.steps_done = 0
        self.rebalances = 0
        sc = self.scenario
        self.n_global = sc.nx * sc.ny * (sc.nz if sc.dim == 3 else 1)
        if backend is None:
            # room for the larger of an even share and this rank's initial share, plus a halo
            # column on each side, times capacity_factor (re-balancing only moves toward even)
            per_col = column_counts(sc, self.params)
            lo, hi = self.cuts[rank]
            share = max(self.n_global / world, float(per_col[lo:hi].sum()))
            cap = int((share + 2 * float(per_col.max())) * capacity_factor) + 4096
            backend = GpuSlabBackend(sc, self.params, self.cuts[rank], cap, device=device, profile=profile)
        elif callable(backend) and not hasattr(backend, "count_sends"):
            backend = backend(self.cuts[rank])          # factory: cut -> backend
        self.be = backend
        # gloo moves CPU tensors only: stage device buffers through the host (tests on one GPU)
        probe = self.be.empty(1, 1)
        self.host_staging = probe.is_cuda and dist.is_initialized() and dist.get_backend() == "gloo"
        self.left = rank - 1 if rank > 0 else None
        self.right = rank + 1 if rank + 1 < world else None
        self.ranges = None
        self._owned = None
        dev = probe.device
        # [sent left, sent right, received from left, received from right]
        self._cnt_all = torch.zeros(4, dtype=torch.int64, device=dev)
        self._cnt_out, self._cnt_in = self._cnt_all[0:2], self._cnt_all[2:4]
        self._bufs = {}

    # ----------------------------------------------------------------- plumbing
    def bind_stream(self, handle: int) -> None:
        self.be.bind_stream(handle)

    def _p2p(self, sends, recvs):
        """sends/recvs: lists of (tensor, peer). Returns the works (async)."""
        if self.host_staging:
            return [_StagedWork(self.dist, sends, recvs)] if (sends or recvs) else []
        ops = [self.dist.P2POp(self.dist.isend, t, p) for t, p in sends]
        ops += [self.dist.P2POp(self.dist.irecv, t, p) for t, p in recvs]
        return self.dist.batch_isend_irecv(ops) if ops else []

    def _exchange_counts(self, nl: int, nr: int) -> Tuple[int, int]:
        dev = self.be.empty(1, 1).device
        sends, recvs = [], []
        out_l = self.torch.zeros(1, dtype=self.torch.int64, device=dev)
        out_r = self.torch.zeros(1, dtype=self.torch.int64, device=dev)
        if self.left is not None:
            sends.append((self.torch.tensor([nl], dtype=self.torch.int64, device=dev), self.left))
            recvs.append((out_l, self.left))
        if self.right is not None:
            sends.append((self.torch.tensor([nr], dtype=self.torch.int64, device=dev), self.right))
            recvs.append((out_r, self.right))
        for w in self._p2p(sends, recvs):
            w.wait()
        return int(out_l.item()), int(out_r.item())

    # ----------------------------------------------------------------- step
    def step(self, k: int = 1) -> None:
        stream = getattr(self.be, "stream", None)   # torch work of the step on the library's stream
        with self.torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
            for _ in range(k):
                if self.rebalance_every and self.steps_done and self.steps_done % self.rebalance_every == 0:
                    self._rebalance()
                self._one_step()
                self.steps_done += 1

    def _rebalance(self) -> None:
        """All-reduce the per-column owned counts, move the cuts (identically on every rank), and
        re-window this rank's context; the next exchange moves the particles that changed owner."""
        hist = self.be.column_counts(global_columns(self.params))
        if self.world > 1 and self.dist.is_initialized():
            on_cpu = self.dist.get_backend() == "gloo"
            t = self.torch.from_numpy(hist)
            if not on_cpu:
                t = t.to(self.be.empty(1, 1).device)
            self.dist.all_reduce(t)
            hist = t.cpu().numpy()
        new = rebalance_cuts(self.cuts, hist)
        if new != self.cuts:
            self.cuts = new
            self.be.recut(new[self.rank])
            self.rebalances += 1

    def _buf(self, name: str, n: int, width: int):
        """Persistent device buffer of at least n rows (grown by 1/8 when too small)."""
        b = self._bufs.get(name)
        if b is None or b.shape[0] < n:
            b = self.be.empty(max(n + n // 8, 1), width)
            self._bufs[name] = b
        return b

    def _one_step(self) -> None:
        be, dt = self.be, self.dt
        # 1. migrants + x,v halo in one exchange. The send counts stay on the device: the packs go
        #    to capacity-sized buffers, the counts go to the neighbours as device tensors, and the
        #    host reads all four counts once.
        be.count_sends_into(self._cnt_out)
        cap = be.send_capacity()
        bl, br = self._buf("send_l", cap, REC_FLOATS), self._buf("send_r", cap, REC_FLOATS)
        if self.left is not None:
            be.pack_send(0, bl, bl.shape[0])
        if self.right is not None:
            be.pack_send(1, br, br.shape[0])
        sends, recvs = [], []
        if self.left is not None:
            sends.append((self._cnt_out[0:1], self.left))
            recvs.append((self._cnt_in[0:1], self.left))
        if self.right is not None:
            sends.append((self._cnt_out[1:2], self.right))
            recvs.append((self._cnt_in[1:2], self.right))
        for w in self._p2p(sends, recvs):
            w.wait()
        nl, nr, il, ir = (int(v) for v in self._cnt_all.cpu().tolist())   # one copy-back, one sync
        if self.left is None:
            nl = il = 0
        if self.right is None:
            nr = ir = 0
        rl, rr = self._buf("recv_l", il, REC_FLOATS), self._buf("recv_r", ir, REC_FLOATS)
        sends = [(bl[:nl], self.left)] if nl else []
        sends += [(br[:nr], self.right)] if nr else []
        recvs = [(rl[:il], self.left)] if il else []
        recvs += [(rr[:ir], self.right)] if ir else []
        for w in self._p2p(sends, recvs):
            w.wait()
        # 2. rebuild + sort; 3. density (reads its slot range on the device), then the ranges
        #    (their copy-back completes while density runs)
        be.assemble(rl, il, rr, ir)
        be.density()
        r = be.ranges()
        self.ranges = r
        # 4. ρ halo: boundary columns out, ghost columns in; interior force meanwhile
        nbl, nbr = r[7] - r[6], r[9] - r[8]
        ngl, ngr = r[1] - r[0], r[5] - r[4]
        sends, recvs = [], []
        if self.left is not None and nbl:
            sl = self._buf("rho_sl", nbl, 2)
            be.pack_rho(0, sl, nbl)
            sends.append((sl[:nbl], self.left))
        if self.right is not None and nbr:
            sr = self._buf("rho_sr", nbr, 2)
            be.pack_rho(1, sr, nbr)
            sends.append((sr[:nbr], self.right))
        gl, gr = self._buf("rho_gl", ngl, 2), self._buf("rho_gr", ngr, 2)
        if ngl:
            recvs.append((gl[:ngl], self.left))
        if ngr:
            recvs.append((gr[:ngr], self.right))
        works = self._p2p(sends, recvs)
        be.force(dt, 1)
        for w in works:
            w.wait()
        be.unpack_rho(0, gl, ngl)
        be.unpack_rho(1, gr, ngr)
        be.force(dt, 2)
        be.finish(dt)

    # ----------------------------------------------------------------- reporting
    def total_particles(self) -> int:
        return self.n_global

    def local_particles(self) -> int:
        if self.ranges is None:
            return self.n_global // self.world
        return self.ranges[3] - self.ranges[2]

    def owned(self) -> np.ndarray:
        return self.be.read_owned()

    def grid_stats(self) -> dict:
        """This rank's slab grid (bench.py's whole-step roofline: key bits and cells)."""
        st = self.be.ctx.stats()
        return {"key_bits": st.key_bits, "ncells": st.grid[0] * st.grid[1] * st.grid[2]}

    def reset_stats(self) -> None:
        self.be.reset_stats()

    def kernel_stats(self) -> dict:
        return self.be.kernel_stats()

    def workload(self, scaling: str = "weak") -> str:
        sc = self.scenario
        kind = "sloshing" if sc.kind == A.SPH_SCENARIO_SLOSHING else "dam-break"
        name = f"{self.config}x{self.world} weak" if scaling == "weak" else f"{self.config} on {self.world} GPUs"
        return (f"{name}: {self.n_global} particles, {sc.dim}D {kind}, column "
                f"{sc.nx}x{sc.ny}x{sc.nz}, tank {sc.tx}x{sc.ty}x{sc.tz} dx, x-slabs {self.cuts}")

    def close(self) -> None:
        self.be.close()
