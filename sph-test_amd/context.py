"""`Context`: one libsphhip.so context (one GPU), the object the controllers drive."""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _abi as A


class Context:
    """A device context: particle buffers, grid, stream (include/sphhip.h)."""

    def __init__(self, model: int, dim: int, capacity: int, device: int = 0, profile: bool = False, ndev: int = 1,
                 validate: bool = False):
        self._L = A.lib()
        flags = (A.SPH_FLAG_PROFILE if profile else 0) | (A.SPH_FLAG_VALIDATE if validate else 0)
        cfg = A.SphConfig(model, dim, capacity, flags, ndev)
        h = C.c_void_p()
        st = self._L.sph_create(C.byref(cfg), device, C.byref(h))
        if st != A.SPH_OK:
            raise A.SphError("sph_create", st, f"model={model} dim={dim} capacity={capacity} device={device}")
        self._h = h
        self.model, self.dim, self.capacity, self.device, self.ndev = model, dim, capacity, device, ndev
        self.n = 0
        self.nbonds = 0

    # -------------------------------------------------------------- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.sph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, fn: str, st: int) -> None:
        A.check(fn, st, self._h)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -------------------------------------------------------------- config
    def resize(self, capacity: int) -> None:
        self._chk("sph_resize", self._L.sph_resize(self._h, capacity))
        self.capacity = capacity

    def set_stream(self, stream_handle: Optional[int]) -> None:
        self._chk("sph_set_stream", self._L.sph_set_stream(self._h, C.c_void_p(stream_handle or 0)))

    def stream(self) -> int:
        s = C.c_void_p()
        self._chk("sph_get_stream", self._L.sph_get_stream(self._h, C.byref(s)))
        return int(s.value or 0)

    # -------------------------------------------------------------- multi-GPU (sphhip.h: the decomposed step)
    def comm_init(self, comm_id: bytes, nranks: int, rank: int) -> None:
        """Join an RCCL communicator (one process per GPU): rank `rank` of `nranks`."""
        cid = A.SphCommId()
        C.memmove(C.byref(cid), comm_id, 128)
        self._chk("sph_comm_init", self._L.sph_comm_init(self._h, C.byref(cid), nranks, rank))

    def set_rebalance(self, every: int) -> None:
        self._chk("sph_set_rebalance", self._L.sph_set_rebalance(self._h, every))

    def decomposition(self) -> A.SphDecomp:
        d = A.SphDecomp()
        self._chk("sph_get_decomposition", self._L.sph_get_decomposition(self._h, C.byref(d)))
        return d

    def set_params(self, params: A.SphParams) -> None:
        self._chk("sph_set_params", self._L.sph_set_params(self._h, C.byref(params)))

    def get_params(self) -> A.SphParams:
        p = A.SphParams()
        self._chk("sph_get_params", self._L.sph_get_params(self._h, C.byref(p)))
        return p

    # -------------------------------------------------------------- data
    def upload_aos84(self, parts: np.ndarray) -> None:
        parts = np.ascontiguousarray(parts, dtype=A.PARTICLE84)
        self._chk("sph_upload_particles_aos84", self._L.sph_upload_particles_aos84(self._h, A.ptr(parts), len(parts)))
        self.n = len(parts)

    def download_aos84(self) -> np.ndarray:
        out = np.zeros(self.n, A.PARTICLE84)
        self._chk("sph_download_particles_aos84", self._L.sph_download_particles_aos84(self._h, A.ptr(out), self.n))
        return out

    def upload_state(self, pos: np.ndarray, vel: Optional[np.ndarray] = None) -> None:
        pos = np.ascontiguousarray(pos, dtype=np.float32).reshape(-1, 3)
        v = None if vel is None else np.ascontiguousarray(vel, dtype=np.float32).reshape(-1, 3)
        self._chk("sph_upload_state", self._L.sph_upload_state(self._h, A.ptr(pos), A.ptr(v), len(pos)))
        self.n = len(pos)

    def init_scenario(self, sc: A.SphScenario) -> None:
        self._chk("sph_init_scenario", self._L.sph_init_scenario(self._h, C.byref(sc)))
        self.n = sc.nx * sc.ny * (sc.nz if sc.dim == 3 else 1)

    def init_particles(self, count: int, active: int, genome_modes: int = 0, default_mode: int = 0) -> None:
        """InitParticles (compute:118-194): count particles, the first `active` initialised."""
        self._chk("sph_init_particles", self._L.sph_init_particles(self._h, count, active, genome_modes, default_mode))
        self.n = count

    def split_particles(self, splits: np.ndarray) -> int:
        """Cell division's buffer edit (sph_split_particles); returns the new active count."""
        splits = np.ascontiguousarray(splits, dtype=A.SPLIT92)
        out = C.c_int32()
        self._chk("sph_split_particles", self._L.sph_split_particles(self._h, A.ptr(splits), len(splits), C.byref(out)))
        self.n = max(self.n, int(out.value))
        self.capacity = max(self.capacity, self.stats().capacity)
        return int(out.value)

    def get_particles(self, first: int, count: int) -> np.ndarray:
        """particleBuffer.GetData(array, 0, first, count) (84-byte records)."""
        out = np.zeros(max(count, 1), A.PARTICLE84)
        self._chk("sph_get_particles_aos84", self._L.sph_get_particles_aos84(self._h, first, count, A.ptr(out)))
        return out[:count]

    def set_particles(self, first: int, parts: np.ndarray) -> None:
        """particleBuffer.SetData(array, 0, first, len(array))."""
        parts = np.ascontiguousarray(parts, dtype=A.PARTICLE84)
        self._chk("sph_set_particles_aos84", self._L.sph_set_particles_aos84(self._h, first, len(parts), A.ptr(parts)))

    def step(self, dt: float, nsteps: int = 1) -> None:
        self._chk("sph_step", self._L.sph_step(self._h, dt, nsteps))

    def set_sim_time(self, t: float) -> None:
        """The simulated time the next step starts at (the sloshing forcing reads it)."""
        self._chk("sph_set_sim_time", self._L.sph_set_sim_time(self._h, float(t)))

    def set_drag(self, selected_id: int, target, strength: float) -> None:
        d = A.SphDragInput(selected_id, (C.c_float * 3)(*target), strength)
        self._chk("sph_set_drag", self._L.sph_set_drag(self._h, C.byref(d)))

    def set_adhesion(self, conns: Optional[np.ndarray]) -> None:
        """Adhesion bonds (AoS-84 AdhesionConnection records); None or empty removes them."""
        if conns is None or len(conns) == 0:
            self._chk("sph_set_adhesion", self._L.sph_set_adhesion(self._h, None, 0))
            self.nbonds = 0
            return
        conns = np.ascontiguousarray(conns, dtype=A.ADHESION84)
        self._chk("sph_set_adhesion", self._L.sph_set_adhesion(self._h, A.ptr(conns), len(conns)))
        self.nbonds = len(conns)

    def adhesion_terms(self) -> np.ndarray:
        """The last step's per-bond fixed-point terms, [nbonds, 16] int32 (include/sphhip.h)."""
        out = np.zeros((max(self.nbonds, 1), 16), np.int32)
        self._chk("sph_read_adhesion_terms", self._L.sph_read_adhesion_terms(self._h, A.ptr(out), self.nbonds))
        return out[: self.nbonds]

    # -------------------------------------------------------------- async readback / render interop
    def request_readback(self, fields: int) -> None:
        """AsyncGPUReadback.Request of SPH_READBACK_* fields of the current state."""
        self._chk("sph_request_readback", self._L.sph_request_readback(self._h, fields))

    def readback_ready(self) -> bool:
        st = self._L.sph_readback_status(self._h)
        if st == A.SPH_READBACK_PENDING:
            return False
        self._chk("sph_readback_status", st)
        return True

    def readback_get(self, field: int) -> np.ndarray:
        cnt = C.c_int32()
        self._chk("sph_readback_count", self._L.sph_readback_count(self._h, C.byref(cnt)))
        n = cnt.value
        if field == A.SPH_READBACK_PARTICLES:
            out = np.zeros(max(n, 1), A.PARTICLE84)
        else:
            out = np.zeros((max(n, 1), 3 if field == A.SPH_READBACK_POSITIONS else 4), np.float32)
        self._chk("sph_readback_get", self._L.sph_readback_get(self._h, field, A.ptr(out), max(n, 1)))
        return out[:n]

    def export_aos84_device(self, dev_ptr: int, count: int) -> None:
        """84-byte records (index order) into a device buffer, on the context stream."""
        self._chk("sph_export_aos84_device", self._L.sph_export_aos84_device(self._h, C.c_void_p(dev_ptr), count))

    def write_draw_args(self, dev_ptr: int) -> None:
        self._chk("sph_write_draw_args", self._L.sph_write_draw_args(self._h, C.c_void_p(dev_ptr)))

    def synchronize(self) -> None:
        self._chk("sph_synchronize", self._L.sph_synchronize(self._h))

    def _read(self, fn: str, comps: int, dtype=np.float32) -> np.ndarray:
        out = np.empty((self.n, comps) if comps > 1 else self.n, dtype)
        self._chk(fn, getattr(self._L, fn)(self._h, A.ptr(out), self.n))
        return out

    def positions(self) -> np.ndarray:
        return self._read("sph_read_positions", 3)

    def velocities(self) -> np.ndarray:
        return self._read("sph_read_velocities", 3)

    def rotations(self) -> np.ndarray:
        return self._read("sph_read_rotations", 4)

    def angular_velocities(self) -> np.ndarray:
        return self._read("sph_read_angular_velocities", 3)

    def density(self) -> np.ndarray:
        return self._read("sph_read_density", 1)

    def pressure_term(self) -> np.ndarray:
        """P/ρ² of the last step's pass 1 (index order)."""
        return self._read("sph_read_pressure_term", 1)

    def torque_int(self) -> np.ndarray:
        return self._read("sph_read_torque_int", 3, np.int32)

    def sorted_ids(self) -> np.ndarray:
        return self._read("sph_read_sorted_ids", 1, np.int32)

    def cell_start(self) -> np.ndarray:
        st = self.stats()
        nc = st.grid[0] * st.grid[1] * st.grid[2] + 1
        out = np.empty(nc, np.uint32)
        self._chk("sph_read_cell_start", self._L.sph_read_cell_start(self._h, A.ptr(out), nc))
        return out

    def path_counts(self, reset: bool = True) -> np.ndarray:
        """Sparse-path counters of the neighbour passes (sph_read_path_counts): density chunked,
        density global, force chunked, force global."""
        out = np.zeros(4, np.uint32)
        self._chk("sph_read_path_counts", self._L.sph_read_path_counts(self._h, A.ptr(out), 1 if reset else 0))
        return out

    def resort_counts(self, reset: bool = True) -> np.ndarray:
        """The incremental re-sort's path counters (sph_read_resort_counts): whole-list ranges, whole-list lanes,
        multi-pass ranges, their passes, the largest dest-entry count of a range, cell shares that re-streamed."""
        out = np.zeros(8, np.uint32)
        self._chk("sph_read_resort_counts", self._L.sph_read_resort_counts(self._h, A.ptr(out), 1 if reset else 0))
        return out[:6]

    def mover_count(self) -> int:
        """Particles whose cell key changed in the last step (sph_read_mover_count; Model S, single context)."""
        out = np.zeros(1, np.uint32)
        self._chk("sph_read_mover_count", self._L.sph_read_mover_count(self._h, A.ptr(out)))
        return int(out[0])

    def debug_kick(self, pid: int, dv) -> None:
        """Test hook (sph_debug_kick): add dv to particle pid's velocity, in every slab that holds it."""
        d = np.ascontiguousarray(dv, dtype=np.float32)
        self._chk("sph_debug_kick", self._L.sph_debug_kick(self._h, int(pid), A.ptr(d)))

    def hit_mask_counts(self, reset: bool = True) -> np.ndarray:
        """(wave-planes of the force pass scanned by distance instead of the hit mask, waves run)
        (sph_read_hit_mask_counts)."""
        out = np.zeros(2, np.uint32)
        self._chk("sph_read_hit_mask_counts", self._L.sph_read_hit_mask_counts(self._h, A.ptr(out), 1 if reset else 0))
        return out

    def radix_sort(self, keys: np.ndarray, key_bits: int):
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        perm = np.empty_like(keys)
        sk = np.empty_like(keys)
        self._chk("sph_debug_radix_sort",
                  self._L.sph_debug_radix_sort(self._h, A.ptr(keys), len(keys), key_bits, A.ptr(perm), A.ptr(sk)))
        return perm, sk

    # -------------------------------------------------------------- stats
    def stats(self) -> A.SphStats:
        s = A.SphStats()
        self._chk("sph_get_stats", self._L.sph_get_stats(self._h, C.byref(s)))
        return s

    def kernel_stats(self) -> dict:
        out = {}
        i = 0
        while True:
            k = A.SphKernelStat()
            if self._L.sph_get_kernel_stat(self._h, i, C.byref(k)) != A.SPH_OK:
                break
            out[k.name.decode()] = {"launches": k.launches, "total_ms": k.total_ms,
                                    "bytes_per_launch": k.bytes_per_launch, "timed": k.timed}
            i += 1
        return out

    def reset_kernel_stats(self) -> None:
        self._chk("sph_reset_kernel_stats", self._L.sph_reset_kernel_stats(self._h))

    def set_profile_every(self, every: int) -> None:
        """SPH_FLAG_PROFILE: time the launches of one step in `every` (sph_set_profile_every)."""
        self._chk("sph_set_profile_every", self._L.sph_set_profile_every(self._h, int(every)))


def scenario_params(sc: A.SphScenario):
    """SPEC_SPH.md §2 constants for a scenario (pure C call, no GPU needed)."""
    p = A.SphParams()
    dt = C.c_float()
    A.check("sph_scenario_params", A.lib().sph_scenario_params(C.byref(sc), C.byref(p), C.byref(dt)))
    return p, float(dt.value)


def comm_unique_id() -> bytes:
    """A new RCCL unique id (rank 0); the caller hands the 128 bytes to every rank."""
    cid = A.SphCommId()
    A.check("sph_comm_unique_id", A.lib().sph_comm_unique_id(C.byref(cid)))
    return C.string_at(C.byref(cid), 128)


def make_scenario(kind: int, dim: int, nx: int, ny: int, nz: int, tx: int, ty: int, tz: int,
                  dx: float = 0.01, seed: int = 1234, jitter: float = 0.01) -> A.SphScenario:
    return A.SphScenario(kind, dim, nx, ny, nz, tx, ty, tz, dx, seed, jitter)
