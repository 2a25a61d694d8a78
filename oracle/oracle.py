"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module. The product path (sph-test_amd/) never does.

Model R restates /root/reference/Assets/Compute/SimulateParticles.compute:102-408;
Model S restates SPEC_SPH.md §2. PARITY UNPINNED by reference fixtures (the reference
ships none and cannot run here): see oracle/oracle.h and DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "liboracle.so"

# SimulateParticles.compute:23-40 (84 bytes, field order kept)
PARTICLE84 = np.dtype([
    ("position", "<f4", (3,)), ("radius", "<f4"),
    ("velocity", "<f4", (3,)), ("mass", "<f4"),
    ("angularVelocity", "<f4", (3,)), ("momentOfInertia", "<f4"),
    ("drag", "<f4"), ("repulsionStrength", "<f4"), ("padding1", "<f4"), ("padding2", "<f4"),
    ("rotation", "<f4", (4,)), ("modeIndex", "<i4"),
])
assert PARTICLE84.itemsize == 84

# SimulateParticles.compute:43-55 (84 bytes, field order kept)
ADHESION84 = np.dtype([
    ("particleA", "<i4"), ("particleB", "<i4"), ("restLength", "<f4"), ("springStiffness", "<f4"),
    ("springDamping", "<f4"), ("connectionColor", "<f4", (4,)), ("initialRelOrientation", "<f4", (4,)),
    ("anchorLocalPosA", "<f4", (3,)), ("anchorLocalPosB", "<f4", (3,)),
    ("anchorConstraintStiffness", "<f4"), ("enableAnchorConstraint", "<i4"),
])
assert ADHESION84.itemsize == 84


class OrGrid(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("inv_cell", C.c_float), ("inv_cell_z", C.c_float),
                ("G", C.c_int32 * 3), ("zwin", C.c_int32), ("xsub", C.c_int32), ("inv_cxs", C.c_float)]


class OrSphParams(C.Structure):
    _fields_ = [
        ("dim", C.c_int32), ("dx", C.c_float), ("h", C.c_float), ("rho0", C.c_float),
        ("c0", C.c_float), ("alpha", C.c_float), ("eps_xsph", C.c_float),
        ("g", C.c_float * 3), ("L", C.c_float * 3), ("wall_e", C.c_float),
        ("f_amp", C.c_float), ("f_freq", C.c_float),
        ("mass", C.c_float), ("B", C.c_float), ("sigma", C.c_float), ("inv_h", C.c_float),
        ("four_h2", C.c_float), ("grid", OrGrid),
    ]


class OrContactParams(C.Structure):
    _fields_ = [
        ("dt", C.c_float), ("spawn_radius", C.c_float), ("global_drag", C.c_float),
        ("torque_factor", C.c_float), ("torque_damping", C.c_float),
        ("boundary_friction", C.c_float), ("roll_mult", C.c_float),
        ("repulsion_strength", C.c_float), ("drag_id", C.c_int32),
        ("drag_target", C.c_float * 3), ("drag_strength", C.c_float),
    ]


def build() -> Path:
    """Compile the oracle with its own Makefile (gcc; no GPU)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = C.CDLL(str(_LIB_PATH))
        P = C.POINTER
        L.or_sph_derive.argtypes = [P(OrSphParams)]
        L.or_sph_step.argtypes = [P(OrSphParams), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_sph_step_diag.argtypes = [P(OrSphParams), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int]
        L.or_sph_force_range_diag.argtypes = [P(OrSphParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_float,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_sph_lattice.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                     C.c_float, C.c_float, C.c_uint32, C.c_float, C.c_void_p]
        L.or_contact_step.argtypes = [P(OrContactParams), C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.or_contact_step_bonds.argtypes = [P(OrContactParams), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_int, C.c_void_p, C.c_int]
        L.or_init_particles.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int,
                                        C.c_int, C.c_void_p]
        L.or_split_particles.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        L.or_split_particles.restype = C.c_int
        L.or_stable_sort.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p]
        L.or_cell_start.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p]
        L.or_keys.argtypes = [P(OrGrid), C.c_int, C.c_void_p, C.c_void_p]
        L.or_sph_density_range.argtypes = [P(OrSphParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_int]
        L.or_sph_force_range.argtypes = [P(OrSphParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_float,
                                         C.c_void_p, C.c_void_p, C.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------- Model S
def sph_params(dim, dx, h, rho0, c0, alpha, eps_xsph, g, L, wall_e, f_amp=0.0, f_freq=0.0):
    p = OrSphParams()
    p.dim, p.dx, p.h, p.rho0, p.c0 = dim, dx, h, rho0, c0
    p.alpha, p.eps_xsph, p.wall_e, p.f_amp, p.f_freq = alpha, eps_xsph, wall_e, f_amp, f_freq
    for a in range(3):
        p.g[a] = g[a]
        p.L[a] = L[a]
    lib().or_sph_derive(C.byref(p))
    return p


def ncells(p: OrSphParams) -> int:
    return int(p.grid.G[0]) * int(p.grid.xsub) * int(p.grid.G[1]) * int(p.grid.G[2])


def sph_step(p: OrSphParams, pos, vel, ids, dt, t=0.0, nthreads=0):
    """One Model S step. Returns (pos, vel, ids, rho, prho, cell_start) in sorted order."""
    pos = np.ascontiguousarray(pos, dtype=np.float32).copy()
    vel = np.ascontiguousarray(vel, dtype=np.float32).copy()
    ids = np.ascontiguousarray(ids, dtype=np.int32).copy()
    n = pos.shape[0]
    rho = np.empty(n, np.float32)
    prho = np.empty(n, np.float32)
    cs = np.empty(ncells(p) + 1, np.uint32)
    lib().or_sph_step(C.byref(p), n, _ptr(pos), _ptr(vel), _ptr(ids), dt, t, _ptr(rho), _ptr(prho),
                      _ptr(cs), nthreads)
    return pos, vel, ids, rho, prho, cs


def sph_step_diag(p: OrSphParams, pos, vel, ids, dt, t=0.0, nthreads=0):
    """sph_step plus, in the same sorted order, acc (n,3): the pair sum a_i without gravity or
    forcing, and mag (n,5): Σ|pair acceleration term|, Σ|pair XSPH term|, the EOS sensitivity and the
    two support-edge conditioning terms (error scales, oracle.h or_sph_step_diag).
    Returns (pos, vel, ids, rho, prho, cell_start, acc, mag)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32).copy()
    vel = np.ascontiguousarray(vel, dtype=np.float32).copy()
    ids = np.ascontiguousarray(ids, dtype=np.int32).copy()
    n = pos.shape[0]
    rho = np.empty(n, np.float32)
    prho = np.empty(n, np.float32)
    cs = np.empty(ncells(p) + 1, np.uint32)
    acc = np.empty((n, 3), np.float32)
    mag = np.empty((n, 5), np.float32)
    lib().or_sph_step_diag(C.byref(p), n, _ptr(pos), _ptr(vel), _ptr(ids), dt, t, _ptr(rho), _ptr(prho),
                           _ptr(cs), _ptr(acc), _ptr(mag), nthreads)
    return pos, vel, ids, rho, prho, cs, acc, mag


def force_range_diag(p: OrSphParams, pos, vel, rho, prho, sk, cs, dt, t=0.0, nthreads=0):
    """Pass 2 + integrate over ALL sorted slots of (pos, vel) with the given (rho, prho) (e.g. the
    GPU's pass-1 output): returns (pos_out, vel_out, acc, mag) in the same sorted order."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    vel = np.ascontiguousarray(vel, dtype=np.float32)
    rho = np.ascontiguousarray(rho, dtype=np.float32)
    prho = np.ascontiguousarray(prho, dtype=np.float32)
    sk = np.ascontiguousarray(sk, dtype=np.uint32)
    cs = np.ascontiguousarray(cs, dtype=np.uint32)
    n = pos.shape[0]
    po, vo = np.empty_like(pos), np.empty_like(vel)
    acc = np.empty((n, 3), np.float32)
    mag = np.empty((n, 5), np.float32)
    lib().or_sph_force_range_diag(C.byref(p), _ptr(pos), _ptr(vel), _ptr(rho), _ptr(prho), _ptr(sk), _ptr(cs), 0, n,
                                  dt, t, _ptr(po), _ptr(vo), _ptr(acc), _ptr(mag), nthreads)
    return po, vo, acc, mag


def density_range(p: OrSphParams, pos, sk, cs, i0, i1, rho, prho, nthreads=0):
    """Pass 1 for sorted targets [i0, i1) (in place into rho/prho)."""
    lib().or_sph_density_range(C.byref(p), _ptr(pos), _ptr(sk), _ptr(cs), i0, i1, _ptr(rho), _ptr(prho), nthreads)


def force_range(p: OrSphParams, pos, vel, rho, prho, sk, cs, i0, i1, dt, t, pos_out, vel_out, nthreads=0):
    """Pass 2 + integrate for sorted targets [i0, i1) (in place into pos_out/vel_out)."""
    lib().or_sph_force_range(C.byref(p), _ptr(pos), _ptr(vel), _ptr(rho), _ptr(prho), _ptr(sk), _ptr(cs), i0, i1,
                             dt, t, _ptr(pos_out), _ptr(vel_out), nthreads)


def lattice(dim, nx, ny, nz, dx, origin=(0.0, 0.0, 0.0), seed=1234, jitter_frac=0.01):
    """Dam-break lattice; jitter amplitude = jitter_frac·dx as ONE fp32 product (as the library)."""
    jitter = float(np.float32(jitter_frac) * np.float32(dx))
    n = nx * ny * (nz if dim == 3 else 1)
    out = np.empty((n, 3), np.float32)
    lib().or_sph_lattice(dim, nx, ny, nz, dx, origin[0], origin[1], origin[2], seed, jitter, _ptr(out))
    return out


def grid_keys(p: OrSphParams, pos):
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    keys = np.empty(pos.shape[0], np.uint32)
    lib().or_keys(C.byref(p.grid), pos.shape[0], _ptr(pos), _ptr(keys))
    return keys


def stable_sort(keys, nkeys):
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.empty(keys.shape[0], np.uint32)
    lib().or_stable_sort(keys.shape[0], _ptr(keys), nkeys, _ptr(perm))
    return perm


def cell_start(sorted_keys, nkeys):
    sk = np.ascontiguousarray(sorted_keys, dtype=np.uint32)
    cs = np.empty(nkeys + 1, np.uint32)
    lib().or_cell_start(sk.shape[0], _ptr(sk), nkeys, _ptr(cs))
    return cs


# ---------------------------------------------------------------- Model R
def contact_params(dt, spawn_radius=15.0, global_drag=1.0, torque_factor=1.0, torque_damping=0.5,
                   boundary_friction=0.8, roll_mult=5.0, repulsion_strength=200.0,
                   drag_id=-1, drag_target=(0.0, 0.0, 0.0), drag_strength=0.0):
    p = OrContactParams()
    p.dt, p.spawn_radius, p.global_drag, p.torque_factor = dt, spawn_radius, global_drag, torque_factor
    p.torque_damping, p.boundary_friction, p.roll_mult = torque_damping, boundary_friction, roll_mult
    p.repulsion_strength, p.drag_id, p.drag_strength = repulsion_strength, drag_id, drag_strength
    for a in range(3):
        p.drag_target[a] = drag_target[a]
    return p


def contact_step(p: OrContactParams, parts, nthreads=0):
    """One Model R step on an AoS-84 structured array. Returns (parts, torque_int[n,3])."""
    parts = np.ascontiguousarray(parts, dtype=PARTICLE84).copy()
    n = parts.shape[0]
    tq = np.empty((n, 3), np.int32)
    lib().or_contact_step(C.byref(p), n, _ptr(parts), _ptr(tq), nthreads)
    return parts, tq


def contact_step_bonds(p: OrContactParams, parts, conns, nthreads=0):
    """One Model R step with adhesion bonds (AoS-84 particles, AoS-84 connections).
    Returns (parts, torque_int[n,3], terms[nconn,16])."""
    parts = np.ascontiguousarray(parts, dtype=PARTICLE84).copy()
    conns = np.ascontiguousarray(conns, dtype=ADHESION84)
    n, m = parts.shape[0], conns.shape[0]
    tq = np.empty((n, 3), np.int32)
    terms = np.zeros((max(m, 1), 16), np.int32)
    lib().or_contact_step_bonds(C.byref(p), n, _ptr(parts), _ptr(tq), _ptr(conns), m, _ptr(terms), nthreads)
    return parts, tq, terms[:m]


def init_particles(n, active, spawn_radius=15.0, min_radius=1.5, max_radius=2.0, density=0.1, genome_modes=0,
                   default_mode=0):
    """InitParticles (compute:118-194) for a buffer of n particles, the first `active` initialised."""
    out = np.zeros(max(n, 1), PARTICLE84)
    lib().or_init_particles(n, active, spawn_radius, min_radius, max_radius, density, genome_modes, default_mode,
                            _ptr(out))
    return out[:n]


# CellSplitData (ParticleSystemController.cs:136-147), 92 bytes
SPLIT92 = np.dtype([
    ("parentIndex", "<i4"), ("positionA", "<f4", (3,)), ("positionB", "<f4", (3,)),
    ("velocityA", "<f4", (3,)), ("velocityB", "<f4", (3,)), ("rotationA", "<f4", (4,)),
    ("rotationB", "<f4", (4,)), ("childAModeIndex", "<i4"), ("childBModeIndex", "<i4"),
])


def split_particles(parts, active, splits):
    """ProcessPendingSplits' buffer edit on a copy of `parts` (grown with zero records when needed).
    Returns (parts, new_active)."""
    splits = np.ascontiguousarray(splits, dtype=SPLIT92)
    need = active + len(splits)
    out = np.zeros(max(len(parts), need), PARTICLE84)
    out[: len(parts)] = parts
    new_active = lib().or_split_particles(_ptr(out), active, _ptr(splits), len(splits))
    return out, new_active


def default_threads() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
