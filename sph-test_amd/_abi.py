"""ctypes binding of libsphhip.so (include/sphhip.h).

This is the Python counterpart of the C# P/Invoke layer shown in INTEGRATION.md. It uses
the same structs, the same entry points and the same error codes. The HIP library is the
product. There is no fallback: if libsphhip.so is missing or fails to load, every call
raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libsphhip.so"

SPH_OK = 0
SPH_ERR_INVALID = -1
SPH_ERR_HIP = -2
SPH_ERR_CAPACITY = -3
SPH_ERR_STATE = -4
SPH_ERR_NOMEM = -5
_STATUS = {0: "SPH_OK", -1: "SPH_ERR_INVALID", -2: "SPH_ERR_HIP", -3: "SPH_ERR_CAPACITY",
           -4: "SPH_ERR_STATE", -5: "SPH_ERR_NOMEM"}

SPH_MODEL_CONTACT = 0
SPH_MODEL_WCSPH = 1
SPH_FLAG_PROFILE = 1
SPH_FLAG_VALIDATE = 2
SPH_SCENARIO_DAMBREAK = 0
SPH_SCENARIO_SLOSHING = 1
SPH_SCENARIO_SPHERE = 2
SPH_READBACK_POSITIONS = 1
SPH_READBACK_ROTATIONS = 2
SPH_READBACK_PARTICLES = 4
SPH_READBACK_PENDING = 1

# SimulateParticles.compute:23-40 / ParticleSystemController.cs:157-175 (84 bytes)
PARTICLE84 = np.dtype([
    ("position", "<f4", (3,)), ("radius", "<f4"),
    ("velocity", "<f4", (3,)), ("mass", "<f4"),
    ("angularVelocity", "<f4", (3,)), ("momentOfInertia", "<f4"),
    ("drag", "<f4"), ("repulsionStrength", "<f4"), ("genomeFlags", "<u4"),
    ("orientConstraintStr", "<f4"),
    ("rotation", "<f4", (4,)), ("modeIndex", "<i4"),
])
assert PARTICLE84.itemsize == 84

# AdhesionConnection (SimulateParticles.compute:43-55; CellAdhesionManager.cs:511-524), 84 bytes
ADHESION84 = np.dtype([
    ("particleA", "<i4"), ("particleB", "<i4"), ("restLength", "<f4"), ("springStiffness", "<f4"),
    ("springDamping", "<f4"), ("connectionColor", "<f4", (4,)), ("initialRelOrientation", "<f4", (4,)),
    ("anchorLocalPosA", "<f4", (3,)), ("anchorLocalPosB", "<f4", (3,)),
    ("anchorConstraintStiffness", "<f4"), ("enableAnchorConstraint", "<i4"),
])
assert ADHESION84.itemsize == 84

# CellSplitData (ParticleSystemController.cs:136-147) == sph_split, 92 bytes
SPLIT92 = np.dtype([
    ("parentIndex", "<i4"), ("positionA", "<f4", (3,)), ("positionB", "<f4", (3,)),
    ("velocityA", "<f4", (3,)), ("velocityB", "<f4", (3,)), ("rotationA", "<f4", (4,)),
    ("rotationB", "<f4", (4,)), ("childAModeIndex", "<i4"), ("childBModeIndex", "<i4"),
])
assert SPLIT92.itemsize == 92


class SphConfig(C.Structure):
    _fields_ = [("model", C.c_int32), ("dim", C.c_int32), ("capacity", C.c_int32), ("flags", C.c_int32),
                ("ndev", C.c_int32)]


class SphParams(C.Structure):
    _fields_ = [
        ("spawn_radius", C.c_float), ("min_radius", C.c_float), ("max_radius", C.c_float),
        ("global_drag_multiplier", C.c_float), ("torque_factor", C.c_float),
        ("torque_damping", C.c_float), ("boundary_friction", C.c_float),
        ("rolling_contact_radius_multiplier", C.c_float), ("density", C.c_float),
        ("repulsion_strength", C.c_float), ("active_particle_count", C.c_int32),
        ("dx", C.c_float), ("h", C.c_float), ("rho0", C.c_float), ("c0", C.c_float),
        ("alpha", C.c_float), ("xsph_eps", C.c_float), ("gravity", C.c_float * 3),
        ("box", C.c_float * 3), ("wall_restitution", C.c_float), ("forcing_amp", C.c_float),
        ("forcing_freq", C.c_float),
    ]


class SphScenario(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dim", C.c_int32), ("nx", C.c_int32), ("ny", C.c_int32),
                ("nz", C.c_int32), ("tx", C.c_int32), ("ty", C.c_int32), ("tz", C.c_int32),
                ("dx", C.c_float), ("seed", C.c_uint32), ("jitter", C.c_float)]


class SphDragInput(C.Structure):
    _fields_ = [("selected_id", C.c_int32), ("target", C.c_float * 3), ("strength", C.c_float)]


class SphStats(C.Structure):
    _fields_ = [("steps", C.c_int64), ("sim_time", C.c_double), ("active", C.c_int32),
                ("capacity", C.c_int32), ("grid", C.c_int32 * 3), ("key_bits", C.c_int32),
                ("device_bytes", C.c_int64)]


class SphKernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("total_ms", C.c_double),
                ("bytes_per_launch", C.c_double), ("timed", C.c_int64)]


class SphSlab(C.Structure):
    _fields_ = [("cx_lo", C.c_int32), ("cx_hi", C.c_int32)]


class SphCommId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


class SphDecomp(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("local_ranks", C.c_int32), ("cut", SphSlab),
                ("owned", C.c_int64), ("total", C.c_int64), ("rebalances", C.c_int32)]


SPH_SLAB_RECORD_BYTES = 32
SPH_ABI_VERSION = 2

assert C.sizeof(SphDragInput) == 20
assert C.sizeof(SphConfig) == 20
assert C.sizeof(SphCommId) == 128

# every entry point declared in include/sphhip.h, with its ctypes signature
_P = C.c_void_p
_I = C.c_int32
SIGNATURES = {
    "sph_abi_version": ([], C.c_int32),
    "sph_last_error": ([_P], C.c_char_p),
    "sph_create": ([C.POINTER(SphConfig), _I, C.POINTER(_P)], C.c_int),
    "sph_destroy": ([_P], None),
    "sph_resize": ([_P, _I], C.c_int),
    "sph_set_stream": ([_P, _P], C.c_int),
    "sph_get_stream": ([_P, C.POINTER(_P)], C.c_int),
    "sph_set_params": ([_P, C.POINTER(SphParams)], C.c_int),
    "sph_get_params": ([_P, C.POINTER(SphParams)], C.c_int),
    "sph_scenario_params": ([C.POINTER(SphScenario), C.POINTER(SphParams), C.POINTER(C.c_float)], C.c_int),
    "sph_upload_particles_aos84": ([_P, _P, _I], C.c_int),
    "sph_download_particles_aos84": ([_P, _P, _I], C.c_int),
    "sph_upload_state": ([_P, _P, _P, _I], C.c_int),
    "sph_init_scenario": ([_P, C.POINTER(SphScenario)], C.c_int),
    "sph_init_particles": ([_P, _I, _I, _I, _I], C.c_int),
    "sph_split_particles": ([_P, _P, _I, C.POINTER(C.c_int32)], C.c_int),
    "sph_get_particles_aos84": ([_P, _I, _I, _P], C.c_int),
    "sph_set_particles_aos84": ([_P, _I, _I, _P], C.c_int),
    "sph_step": ([_P, C.c_float, _I], C.c_int),
    "sph_set_sim_time": ([_P, C.c_double], C.c_int),
    "sph_set_drag": ([_P, C.POINTER(SphDragInput)], C.c_int),
    "sph_set_adhesion": ([_P, _P, _I], C.c_int),
    "sph_read_adhesion_terms": ([_P, _P, _I], C.c_int),
    "sph_read_positions": ([_P, _P, _I], C.c_int),
    "sph_read_rotations": ([_P, _P, _I], C.c_int),
    "sph_read_velocities": ([_P, _P, _I], C.c_int),
    "sph_read_angular_velocities": ([_P, _P, _I], C.c_int),
    "sph_read_density": ([_P, _P, _I], C.c_int),
    "sph_read_pressure_term": ([_P, _P, _I], C.c_int),
    "sph_synchronize": ([_P], C.c_int),
    "sph_request_readback": ([_P, _I], C.c_int),
    "sph_readback_status": ([_P], C.c_int),
    "sph_readback_get": ([_P, _I, _P, _I], C.c_int),
    "sph_readback_count": ([_P, C.POINTER(C.c_int32)], C.c_int),
    "sph_export_aos84_device": ([_P, _P, _I], C.c_int),
    "sph_write_draw_args": ([_P, _P], C.c_int),
    "sph_get_stats": ([_P, C.POINTER(SphStats)], C.c_int),
    "sph_get_kernel_stat": ([_P, _I, C.POINTER(SphKernelStat)], C.c_int),
    "sph_reset_kernel_stats": ([_P], C.c_int),
    "sph_set_profile_every": ([_P, _I], C.c_int),
    "sph_read_sorted_ids": ([_P, _P, _I], C.c_int),
    "sph_read_cell_start": ([_P, _P, _I], C.c_int),
    "sph_read_torque_int": ([_P, _P, _I], C.c_int),
    "sph_read_path_counts": ([_P, _P, _I], C.c_int),
    "sph_read_mover_count": ([_P, _P], C.c_int),
    "sph_read_resort_counts": ([_P, _P, _I], C.c_int),
    "sph_read_hit_mask_counts": ([_P, _P, _I], C.c_int),
    "sph_debug_radix_sort": ([_P, _P, _I, _I, _P, _P], C.c_int),
    "sph_debug_kick": ([_P, _I, _P], C.c_int),
    "sph_slab_set": ([_P, C.POINTER(SphSlab)], C.c_int),
    "sph_slab_init_scenario": ([_P, C.POINTER(SphScenario)], C.c_int),
    "sph_slab_count_sends": ([_P, C.POINTER(C.c_int32)], C.c_int),
    "sph_slab_count_sends_async": ([_P, _P], C.c_int),
    "sph_slab_column_counts": ([_P, _P, _I], C.c_int),
    "sph_slab_recut": ([_P, C.POINTER(SphSlab)], C.c_int),
    "sph_slab_send_capacity": ([_P, C.POINTER(C.c_int32)], C.c_int),
    "sph_slab_pack_send": ([_P, _I, _P, _I], C.c_int),
    "sph_slab_assemble": ([_P, _P, _I, _P, _I], C.c_int),
    "sph_slab_ranges": ([_P, C.POINTER(C.c_int32)], C.c_int),
    "sph_slab_density": ([_P], C.c_int),
    "sph_slab_pack_rho": ([_P, _I, _P, _I], C.c_int),
    "sph_slab_unpack_rho": ([_P, _I, _P, _I], C.c_int),
    "sph_slab_force": ([_P, C.c_float, _I], C.c_int),
    "sph_slab_finish_step": ([_P, C.c_float], C.c_int),
    "sph_slab_read_owned": ([_P, _P, _I, C.POINTER(C.c_int32)], C.c_int),
    "sph_comm_unique_id": ([C.POINTER(SphCommId)], C.c_int),
    "sph_comm_init": ([_P, C.POINTER(SphCommId), _I, _I], C.c_int),
    "sph_set_rebalance": ([_P, _I], C.c_int),
    "sph_get_decomposition": ([_P, C.POINTER(SphDecomp)], C.c_int),
}


class SphError(RuntimeError):
    def __init__(self, fn: str, status: int, message: str = ""):
        self.status = status
        super().__init__(f"{fn} -> {_STATUS.get(status, status)}: {message}")


_lib = None


def lib() -> C.CDLL:
    """Load libsphhip.so from the package directory. Raises if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same SONAME as
        # ROCm's) and whichever loads first serves both. Load torch's first when torch is
        # installed, so torch streams/RCCL and this library share one runtime and stream
        # handles are valid across them.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = lib_path()
        if not path.exists():
            raise RuntimeError(f"libsphhip.so not built at {path}: run __graft_entry__.build()")
        L = C.CDLL(str(path))
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def lib_path() -> Path:
    """The library lib() loads (SPHHIP_LIB overrides the in-tree build, for variant A/Bs)."""
    return Path(os.environ.get("SPHHIP_LIB", str(LIB_PATH)))


def device_code_hash(path: Optional[Path] = None) -> str:
    """sha256 (16 hex digits) of the library's gfx950 code objects: the ELF section `.hip_fatbin` of
    libsphhip.so. It identifies the kernels that ran, independent of host-only changes, and stamps the
    committed counter files (profiles/pmc_*.json, clock_*.json) so that bench.py uses counters only
    of the kernels it is timing."""
    import hashlib
    import struct
    data = Path(path or lib_path()).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise RuntimeError(f"{path}: not a 64-bit ELF")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    for name, _typ, _flags, _addr, off, size in secs:
        end = data.index(b"\0", stro + name)
        if data[stro + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise RuntimeError(f"{path}: no .hip_fatbin section")


def ptr(a) -> C.c_void_p:
    if a is None:
        return C.c_void_p(0)
    if isinstance(a, np.ndarray):
        return C.c_void_p(a.ctypes.data)
    return C.c_void_p(int(a))


def check(fn: str, status: int, ctx=None) -> None:
    if status != SPH_OK:
        msg = lib().sph_last_error(ctx).decode(errors="replace") if ctx else ""
        raise SphError(fn, status, msg)
