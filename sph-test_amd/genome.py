"""Genome, scene configuration and the Unity math the host-side cell division uses.

* `CellGenome` / `GenomeMode` mirror the reference's ScriptableObject
  (/root/reference/Assets/Scripts/Genome System/CellGenome.cs:6-170): same field names and defaults.
* `load_genome_asset` / `load_scene_controller` read the reference's own Unity YAML files (a genome
  `.asset` such as NewCellGenome.asset, and the `ParticleSystemController` block of a `.unity`
  scene such as `Particle Simulation.unity:151-178`) so a shipped scenario runs headless. Unity
  YAML carries `!u!` tags and `&anchor` ids per document; the reader strips those and parses
  each document with `yaml.safe_load` (nothing in the file is executed).
* `euler`, `look_rotation`, `rotate` restate UnityEngine.Quaternion.Euler / LookRotation /
  operator*(Quaternion, Vector3) in float32 (Unity is closed source: their published
  conventions — Euler applies z, then x, then y, in degrees; LookRotation's z axis is `forward`,
  its y axis the projection of `upwards` — parity unpinned).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field, fields
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np

f32 = np.float32


@dataclass
class GenomeMode:
    """GenomeMode (CellGenome.cs:124-170)."""
    index: int = 0
    modeName: str = ""
    splitInterval: float = 5.0
    isInitial: bool = False
    parentMakeAdhesion: bool = False
    modeColor: tuple = (1.0, 1.0, 1.0, 1.0)
    parentSplitYaw: float = 0.0
    parentSplitPitch: float = 0.0
    childAModeIndex: int = -1
    childA_OrientationYaw: float = 0.0
    childA_OrientationPitch: float = 0.0
    childA_KeepAdhesion: bool = False
    childBModeIndex: int = -1
    childB_OrientationYaw: float = 0.0
    childB_OrientationPitch: float = 0.0
    childB_KeepAdhesion: bool = False
    adhesionRestLength: float = 3.0
    adhesionSpringStiffness: float = 100.0
    adhesionSpringDamping: float = 5.0
    orientationConstraintStrength: float = 0.5
    maxAllowedAngleDeviation: float = 45.0
    adhesionCanBreak: bool = False
    adhesionBreakForce: float = 1000.0


@dataclass
class CellGenome:
    """CellGenome (CellGenome.cs:6-122)."""
    modes: List[GenomeMode] = field(default_factory=list)

    def RefreshModeIndexes(self) -> None:                       # :12-20
        for i, m in enumerate(self.modes):
            m.index = i
            if not m.modeName:
                m.modeName = f"Mode {i}"

    def GetInitialModes(self) -> List[int]:                     # :26-37
        return [i for i, m in enumerate(self.modes) if m.isInitial]

    def ValidateForSimulation(self) -> None:                    # :73-90
        initial = self.GetInitialModes()
        if not initial and self.modes:
            self.modes[0].isInitial = True
        elif len(initial) > 1:
            names = ", ".join(f"'{self.modes[i].modeName}'" for i in initial)
            raise ValueError(f"Multiple initial modes detected: {names}. Only one mode can be marked as "
                             "initial during simulation.")


# ---------------------------------------------------------------- Unity YAML
_DOC = re.compile(r"^--- !u!(\d+) &(-?\d+)(?: stripped)?\s*$", re.M)


def unity_documents(text: str) -> List[tuple]:
    """Split a Unity YAML file into (class_id, file_id, mapping) documents."""
    import yaml
    body = "\n".join(line for line in text.splitlines() if not line.startswith("%"))
    out = []
    marks = list(_DOC.finditer(body))
    for k, m in enumerate(marks):
        end = marks[k + 1].start() if k + 1 < len(marks) else len(body)
        doc = yaml.safe_load(body[m.end():end]) or {}
        out.append((int(m.group(1)), int(m.group(2)), doc))
    return out


def _coerce(value, default):
    if isinstance(default, bool):
        return bool(int(value))
    if isinstance(default, int):
        return int(value)
    if isinstance(default, float):
        return float(value)
    if isinstance(default, tuple) and isinstance(value, dict):
        return tuple(float(value[c]) for c in ("r", "g", "b", "a"))
    if isinstance(default, str):
        return "" if value is None else str(value)
    return value


def genome_from_mapping(mb: dict) -> CellGenome:
    g = CellGenome()
    proto = GenomeMode()
    for raw in mb.get("modes") or []:
        kw = {}
        for f in fields(GenomeMode):
            if f.name in raw:
                kw[f.name] = _coerce(raw[f.name], getattr(proto, f.name))
        g.modes.append(GenomeMode(**kw))
    g.RefreshModeIndexes()
    return g


def load_genome_asset(path) -> CellGenome:
    """A CellGenome `.asset` (e.g. Assets/Scripts/Genome System/NewCellGenome.asset)."""
    for cls, _, doc in unity_documents(Path(path).read_text()):
        mb = doc.get("MonoBehaviour") if cls == 114 else None
        if mb is not None and "modes" in mb:
            return genome_from_mapping(mb)
    raise ValueError(f"{path}: no CellGenome MonoBehaviour")


# ParticleSystemController's serialized inspector fields (ParticleSystemController.cs:11-28)
CONTROLLER_FIELDS = ("particleCount", "minRadius", "maxRadius", "spawnRadius", "globalDragMultiplier",
                     "torqueFactor", "torqueDamping", "boundaryFriction", "rollingContactRadiusMultiplier",
                     "density", "repulsionStrength", "spawnOverlapOffset", "splitVelocityMagnitude")


def load_scene_controller(path) -> Dict[str, float]:
    """The ParticleSystemController inspector values of a `.unity` scene (the MonoBehaviour that
    serializes `particleCount` and `computeShader`), e.g. Particle Simulation.unity:151-163."""
    for cls, _, doc in unity_documents(Path(path).read_text()):
        mb = doc.get("MonoBehaviour") if cls == 114 else None
        if mb is not None and "particleCount" in mb and "computeShader" in mb:
            out = {k: mb[k] for k in CONTROLLER_FIELDS if k in mb}
            out["particleCount"] = int(out.get("particleCount", 0))
            return out
    raise ValueError(f"{path}: no ParticleSystemController")


# ---------------------------------------------------------------- Unity quaternion math (float32)
def qmul(a, b):
    ax, ay, az, aw = (f32(v) for v in a)
    bx, by, bz, bw = (f32(v) for v in b)
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz], f32)


def rotate(q, v):
    """Quaternion * Vector3."""
    q = np.asarray(q, f32)
    v = np.asarray(v, f32)
    u, w = q[:3], q[3]
    t = f32(2.0) * np.cross(u, v).astype(f32)
    return (v + w * t + np.cross(u, t)).astype(f32)


def q_inverse(q):
    """Quaternion.Inverse of a rotation: the conjugate (Unity's native code is closed; rotations are unit)."""
    x, y, z, w = (f32(v) for v in q)
    return np.array([-x, -y, -z, w], f32)


def normalized(v):
    """Vector3.normalized: v / |v| when |v| > 1e-5, else zero."""
    v = np.asarray(v, f32)
    m = f32(math.sqrt(float(np.dot(v, v).astype(f32))))
    return (v / m).astype(f32) if m > f32(1e-5) else np.zeros(3, f32)


def dot(a, b):
    """Vector3.Dot in float32."""
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    return f32(a[0] * b[0] + a[1] * b[1] + a[2] * b[2])


def distance(a, b):
    """Vector3.Distance."""
    d = (np.asarray(a, f32) - np.asarray(b, f32)).astype(f32)
    return f32(math.sqrt(float(dot(d, d))))


def _axis_angle(axis, deg):
    h = math.radians(float(deg)) * 0.5
    s = math.sin(h)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, math.cos(h)], f32)


def euler(x, y, z):
    """Quaternion.Euler(x, y, z): rotate by z about Z, then x about X, then y about Y."""
    return qmul(qmul(_axis_angle((0, 1, 0), y), _axis_angle((1, 0, 0), x)), _axis_angle((0, 0, 1), z))


def look_rotation(forward, up=(0.0, 1.0, 0.0)):
    """Quaternion.LookRotation(forward, upwards)."""
    f = np.asarray(forward, np.float64)
    nf = np.linalg.norm(f)
    if nf < 1e-12:
        return np.array([0, 0, 0, 1], f32)
    zc = f / nf
    xc = np.cross(np.asarray(up, np.float64), zc)
    nx = np.linalg.norm(xc)
    if nx < 1e-12:   # forward parallel to up: any perpendicular x axis
        xc = np.cross((1.0, 0.0, 0.0) if abs(zc[0]) < 0.9 else (0.0, 1.0, 0.0), zc)
        nx = np.linalg.norm(xc)
    xc /= nx
    yc = np.cross(zc, xc)
    m = np.stack([xc, yc, zc], axis=1)   # columns = local axes in world space
    tr = m[0, 0] + m[1, 1] + m[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        q = [(m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s, 0.25 * s]
    elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        s = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        q = [0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s, (m[2, 1] - m[1, 2]) / s]
    elif m[1, 1] > m[2, 2]:
        s = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        q = [(m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s, (m[0, 2] - m[2, 0]) / s]
    else:
        s = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
        q = [(m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s, (m[1, 0] - m[0, 1]) / s]
    q = np.array(q, np.float64)
    return (q / np.linalg.norm(q)).astype(f32)


def get_direction(yaw, pitch):
    """ParticleSystemController.GetDirection (:966-969): Quaternion.Euler(pitch, yaw, 0) * forward."""
    return rotate(euler(pitch, yaw, 0.0), (0.0, 0.0, 1.0))


def initial_mode_index(genome: Optional[CellGenome]) -> int:
    """GetInitialModeIndex (ParticleSystemController.cs:1274-1286)."""
    if genome is None or not genome.modes:
        return 0
    for i, m in enumerate(genome.modes):
        if m.isInitial:
            return i
    return 0
