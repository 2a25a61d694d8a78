"""Host-side controllers: the reference's controller API over libsphhip.so.

`ParticleSystemController` mirrors the public surface of the reference's MonoBehaviour
(/root/reference/Assets/Scripts/ParticleSystemController.cs). It keeps the inspector fields
(:11-24), the CPU-side arrays `CpuParticlePositions` / `CpuParticleRotations` (:89-92),
`LastSelectedParticleID` (:126), `Start()` (:211) and `Update(dt)` (:244). The reference's
eleven Dispatch calls become one `sph_step`.

`SPHSim` is the north-star controller for Model S (SPEC_SPH.md §2). It covers the dam-break
and sloshing scenarios of BASELINE.json.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _abi as A
from .context import Context, make_scenario, scenario_params

# BASELINE.json configs: (kind, dim, fluid nx,ny,nz, tank tx,ty,tz)
CONFIGS = {
    "C1": (A.SPH_SCENARIO_DAMBREAK, 2, 64, 64, 1, 256, 128, 1),
    "C2": (A.SPH_SCENARIO_DAMBREAK, 3, 32, 64, 128, 128, 128, 128),
    "C3": (A.SPH_SCENARIO_DAMBREAK, 3, 64, 128, 128, 256, 256, 128),
    "C4": (A.SPH_SCENARIO_SLOSHING, 3, 256, 64, 256, 256, 128, 256),
    "C5": (A.SPH_SCENARIO_DAMBREAK, 3, 128, 256, 512, 512, 512, 512),
}


def config_scenario(name: str, dx: float = 0.01, seed: int = 1234) -> A.SphScenario:
    kind, dim, nx, ny, nz, tx, ty, tz = CONFIGS[name]
    return make_scenario(kind, dim, nx, ny, nz, tx, ty, tz, dx=dx, seed=seed)


class SPHSim:
    """Weakly-compressible SPH simulation on one GPU (Model S)."""

    def __init__(self, scenario: A.SphScenario, device: int = 0, capacity: Optional[int] = None,
                 profile: bool = False):
        self.scenario = scenario
        self.params, self.dt = scenario_params(scenario)
        n = scenario.nx * scenario.ny * (scenario.nz if scenario.dim == 3 else 1)
        self.ctx = Context(A.SPH_MODEL_WCSPH, scenario.dim, capacity or n, device=device, profile=profile)
        self.ctx.set_params(self.params)
        self.ctx.init_scenario(scenario)

    @classmethod
    def from_config(cls, name: str, **kw) -> "SPHSim":
        return cls(config_scenario(name), **kw)

    @property
    def n(self) -> int:
        return self.ctx.n

    def step(self, nsteps: int = 1, dt: Optional[float] = None) -> None:
        self.ctx.step(self.dt if dt is None else dt, nsteps)

    def positions(self) -> np.ndarray:
        return self.ctx.positions()

    def velocities(self) -> np.ndarray:
        return self.ctx.velocities()

    def density(self) -> np.ndarray:
        return self.ctx.density()

    def close(self) -> None:
        self.ctx.close()


@dataclass
class DragInput:
    """DragInput (ParticleSystemController.cs:149-154)."""
    selectedID: int = -1
    targetPosition: tuple = (0.0, 0.0, 0.0)
    strength: float = 0.0


class ParticleSystemController:
    """Mirror of the reference controller's public API, driving Model R on the GPU."""

    def __init__(self, particleCount: int = 10000, device: int = 0):
        # [Header("Particle Configuration")]  ParticleSystemController.cs:11-15
        self.particleCount = particleCount
        self.minRadius = 1.5
        self.maxRadius = 2.0
        self.spawnRadius = 15.0
        # [Header("Simulation Settings")]  :17-24
        self.globalDragMultiplier = 1.0
        self.torqueFactor = 1.0
        self.torqueDamping = 0.5
        self.boundaryFriction = 0.8
        self.rollingContactRadiusMultiplier = 5.0
        self.density = 0.1
        self.repulsionStrength = 200.0
        # [Header("Cell Division Settings")]  :26-28 (division itself is §8f-2, not yet built)
        self.spawnOverlapOffset = 0.5
        self.splitVelocityMagnitude = 0.5
        self.device = device
        self.activeParticleCount = 1            # :95
        self.CpuParticlePositions: Optional[np.ndarray] = None   # :89-90
        self.CpuParticleRotations: Optional[np.ndarray] = None   # :91-92
        self.LastSelectedParticleID = -1        # :125-126
        self.drag = DragInput()
        # [Header("Adhesion Visualization")] :55-56 — any object with GetAdhesionConnectionsForGPU()
        # returning an ADHESION84 array (CellAdhesionManager.cs:524-564)
        self.adhesionManager = None
        self.maxAdhesionConnections = 4096      # :128-129
        self._bonds_uploaded: Optional[bytes] = None
        self._ctx: Optional[Context] = None

    # ------------------------------------------------------------------ lifecycle
    def Start(self, particles: Optional[np.ndarray] = None) -> None:
        """InitializeBuffers (:373) + particle upload. `particles` is an AoS-84 array (PARTICLE84)."""
        self._ctx = Context(A.SPH_MODEL_CONTACT, 3, self.particleCount, device=self.device)
        if particles is not None:
            self._ctx.upload_aos84(particles)
            self.activeParticleCount = len(particles)
        self._push_uniforms()
        self.CpuParticlePositions = np.zeros((self.particleCount, 3), np.float32)
        self.CpuParticleRotations = np.zeros((self.particleCount, 4), np.float32)

    def _push_uniforms(self) -> None:
        p = self._ctx.get_params()
        p.spawn_radius = self.spawnRadius
        p.min_radius, p.max_radius = self.minRadius, self.maxRadius
        p.global_drag_multiplier = self.globalDragMultiplier
        p.torque_factor = self.torqueFactor
        p.torque_damping = self.torqueDamping
        p.boundary_friction = self.boundaryFriction
        p.rolling_contact_radius_multiplier = self.rollingContactRadiusMultiplier
        p.density = self.density
        p.repulsion_strength = self.repulsionStrength
        p.active_particle_count = self.activeParticleCount
        self._ctx.set_params(p)

    def _push_adhesion(self) -> None:
        """:285-303 — the manager's bonds, capped at maxAdhesionConnections, applied this frame
        when there is at least one. Re-uploaded only when they changed."""
        conns = None
        if self.adhesionManager is not None:
            conns = np.ascontiguousarray(self.adhesionManager.GetAdhesionConnectionsForGPU(), dtype=A.ADHESION84)
            conns = conns[: min(len(conns), self.maxAdhesionConnections)]
        blob = conns.tobytes() if conns is not None and len(conns) > 0 else b""
        if blob != self._bonds_uploaded:
            self._ctx.set_adhesion(conns if blob else None)
            self._bonds_uploaded = blob

    def Update(self, dt: float) -> None:
        """One frame: uniforms (:255-263), the step with adhesion (:265-331), readback (:332-333)."""
        self._push_uniforms()
        self._push_adhesion()
        d = self.drag
        self._ctx.set_drag(d.selectedID, d.targetPosition, d.strength)
        self._ctx.step(dt, 1)
        n = self._ctx.n
        self.CpuParticlePositions[:n] = self._ctx.positions()
        self.CpuParticleRotations[:n] = self._ctx.rotations()

    def ResizeParticleBuffers(self, newCapacity: int) -> None:
        """:1162-1222 — keep the particles, grow the buffers."""
        self._ctx.resize(newCapacity)
        self.particleCount = newCapacity
        pos = np.zeros((newCapacity, 3), np.float32)
        rot = np.zeros((newCapacity, 4), np.float32)
        pos[: len(self.CpuParticlePositions)] = self.CpuParticlePositions[:newCapacity]
        rot[: len(self.CpuParticleRotations)] = self.CpuParticleRotations[:newCapacity]
        self.CpuParticlePositions, self.CpuParticleRotations = pos, rot

    def GetParticles(self) -> np.ndarray:
        """particleBuffer.GetData (:519, :794): the full AoS-84 state."""
        return self._ctx.download_aos84()

    def SetParticles(self, parts: np.ndarray) -> None:
        """particleBuffer.SetData (:522, :959)."""
        self._ctx.upload_aos84(parts)

    def OnDestroy(self) -> None:
        """ReleaseBuffers (:453-482); the reference never calls it."""
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    @property
    def context(self) -> Context:
        return self._ctx
