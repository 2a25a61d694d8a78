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
from typing import List, Optional

import numpy as np

from . import _abi as A
from .context import Context, make_scenario, scenario_params
from .genome import (CellGenome, get_direction, initial_mode_index, load_genome_asset, load_scene_controller,
                     look_rotation, rotate)

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
                 profile: bool = False, ndev: int = 1, rebalance_every: Optional[int] = None,
                 validate: bool = False):
        """ndev > 1: the domain is cut into x-slabs over ndev GPUs (device, device+1, ...) inside the
        library; positions() / velocities() / density() still return every particle in index order."""
        self.scenario = scenario
        self.params, self.dt = scenario_params(scenario)
        n = scenario.nx * scenario.ny * (scenario.nz if scenario.dim == 3 else 1)
        self.ctx = Context(A.SPH_MODEL_WCSPH, scenario.dim, capacity or (0 if ndev > 1 else n), device=device,
                           profile=profile, ndev=ndev, validate=validate)
        self.ctx.set_params(self.params)
        if ndev > 1 and rebalance_every is not None:
            self.ctx.set_rebalance(rebalance_every)
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


@dataclass
class ParticleIDData:
    """ParticleIDData (ParticleSystemController.cs:178-191)."""
    parentID: int = 0
    uniqueID: int = 0
    childType: str = "\0"

    def GetFormattedID(self) -> str:
        if self.childType == "\0":
            return "Unknown"
        return f"{self.parentID:02d}.{self.uniqueID:02d}.{self.childType}"


class ParticleSystemController:
    """Mirror of the reference controller's public API, driving Model R on the GPU.

    The per-frame GPU work is one `sph_step` (contact, adhesion, drag, motion, rotation). Cell
    division keeps the reference's host logic (timers, SplitCell's child placement) and hands the
    buffer edit to the device (`sph_split_particles`), so the particle buffer never makes the
    host round trip the reference's ProcessPendingSplits does (:793-794, :959)."""

    def __init__(self, particleCount: int = 10000, device: int = 0, backend=None):
        """backend: a factory (model, dim, capacity, device) -> context (default: the libsphhip Context)."""
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
        # [Header("Cell Division Settings")]  :26-28
        self.spawnOverlapOffset = 0.5
        self.splitVelocityMagnitude = 0.5
        # [Header("Genome")] :30-31 (a genome.CellGenome)
        self.genome: Optional[CellGenome] = None
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
        # True: Update ends with the reference's synchronous GetData (:332-333). False: positions and
        # rotations arrive through the asynchronous readback one frame later (:1142-1158), so the
        # host never waits on the GPU inside Update.
        self.immediateReadback = True
        self.nextUniqueIDCounter = 1            # :98
        self.cellSplitTimers: Optional[np.ndarray] = None   # :101
        self.pendingSplits: List[np.void] = []  # :104 (CellSplitData records)
        self.ParticleIDs: List[ParticleIDData] = []          # :118-119
        self._bonds_uploaded: Optional[bytes] = None
        self._rb_requested = False
        self._backend = backend if backend is not None else (lambda m, d, c, dev: Context(m, d, c, device=dev))
        self._ctx: Optional[Context] = None
        self.frameCount = 0                     # Unity's Time.frameCount: +1 per Update

    @classmethod
    def from_scene(cls, scene_path, genome_path=None, device: int = 0, backend=None) -> "ParticleSystemController":
        """The controller as a Unity scene serializes it (e.g. Particle Simulation.unity:151-178),
        with an optional genome asset (e.g. NewCellGenome.asset)."""
        vals = load_scene_controller(scene_path)
        ctl = cls(particleCount=vals.pop("particleCount"), device=device, backend=backend)
        for k, v in vals.items():
            setattr(ctl, k, float(v))
        if genome_path is not None:
            ctl.genome = load_genome_asset(genome_path)
        return ctl

    # ------------------------------------------------------------------ lifecycle
    def Start(self, particles: Optional[np.ndarray] = None) -> None:
        """Start (:211-242): InitializeBuffers (:373) then InitializeParticles (:484-552), or the given
        AoS-84 particles (PARTICLE84) uploaded as they are."""
        if self.genome is not None:
            self.genome.ValidateForSimulation()             # :216-226 (raises on several initial modes)
        self._ctx = self._backend(A.SPH_MODEL_CONTACT, 3, self.particleCount, self.device)
        if particles is not None:
            self._ctx.upload_aos84(particles)
            self.activeParticleCount = len(particles)
            self._push_uniforms()
        else:
            self.activeParticleCount = 1                    # :506-508
            self._push_uniforms()
            # genomeModesCount / defaultGenomeMode are never set on the compute shader, so
            # InitParticles sees 0 modes (modeIndex -1) and the host then sets particle 0's mode (:514-523)
            self._ctx.init_particles(self.particleCount, self.activeParticleCount)
            if self.genome is not None and self.genome.modes:
                first = self._ctx.get_particles(0, 1)
                first["modeIndex"] = initial_mode_index(self.genome)
                self._ctx.set_particles(0, first)
        self.ParticleIDs = [ParticleIDData() for _ in range(self.particleCount)]
        self.ParticleIDs[0] = ParticleIDData(0, 0, "A")     # :486-494
        self.cellSplitTimers = np.zeros(self.particleCount, np.float32)
        self.CpuParticlePositions = np.zeros((self.particleCount, 3), np.float32)
        self.CpuParticleRotations = np.zeros((self.particleCount, 4), np.float32)
        self._readback()

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

    def _readback(self) -> None:
        """Copy*ToReadbackBuffer + GetData (:325-333)."""
        n = self._ctx.n
        self.CpuParticlePositions[:n] = self._ctx.positions()
        self.CpuParticleRotations[:n] = self._ctx.rotations()

    def RequestParticleDataAsync(self) -> None:
        """:1115-1159 — deliver a finished asynchronous readback into the CPU arrays."""
        if self._rb_requested and self._ctx.readback_ready():
            pos = self._ctx.readback_get(A.SPH_READBACK_POSITIONS)
            rot = self._ctx.readback_get(A.SPH_READBACK_ROTATIONS)
            self.CpuParticlePositions[: len(pos)] = pos
            self.CpuParticleRotations[: len(rot)] = rot
            self._rb_requested = False

    def Frame(self, dt: float) -> None:
        """One Unity frame of the scene: this Update, then the adhesion manager's LateUpdate (Unity runs
        every script's LateUpdate after all Updates; CellAdhesionManager.cs:72-75)."""
        self.Update(dt)
        late = getattr(self.adhesionManager, "LateUpdate", None)
        if late is not None:
            late()

    def cached_mode_indices(self) -> np.ndarray:
        """modeIndex of every particle (CellAdhesionManager reads the controller's cachedParticleData)."""
        return self._ctx.get_particles(0, self._ctx.n)["modeIndex"]

    def Update(self, dt: float) -> None:
        """One frame (:244-351): readback delivery (:250), division (:253), uniforms (:255-263), the
        step with adhesion (:265-331), readback (:332-333)."""
        self.frameCount += 1
        if not self.immediateReadback:
            self.RequestParticleDataAsync()
        self.UpdateCellDivisionTimers(dt)
        self._push_uniforms()
        self._push_adhesion()
        d = self.drag
        self._ctx.set_drag(d.selectedID, d.targetPosition, d.strength)
        self._ctx.step(dt, 1)
        if self.immediateReadback:
            self._readback()
        elif not self._rb_requested:
            self._ctx.request_readback(A.SPH_READBACK_POSITIONS | A.SPH_READBACK_ROTATIONS)
            self._rb_requested = True

    # ------------------------------------------------------------------ cell division
    def UpdateCellDivisionTimers(self, deltaTime: float) -> None:
        """:631-727 — process last frame's splits, advance the timers, pick the cells due."""
        if self.pendingSplits:
            self.ProcessPendingSplits()
        allowed = self.particleCount - self.activeParticleCount
        if allowed <= 0 or self.genome is None or not self.genome.modes:
            return
        act = self.activeParticleCount
        self.cellSplitTimers[:act] += np.float32(deltaTime)
        modes = self._ctx.get_particles(0, act)["modeIndex"]   # the cached readback (:662-714)
        ready = []
        eps = np.float32(0.001)
        for i in range(act):
            m = int(modes[i])
            if 0 <= m < len(self.genome.modes):
                if self.cellSplitTimers[i] >= np.float32(self.genome.modes[m].splitInterval) - eps:
                    if len(ready) < allowed:
                        ready.append(i)
                    self.cellSplitTimers[i] = 0.0
        for i in ready:
            self.SplitCell(i, int(modes[i]))

    def SplitCell(self, parentIndex: int, parentModeIndex: Optional[int] = None) -> None:
        """:729-778 — the children's placement from the parent's last read-back pose."""
        g = self.genome
        if g is None or not g.modes or parentIndex >= self.activeParticleCount:
            return
        parentPos = self.CpuParticlePositions[parentIndex]
        parentRot = self.CpuParticleRotations[parentIndex]
        if parentModeIndex is None:
            parentModeIndex = int(self._ctx.get_particles(parentIndex, 1)["modeIndex"][0])
        if not 0 <= parentModeIndex < len(g.modes):
            parentModeIndex = initial_mode_index(g)
        mode = g.modes[parentModeIndex]
        a = mode.childAModeIndex if 0 <= mode.childAModeIndex < len(g.modes) else parentModeIndex
        b = mode.childBModeIndex if 0 <= mode.childBModeIndex < len(g.modes) else parentModeIndex
        forward, up, right = (rotate(parentRot, v) for v in ((0, 0, 1), (0, 1, 0), (1, 0, 0)))

        def world(d):
            return (right * d[0] + up * d[1] + forward * d[2]).astype(np.float32)

        split_dir = world(get_direction(mode.parentSplitYaw, mode.parentSplitPitch))
        off = np.float32(self.spawnOverlapOffset)
        vmag = np.float32(self.splitVelocityMagnitude)
        rec = np.zeros(1, A.SPLIT92)[0]
        rec["parentIndex"] = parentIndex
        rec["positionA"] = parentPos + split_dir * off
        rec["positionB"] = parentPos - split_dir * off
        rec["velocityA"] = split_dir * vmag          # parentVelocity = zero (:761)
        rec["velocityB"] = -split_dir * vmag
        rec["rotationA"] = look_rotation(world(get_direction(mode.childA_OrientationYaw, mode.childA_OrientationPitch)), up)
        rec["rotationB"] = look_rotation(world(get_direction(mode.childB_OrientationYaw, mode.childB_OrientationPitch)), up)
        rec["childAModeIndex"], rec["childBModeIndex"] = a, b
        self.pendingSplits.append(rec)

    def ProcessPendingSplits(self) -> None:
        """:780-964 — IDs, timers and the device-side buffer edit (sph_split_particles)."""
        if not self.pendingSplits:
            return
        splits = np.array(self.pendingSplits, dtype=A.SPLIT92)
        self.pendingSplits = []
        act0 = self.activeParticleCount
        new_active = self._ctx.split_particles(splits)
        cap = self._ctx.stats().capacity
        if cap > self.particleCount:                        # the device grew the buffers (:788-792)
            self._grow_host(cap)
        handle = getattr(self.adhesionManager, "HandleCellSplit", None)
        g = self.genome
        for k, sp in enumerate(splits):
            pidx = int(sp["parentIndex"])
            parent_uid = self.ParticleIDs[pidx].uniqueID
            b_idx = act0 + k
            self.ParticleIDs[pidx] = ParticleIDData(parent_uid, self.nextUniqueIDCounter, "A")
            self.ParticleIDs[b_idx] = ParticleIDData(parent_uid, self.nextUniqueIDCounter + 1, "B")
            self.nextUniqueIDCounter += 2
            self.cellSplitTimers[pidx] = 0.0
            self.cellSplitTimers[b_idx] = 0.0
            if handle is not None and g is not None:   # :929-951
                # "the parent's mode" is read after the parent's record became child A's (:854-857, :933)
                pm = int(sp["childAModeIndex"])
                mode = g.modes[pm if 0 <= pm < len(g.modes) else 0]
                handle(pidx, pidx, b_idx, mode.parentSplitYaw, mode.parentSplitPitch, self.CpuParticleRotations[pidx],
                       self.CpuParticlePositions[pidx], int(sp["childAModeIndex"]), int(sp["childBModeIndex"]),
                       mode.parentMakeAdhesion, mode.childA_KeepAdhesion, mode.childB_KeepAdhesion)
            self.activeParticleCount = act0 + k + 1
        self.activeParticleCount = new_active

    def _grow_host(self, cap: int) -> None:
        old = self.particleCount
        self.particleCount = cap
        self.ParticleIDs += [ParticleIDData() for _ in range(cap - old)]
        for name, shape in (("cellSplitTimers", (cap,)), ("CpuParticlePositions", (cap, 3)),
                            ("CpuParticleRotations", (cap, 4))):
            arr = getattr(self, name)
            new = np.zeros(shape, np.float32)
            new[:old] = arr[:old]
            setattr(self, name, new)

    def ResizeParticleBuffers(self, newCapacity: int) -> None:
        """:1162-1222 — keep the particles, grow the buffers (device-to-device)."""
        self._ctx.resize(newCapacity)
        if newCapacity > self.particleCount:
            self._grow_host(newCapacity)
        self.particleCount = newCapacity

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
