"""Host mirror of the reference's bond bookkeeping, `CellAdhesionManager` (Assets/Scripts/CellAdhesionManager.cs).

The bonds the adhesion kernels consume (`adhesion.hip`) are created and edited on the host
when cells divide. This module keeps that logic with the reference's names, order and quirks, so the shipped
scene runs with the bonds its genome asks for (`NewCellGenome.asset`: parentMakeAdhesion, both children keep
their adhesions):

  * AddBond (:86-129): no self, negative or duplicate bonds; creationFrame = the frame counter;
    initialRelOrientation = Inverse(rotA) * rotB from the controller's last read-back rotations;
  * HandleCellSplit (:425-510): the parent's bonds move to the children by the parent-side zone
    (ZoneC: both / A / B by the keep flags; ZoneB -> child A; ZoneA -> child B), then the child-to-child bond;
  * LateUpdate -> UpdateBondVisuals (:72-75, :245-304) minus drawing: UpdateBondZones (:338-424; zones
    re-classified for two frames, anchors fixed on the frame after creation) and FilterBonds (:184-243;
    per (cell, zone) end keep only the shortest bond);
  * GetAdhesionConnectionsForGPU (:524-564): the 84-byte records `sph_set_adhesion` takes.

Quirks kept: GetIndexForUniqueID scans ParticleIDs linearly (inactive slots hold uniqueID 0); the export's
mode is `uniqueID % modes.Count`; FilterBonds orders ties by list order (LINQ OrderBy is stable).
Deterministic choice: UpdateBondZones reads each cell's mode from the controller's current particle data
(the reference reads `cachedParticleData`, whose age depends on AsyncGPUReadback latency). Unity's
Quaternion/Vector3 code is closed source: the math here (genome.py) is a float32 restatement, parity
unpinned against Unity itself; tests/test_gpu_shipped_bonds.py checks the GPU run against an oracle replay
of this same host logic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import IntEnum
from typing import List, Optional

import numpy as np

from . import _abi as A
from .genome import distance, dot, euler, normalized, q_inverse, qmul, rotate

f32 = np.float32
RAD2DEG = f32(57.29578)


class BondZone(IntEnum):
    ZoneA = 0
    ZoneB = 1
    ZoneC = 2


@dataclass
class BondAnchor:
    """CellAdhesionManager.BondAnchor (:27-32)."""
    localPosition: np.ndarray
    cellID: int
    radius: float


@dataclass(eq=False)
class AdhesionBond:
    """CellAdhesionManager.AdhesionBond (:35-54); compared by identity, as the C# class."""
    cellA: int
    cellB: int
    zoneA: BondZone
    zoneB: BondZone
    isChildToChild: bool = False
    childAUniqueID: int = -1
    childBUniqueID: int = -1
    initialZoneA: BondZone = BondZone.ZoneA
    initialZoneB: BondZone = BondZone.ZoneA
    creationFrame: int = 0
    initialRelOrientation: np.ndarray = field(default_factory=lambda: np.array([0, 0, 0, 1], f32))
    anchorA: Optional[BondAnchor] = None
    anchorB: Optional[BondAnchor] = None


class CellAdhesionManager:
    """The reference manager's bond logic (see module doc). `controller` is a ParticleSystemController."""

    def __init__(self, particleSystemController=None):
        self.particleSystemController = particleSystemController
        self.enableAnchorConstraints = True     # :18
        self.bonds: List[AdhesionBond] = []     # :23

    # ------------------------------------------------------------------ helpers
    def _frame(self) -> int:
        return self.particleSystemController.frameCount    # Time.frameCount

    def GetIndexForUniqueID(self, uniqueID: int) -> int:
        """:307-318 — the first slot whose uniqueID matches (inactive slots hold 0)."""
        ctl = self.particleSystemController
        if ctl is None or not ctl.ParticleIDs:
            return -1
        for i, d in enumerate(ctl.ParticleIDs):
            if d.uniqueID == uniqueID:
                return i
        return -1

    def ClassifyBondDirection(self, cellPos, cellRot, otherPos, splitYaw, splitPitch, inheritanceAngleDeg=10.0):
        """:320-336."""
        bondDirWorld = normalized(np.asarray(otherPos, f32) - np.asarray(cellPos, f32))
        bondDirLocal = rotate(q_inverse(cellRot), bondDirWorld)
        splitDirLocal = rotate(euler(splitPitch, splitYaw, 0.0), (0.0, 0.0, 1.0))
        d = dot(bondDirLocal, splitDirLocal)
        angle = f32(math.acos(float(min(max(d, f32(-1.0)), f32(1.0))))) * RAD2DEG
        halfWidth = f32(inheritanceAngleDeg) * f32(1.0)
        if abs(angle - f32(90.0)) <= halfWidth:
            return BondZone.ZoneC
        return BondZone.ZoneB if d > 0 else BondZone.ZoneA

    # ------------------------------------------------------------------ bonds
    def AddBond(self, cellA, cellB, zoneA, zoneB, isChildToChild=False, childAUniqueID=-1, childBUniqueID=-1):
        """:86-129."""
        if cellA == cellB or cellA < 0 or cellB < 0:
            return
        if any((b.cellA == cellA and b.cellB == cellB) or (b.cellA == cellB and b.cellB == cellA) for b in self.bonds):
            return
        bond = AdhesionBond(cellA, cellB, BondZone(zoneA), BondZone(zoneB), isChildToChild, childAUniqueID,
                            childBUniqueID, BondZone(zoneA), BondZone(zoneB), self._frame())
        ctl = self.particleSystemController
        rots = ctl.CpuParticleRotations if ctl is not None else None
        if rots is not None:
            ia, ib = self.GetIndexForUniqueID(cellA), self.GetIndexForUniqueID(cellB)
            if 0 <= ia < len(rots) and 0 <= ib < len(rots):
                bond.initialRelOrientation = qmul(q_inverse(rots[ia]), rots[ib])
        self.bonds.append(bond)

    def ClearBonds(self) -> None:
        self.bonds.clear()

    def HandleCellSplit(self, parentIndex, childAIndex, childBIndex, parentSplitYaw, parentSplitPitch,
                        parentRotation, parentPosition, childAModeIndex, childBModeIndex, parentMakeAdhesion,
                        childA_KeepAdhesion, childB_KeepAdhesion) -> None:
        """:425-510."""
        ctl = self.particleSystemController
        ids = ctl.ParticleIDs if ctl is not None else []
        if ctl is None or childAIndex < 0 or childBIndex < 0 or childAIndex >= len(ids) or childBIndex >= len(ids):
            return
        uniqueA = ids[childAIndex].uniqueID
        uniqueB = ids[childBIndex].uniqueID
        parentUniqueID = ids[childAIndex].parentID
        parentBonds = []
        for bond in list(self.bonds):
            if bond.cellA == parentUniqueID or bond.cellB == parentUniqueID:
                parentBonds.append(bond)
                self.bonds.remove(bond)
        for pb in parentBonds:
            parentIsA = pb.cellA == parentUniqueID
            neighborID = pb.cellB if parentIsA else pb.cellA
            neighborZone = pb.zoneB if parentIsA else pb.zoneA
            parentZone = pb.zoneA if parentIsA else pb.zoneB
            if parentZone == BondZone.ZoneC:
                # the reference passes the bond's zoneA (not the parent-side zone) for the child's end
                if childA_KeepAdhesion and childB_KeepAdhesion:
                    self.AddBond(uniqueA, neighborID, pb.zoneA, neighborZone)
                    self.AddBond(uniqueB, neighborID, pb.zoneA, neighborZone)
                elif childA_KeepAdhesion:
                    self.AddBond(uniqueA, neighborID, pb.zoneA, neighborZone)
                elif childB_KeepAdhesion:
                    self.AddBond(uniqueB, neighborID, pb.zoneA, neighborZone)
            elif parentZone == BondZone.ZoneB and childA_KeepAdhesion:
                self.AddBond(uniqueA, neighborID, BondZone.ZoneB, neighborZone)
            elif parentZone == BondZone.ZoneA and childB_KeepAdhesion:
                self.AddBond(uniqueB, neighborID, BondZone.ZoneA, neighborZone)
        if parentMakeAdhesion:
            self.AddBond(uniqueA, uniqueB, BondZone.ZoneC, BondZone.ZoneC, True, uniqueA, uniqueB)

    # ------------------------------------------------------------------ per frame
    def LateUpdate(self) -> None:
        """:72-75 -> UpdateBondVisuals (:245-304): zones, filtering (the line renderers are not built)."""
        if self.particleSystemController is None:
            return
        self.UpdateBondZones()
        self.FilterBonds()

    def UpdateBondZones(self) -> None:
        """:338-424."""
        ctl = self.particleSystemController
        if ctl is None or not ctl.ParticleIDs or ctl.genome is None:
            return
        genome = ctl.genome
        pos, rot = ctl.CpuParticlePositions, ctl.CpuParticleRotations
        frame = self._frame()
        modes = None
        for bond in self.bonds:
            if frame > bond.creationFrame + 1:
                continue
            ia, ib = self.GetIndexForUniqueID(bond.cellA), self.GetIndexForUniqueID(bond.cellB)
            if ia < 0 or ib < 0 or ia >= len(pos) or ib >= len(pos) or rot is None or ia >= len(rot) or ib >= len(rot):
                continue
            posA, posB, rotA, rotB = pos[ia], pos[ib], rot[ia], rot[ib]
            if frame == bond.creationFrame + 1 and (bond.anchorA is None or bond.anchorB is None):
                direction = normalized(posB - posA)
                one = f32(1.0)                           # cellRadiusA = cellRadiusB = 1 (:381-382)
                anchorPosA = (posA + direction * one).astype(f32)
                anchorPosB = (posB + (-direction) * one).astype(f32)
                bond.anchorA = BondAnchor(rotate(q_inverse(rotA), (anchorPosA - posA).astype(f32)), bond.cellA, 1.0)
                bond.anchorB = BondAnchor(rotate(q_inverse(rotB), (anchorPosB - posB).astype(f32)), bond.cellB, 1.0)
            if modes is None:
                modes = ctl.cached_mode_indices()
            ma = int(modes[ia]) if ia < len(modes) else 0
            mb = int(modes[ib]) if ib < len(modes) else 0
            yA = pA = yB = pB = 0.0
            if 0 <= ma < len(genome.modes):
                yA, pA = genome.modes[ma].parentSplitYaw, genome.modes[ma].parentSplitPitch
            if 0 <= mb < len(genome.modes):
                yB, pB = genome.modes[mb].parentSplitYaw, genome.modes[mb].parentSplitPitch
            bond.zoneA = self.ClassifyBondDirection(posA, rotA, posB, yA, pA)
            bond.zoneB = self.ClassifyBondDirection(posB, rotB, posA, yB, pB)

    def _length(self, b: AdhesionBond) -> float:
        pos = self.particleSystemController.CpuParticlePositions
        ia, ib = self.GetIndexForUniqueID(b.cellA), self.GetIndexForUniqueID(b.cellB)
        if ia < 0 or ib < 0 or ia >= len(pos) or ib >= len(pos):
            return float(np.finfo(f32).max)
        return float(distance(pos[ia], pos[ib]))

    def FilterBonds(self) -> None:
        """:184-243 — for each (cell, zone) end shared by several bonds (created before this frame),
        keep the shortest, unless the group holds a bond that is ZoneC on one end and A/B on the other."""
        if not self.bonds or self.particleSystemController is None:
            return
        frame = self._frame()
        to_remove = []
        for end in ("A", "B"):
            groups = {}
            for b in self.bonds:
                if b.creationFrame < frame:
                    key = (b.cellA, b.zoneA) if end == "A" else (b.cellB, b.zoneB)
                    groups.setdefault(key, []).append(b)
            for group in groups.values():
                def mixed(b):
                    mine, other = (b.zoneA, b.zoneB) if end == "A" else (b.zoneB, b.zoneA)
                    return (mine == BondZone.ZoneC and other in (BondZone.ZoneA, BondZone.ZoneB)) or \
                           (mine in (BondZone.ZoneA, BondZone.ZoneB) and other == BondZone.ZoneC)
                if any(mixed(b) for b in group):
                    continue
                if len(group) > 1:
                    shortest = min(group, key=self._length)    # first of the minima: OrderBy is stable
                    for b in group:
                        if b is not shortest and all(b is not r for r in to_remove):
                            to_remove.append(b)
        if to_remove:
            self.bonds = [b for b in self.bonds if all(b is not r for r in to_remove)]

    # ------------------------------------------------------------------ export
    def GetAdhesionConnectionsForGPU(self) -> np.ndarray:
        """:524-564 — AdhesionConnectionExport records (ADHESION84) for sph_set_adhesion."""
        ctl = self.particleSystemController
        if ctl is None:
            return np.zeros(0, A.ADHESION84)
        ids, genome = ctl.ParticleIDs, ctl.genome
        rows = []
        for bond in self.bonds:
            ia, ib = self.GetIndexForUniqueID(bond.cellA), self.GetIndexForUniqueID(bond.cellB)
            if ia < 0 or ib < 0:
                continue
            modeA = 0
            if ids and ia < len(ids) and genome is not None and len(genome.modes) > 0:
                modeA = ids[ia].uniqueID % len(genome.modes)
            rest, stiff, damp, ocs, color = f32(2.0), f32(100.0), f32(5.0), f32(0.5), (1.0, 1.0, 1.0, 1.0)
            if genome is not None and modeA < len(genome.modes):
                m = genome.modes[modeA]
                rest, stiff, damp = f32(m.adhesionRestLength), f32(m.adhesionSpringStiffness), f32(m.adhesionSpringDamping)
                ocs, color = f32(m.orientationConstraintStrength), m.modeColor
            r = np.zeros(1, A.ADHESION84)[0]
            r["particleA"], r["particleB"] = ia, ib
            r["restLength"], r["springStiffness"], r["springDamping"] = rest, stiff, damp
            r["connectionColor"] = np.asarray(color, f32)
            r["initialRelOrientation"] = bond.initialRelOrientation
            r["anchorLocalPosA"] = bond.anchorA.localPosition if bond.anchorA is not None else np.zeros(3, f32)
            r["anchorLocalPosB"] = bond.anchorB.localPosition if bond.anchorB is not None else np.zeros(3, f32)
            r["anchorConstraintStiffness"] = ocs * f32(10.0)
            r["enableAnchorConstraint"] = 1 if self.enableAnchorConstraints else 0
            rows.append(r)
        return np.array(rows, A.ADHESION84) if rows else np.zeros(0, A.ADHESION84)
