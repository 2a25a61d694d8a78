"""The CellAdhesionManager mirror (sph-test_amd/adhesion_manager.py; CellAdhesionManager.cs) on CPU:
its rules on small hand-made cases, and the shipped scene with its bonds replayed on the C oracle
(tests/oracle_backend.py). The GPU run of the same scene is compared with this replay frame by frame in
tests/test_gpu_shipped_bonds.py."""
import numpy as np
import pytest

from oracle_backend import oracle_backend
from shipped_scene import shipped_controller


class _Ctl:
    """The controller fields the manager reads."""
    def __init__(self, pkg, n=4):
        self.ParticleIDs = [pkg.ParticleIDData() for _ in range(n)]
        self.CpuParticlePositions = np.zeros((n, 3), np.float32)
        self.CpuParticleRotations = np.tile(np.array([0, 0, 0, 1], np.float32), (n, 1))
        self.genome = None
        self.frameCount = 10

    def cached_mode_indices(self):
        return np.zeros(len(self.ParticleIDs), np.int32)


def _ids(pkg, ctl, uids, parents=None):
    for i, u in enumerate(uids):
        ctl.ParticleIDs[i] = pkg.ParticleIDData(parents[i] if parents else 0, u, "A")


def test_add_bond_rejects_self_negative_and_duplicates(pkg):
    ctl = _Ctl(pkg)
    _ids(pkg, ctl, [1, 2, 3, 4])
    m = pkg.CellAdhesionManager(ctl)
    Z = pkg.BondZone
    m.AddBond(1, 1, Z.ZoneC, Z.ZoneC)
    m.AddBond(-1, 2, Z.ZoneC, Z.ZoneC)
    m.AddBond(1, 2, Z.ZoneC, Z.ZoneC)
    m.AddBond(2, 1, Z.ZoneA, Z.ZoneB)          # same pair, other order (:90)
    assert [(b.cellA, b.cellB) for b in m.bonds] == [(1, 2)]
    assert m.bonds[0].creationFrame == 10


def test_classify_bond_direction_zones(pkg):
    m = pkg.CellAdhesionManager(_Ctl(pkg))
    Z = pkg.BondZone
    q = np.array([0, 0, 0, 1], np.float32)
    o = np.zeros(3, np.float32)
    # split direction = local forward (+z) at yaw = pitch = 0
    assert m.ClassifyBondDirection(o, q, (0, 0, 1), 0, 0) == Z.ZoneB
    assert m.ClassifyBondDirection(o, q, (0, 0, -1), 0, 0) == Z.ZoneA
    assert m.ClassifyBondDirection(o, q, (1, 0, 0), 0, 0) == Z.ZoneC       # equatorial band ±10°
    assert m.ClassifyBondDirection(o, q, (1, 0, 0.15), 0, 0) == Z.ZoneC    # 8.5° off the equator
    assert m.ClassifyBondDirection(o, q, (1, 0, 0.2), 0, 0) == Z.ZoneB     # 11.3°
    assert m.ClassifyBondDirection(o, q, (1, 0, 0), 90, 0) == Z.ZoneB      # split yaw 90: +x


def test_handle_cell_split_transfers_by_zone(pkg):
    """:452-509 — ZoneB ends go to child A, ZoneA ends to child B, ZoneC ends to both (keep flags), then
    the child-to-child bond."""
    ctl = _Ctl(pkg, 6)
    Z = pkg.BondZone
    m = pkg.CellAdhesionManager(ctl)
    _ids(pkg, ctl, [7, 8, 9, 10, 0, 0])
    m.AddBond(7, 8, Z.ZoneB, Z.ZoneA)   # parent 7's end in ZoneB -> child A
    m.AddBond(9, 7, Z.ZoneC, Z.ZoneA)   # parent is cellB, its end ZoneA -> child B
    m.AddBond(7, 10, Z.ZoneC, Z.ZoneC)  # ZoneC -> both children
    # the split: parent 7 at slot 0 becomes child A (uid 11), child B (uid 12) at slot 4
    ctl.ParticleIDs[0] = pkg.ParticleIDData(7, 11, "A")
    ctl.ParticleIDs[4] = pkg.ParticleIDData(7, 12, "B")
    m.HandleCellSplit(0, 0, 4, 0.0, 0.0, None, None, 0, 0, True, True, True)
    got = sorted((b.cellA, b.cellB, int(b.zoneA), int(b.zoneB), b.isChildToChild) for b in m.bonds)
    assert got == sorted([
        (11, 8, int(Z.ZoneB), int(Z.ZoneA), False),
        (12, 9, int(Z.ZoneA), int(Z.ZoneC), False),
        (11, 10, int(Z.ZoneC), int(Z.ZoneC), False),   # ZoneC: both get the bond's zoneA (:477-478)
        (12, 10, int(Z.ZoneC), int(Z.ZoneC), False),
        (11, 12, int(Z.ZoneC), int(Z.ZoneC), True),
    ])
    # keep flags off: the parent's bonds are dropped, only the child-to-child bond is made
    m2 = pkg.CellAdhesionManager(ctl)
    m2.AddBond(11, 8, Z.ZoneB, Z.ZoneA)
    ctl.ParticleIDs[0] = pkg.ParticleIDData(11, 13, "A")
    ctl.ParticleIDs[5] = pkg.ParticleIDData(11, 14, "B")
    m2.HandleCellSplit(0, 0, 5, 0.0, 0.0, None, None, 0, 0, True, False, False)
    assert [(b.cellA, b.cellB) for b in m2.bonds] == [(13, 14)]


def test_filter_keeps_the_shortest_per_end(pkg):
    ctl = _Ctl(pkg)
    Z = pkg.BondZone
    _ids(pkg, ctl, [1, 2, 3, 4])
    ctl.CpuParticlePositions[:] = [(0, 0, 0), (1, 0, 0), (3, 0, 0), (0, 5, 0)]
    m = pkg.CellAdhesionManager(ctl)
    m.AddBond(1, 3, Z.ZoneB, Z.ZoneA)
    m.AddBond(1, 2, Z.ZoneB, Z.ZoneA)
    m.AddBond(1, 4, Z.ZoneC, Z.ZoneA)   # another end zone: its own group
    ctl.frameCount += 1                 # bonds of the current frame are exempt (:193)
    m.FilterBonds()
    assert [(b.cellA, b.cellB) for b in m.bonds] == [(1, 2), (1, 4)]
    # a group holding a ZoneC <-> ZoneA/B bond is not filtered (:197-200)
    m = pkg.CellAdhesionManager(ctl)
    ctl.frameCount = 10
    m.AddBond(1, 3, Z.ZoneC, Z.ZoneA)
    m.AddBond(1, 2, Z.ZoneC, Z.ZoneC)
    ctl.frameCount += 1
    m.FilterBonds()
    assert len(m.bonds) == 2


def _shipped_run(pkg, backend, frames=960):
    ctl = shipped_controller(pkg, backend=backend, bonds=True)
    ctl.Start()
    log = []
    for _ in range(frames):
        ctl.Frame(1.0 / 60.0)
        log.append((ctl.activeParticleCount, ctl.adhesionManager.GetAdhesionConnectionsForGPU().tobytes(),
                    ctl.CpuParticlePositions.tobytes(), ctl.CpuParticleRotations.tobytes()))
    return ctl, log


def test_shipped_scene_bonds_on_the_oracle(pkg, oracle):
    """The reference's scene with its bonds (NewCellGenome.asset: parentMakeAdhesion, both children keep
    adhesion), 16 s at 60 fps on the oracle: the child-to-child bond appears at the first division, its
    anchors one frame later; the second round of divisions re-distributes it and FilterBonds trims the
    result to one bond per (cell, zone) end."""
    ctl, log = _shipped_run(pkg, oracle_backend(oracle))
    m = ctl.adhesionManager
    n_bonds = [len(np.frombuffer(b, pkg.ADHESION84)) for _, b, _, _ in log]
    assert n_bonds[299] == 0 and n_bonds[300] == 1       # first division applied at frame 301
    assert max(n_bonds[300:600]) == 1 and n_bonds[-1] == 4
    assert ctl.activeParticleCount == 4
    first = [b for b in m.bonds if b.isChildToChild]
    assert all(b.anchorA is not None and b.anchorB is not None for b in m.bonds)
    assert len(first) == 2                               # (3,4) and (5,6): each second-round pair
    conns = m.GetAdhesionConnectionsForGPU()
    assert (conns["particleA"] < 4).all() and (conns["particleB"] < 4).all()
    assert np.allclose(conns["restLength"], 2.96) and np.allclose(conns["anchorConstraintStiffness"], 4.93)
    parts = ctl.GetParticles()[:4]
    assert np.isfinite(parts["position"]).all()
    # the bonded cells sit near the rest length apart (radii 2: contact repulsion keeps them >= ~4 apart)
    d = np.linalg.norm(parts["position"][conns["particleA"]] - parts["position"][conns["particleB"]], axis=1)
    assert (d > 2.0).all() and (d < 6.0).all()


def test_shipped_scene_without_manager_has_no_bonds(pkg, oracle):
    ctl = shipped_controller(pkg, backend=oracle_backend(oracle))
    ctl.Start()
    for _ in range(400):
        ctl.Frame(1.0 / 60.0)
    assert ctl.activeParticleCount == 2 and ctl.adhesionManager is None
