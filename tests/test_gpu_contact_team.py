"""Model R with several lanes per target (contact.hip, contact_accumulate_team) against one lane per
target: the team walks its hits in lane order, so the float totals are summed in the serial order and
every team size must give BIT-IDENTICAL particles and int torques, over several steps, with and
without adhesion bonds and with inactive slots. SPH_CT_TEAM is read at context creation.
"""
import numpy as np
import pytest

from adhesion_cases import bonded_sphere
from test_gpu_parity import random_sphere

pytestmark = pytest.mark.gpu


class _Manager:
    def __init__(self, conns):
        self.conns = conns

    def GetAdhesionConnectionsForGPU(self):
        return self.conns


def _run(pkg, monkeypatch, team, parts, steps, conns=None, active=None):
    monkeypatch.setenv("SPH_CT_TEAM", str(team))
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    if conns is not None:
        ctl.adhesionManager = _Manager(conns)
    ctl.Start(parts.copy())
    if active is not None:
        ctl.activeParticleCount = active
        ctl.drag.selectedID = 17
        ctl.drag.targetPosition = (3.0, -2.0, 1.0)
        ctl.drag.strength = 100.0
    for _ in range(steps):
        ctl.Update(0.01)
    out = ctl.GetParticles(), ctl.context.torque_int()
    ctl.OnDestroy()
    return out


@pytest.mark.parametrize("n,steps,active", [(64, 5, None), (4096, 5, None), (32768, 2, None), (2000, 3, 1500)])
def test_team_sizes_bit_identical(pkg, monkeypatch, n, steps, active):
    parts = random_sphere(pkg.PARTICLE84, n, seed=11)
    ref, tq_ref = _run(pkg, monkeypatch, 1, parts, steps, active=active)
    for team in (16, 64, 65):   # 65: the flat form (one wave per target, contact.hip CT_FLAT)
        got, tq = _run(pkg, monkeypatch, team, parts, steps, active=active)
        assert got.tobytes() == ref.tobytes(), f"team {team}"
        assert np.array_equal(tq, tq_ref), f"team {team}"


def test_team_sizes_bit_identical_with_bonds(pkg, monkeypatch):
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 4096, seed=7)
    conns = conns[:4096]
    ref, tq_ref = _run(pkg, monkeypatch, 1, parts, 3, conns=conns)
    for team in (16, 64, 65):   # 65: the flat form (one wave per target, contact.hip CT_FLAT)
        got, tq = _run(pkg, monkeypatch, team, parts, 3, conns=conns)
        assert got.tobytes() == ref.tobytes(), f"team {team}"
        assert np.array_equal(tq, tq_ref), f"team {team}"
