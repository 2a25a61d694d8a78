"""Model R's one-launch step at the reference's scale (contact.hip k_contact_fused: the re-sort, contact, drag, motion
and rotation in one dispatch, reading the previous step's arrays through this step's permutation) against the
two-launch path (k_mv_rank + the contact pass; SPH_FUSED=0, read at context creation): whole runs must agree BIT FOR
BIT, particles, int torques and slot order, including inactive slots, the drag input and a state where many particles
change cells each step (the movers' bitonic sort). The oracle comparison of the fused path is test_gpu_parity.py::test_contact_bit_exact[4096-10]."""
import numpy as np
import pytest

from test_gpu_parity import random_sphere

pytestmark = pytest.mark.gpu


def _ctl(pkg, monkeypatch, flag, parts, setup=None):
    monkeypatch.setenv("SPH_FUSED", flag)
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    ctl.Start(parts.copy())
    monkeypatch.delenv("SPH_FUSED")
    if setup:
        setup(ctl)
    return ctl


def _same(a, b, what):
    assert a.GetParticles().tobytes() == b.GetParticles().tobytes(), f"{what}: particles differ"
    assert np.array_equal(a.context.torque_int(), b.context.torque_int()), f"{what}: torques differ"
    assert np.array_equal(a.context.sorted_ids(), b.context.sorted_ids()), f"{what}: slot order differs"


@pytest.mark.parametrize("case", ["sphere", "drag_inactive", "many_movers", "n64"])
def test_fused_step_bit_identical(pkg, monkeypatch, case):
    n = 64 if case == "n64" else 4096
    parts = random_sphere(pkg.PARTICLE84, n, seed=7)
    if case == "many_movers":   # cells of 4 units: ~1/3 of the particles change cell per step at these speeds
        parts["velocity"] *= 60.0
    setup = None
    if case == "drag_inactive":
        def setup(ctl):
            ctl.activeParticleCount = 3000
            ctl.drag.selectedID = 17
            ctl.drag.targetPosition = (3.0, -2.0, 1.0)
            ctl.drag.strength = 100.0
    two = _ctl(pkg, monkeypatch, "0", parts, setup)
    one = _ctl(pkg, monkeypatch, "1", parts, setup)
    try:
        for k in (1, 2, 5, 40):
            for _ in range(k):
                two.Update(0.01)
                one.Update(0.01)
            _same(two, one, f"{case}, after {k} more steps")
    finally:
        two.OnDestroy()
        one.OnDestroy()
