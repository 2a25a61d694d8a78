"""Known-answer tests pinning the oracle's adhesion pass.

Each case is derived by hand from the HLSL text of ApplyAdhesionConstraints /
ApplyAdhesionDeltas (/root/reference/Assets/Compute/SimulateParticles.compute:424-607) and the
dispatch order of ParticleSystemController.Update (ParticleSystemController.cs:284-331),
evaluated in float64 numpy, and compared with the oracle's fp32 output. The fixed-point terms
(×1e6, round half to even) are compared to ±1 LSB: a float32 product may land on the other side
of a .5 boundary than the float64 one.
"""
import math

import numpy as np
import pytest

SCALE = 1_000_000


def _parts(O, n, spacing=5.0):
    p = np.zeros(n, O.PARTICLE84)
    p["position"][:, 0] = np.arange(n) * spacing    # far apart: no contacts (radius 0.2)
    p["rotation"] = (0, 0, 0, 1)
    p["radius"] = 0.2
    p["mass"] = 1.0
    p["momentOfInertia"] = 1.0
    p["drag"] = 1.0
    return p


def _bond(O, a, b, rest=2.0, k=100.0, damp=0.0, stiff=0.0, enable=0, relq=(0, 0, 0, 1),
          anc_a=(0, 0, 0), anc_b=(0, 0, 0)):
    c = np.zeros(1, O.ADHESION84)
    c["particleA"], c["particleB"] = a, b
    c["restLength"], c["springStiffness"], c["springDamping"] = rest, k, damp
    c["connectionColor"] = (1, 1, 1, 1)
    c["initialRelOrientation"] = relq
    c["anchorLocalPosA"], c["anchorLocalPosB"] = anc_a, anc_b
    c["anchorConstraintStiffness"] = stiff
    c["enableAnchorConstraint"] = enable
    return c


def test_spring_stretch(oracle):
    """:437-456 + :593-599 + UpdateMotion: a stretched spring pulls the pair together."""
    O = oracle
    p = _parts(O, 2, spacing=3.0)
    p["mass"][1] = 2.0
    dt = 0.01
    cp = O.contact_params(dt, spawn_radius=100.0, global_drag=0.0)
    out, _, terms = O.contact_step_bonds(cp, p, _bond(O, 0, 1, rest=2.0, k=100.0))
    F = 1.0 * 100.0                                   # displacement 1, along +x (A -> B)
    assert terms[0, 0] == pytest.approx(F / 1.0 * dt * SCALE, abs=1)
    assert terms[0, 4] == pytest.approx(-F / 2.0 * dt * SCALE, abs=1)
    assert (terms[0, [1, 2, 3, 5, 6, 7]] == 0).all() and (terms[0, 8:] == 0).all()
    assert out["velocity"][0][0] == pytest.approx(1.0, rel=1e-6)
    assert out["velocity"][1][0] == pytest.approx(-0.5, rel=1e-6)
    assert out["position"][0][0] == pytest.approx(0.0 + 1.0 * dt, rel=1e-6)


def test_spring_damping_uses_post_contact_velocity(oracle):
    """:444-446: the damping term reads the velocities ApplySPHForces left (controller:284)."""
    O = oracle
    p = _parts(O, 2, spacing=2.0)                     # at rest length: only damping acts
    p["velocity"][1] = (0.5, 0.3, 0)
    dt = 0.01
    cp = O.contact_params(dt, spawn_radius=100.0, global_drag=0.0)
    _, _, terms = O.contact_step_bonds(cp, p, _bond(O, 0, 1, rest=2.0, k=100.0, damp=5.0))
    Fd = 0.5 * 5.0                                    # dot(relVel, dir) · damping, along +x
    assert terms[0, 0] == pytest.approx(Fd * dt * SCALE, abs=1)
    assert terms[0, 4] == pytest.approx(-Fd * dt * SCALE, abs=1)


def test_relative_orientation_correction(oracle):
    """:541-582: B turned by θ about z against an identity rest orientation is turned back,
    A is turned toward it; both by ±(2·stiffness·dt)·θ/2."""
    O = oracle
    p = _parts(O, 2, spacing=2.0)
    th = 0.3
    p["rotation"][1] = (0, 0, math.sin(th / 2), math.cos(th / 2))
    dt, stiff = 0.01, 5.0
    cp = O.contact_params(dt, spawn_radius=100.0, global_drag=0.0, torque_damping=0.0)
    _, _, terms = O.contact_step_bonds(cp, p, _bond(O, 0, 1, k=0.0, stiff=stiff, enable=1))
    ocs = stiff * dt * 2.0
    # correction = conj(qB) -> axis (0,0,-1), angle θ
    angA, angB = -ocs * th * 0.5, ocs * th * 0.5
    rqA = np.array([0, 0, -math.sin(angA / 2), math.cos(angA / 2)])
    dqA = rqA - np.array([0, 0, 0, 1.0])              # quat_mul(rqA, identity) - identity
    c, s = math.cos(angB / 2), math.sin(angB / 2)
    qB = np.array([0, 0, math.sin(th / 2), math.cos(th / 2)])
    # quat_mul((0,0,-s,c), qB): both about z
    rB = np.array([0, 0, c * qB[2] + qB[3] * (-s), c * qB[3] - (-s) * qB[2]])
    dqB = rB - qB
    np.testing.assert_allclose(terms[0, 8:12], np.round(dqA * SCALE), atol=1)
    np.testing.assert_allclose(terms[0, 12:16], np.round(dqB * SCALE), atol=1)
    assert (terms[0, :8] == 0).all()                  # k = 0, at rest length: no Δv


def test_anchor_push_turns_anchor_toward_partner(oracle):
    """:462-514: A's anchor points along +y, B sits along +x: A is turned about +z-… so that the
    anchor swings toward B (rotAxis = rA × dir, angle = strength·|…|·5)."""
    O = oracle
    p = _parts(O, 2, spacing=4.0)
    dt, stiff = 0.01, 2.0
    cp = O.contact_params(dt, spawn_radius=100.0, global_drag=0.0, torque_damping=0.0)
    # anchors: A at +y (1 unit), B at its centre (zero length: no push on B)
    _, _, terms = O.contact_step_bonds(cp, p, _bond(O, 0, 1, k=0.0, rest=4.0, stiff=stiff, enable=1,
                                                     anc_a=(0, 1, 0), anc_b=(0, 0, 0)))
    anchor_delta = np.array([4.0, -1.0, 0.0])
    d = anchor_delta / np.linalg.norm(anchor_delta)
    rA = np.array([0, 1.0, 0])
    axis = np.cross(rA, d)
    axis /= np.linalg.norm(axis)
    eff = abs(np.dot(np.cross(axis, rA), d))
    ang = stiff * dt * eff * 5.0
    rq = np.array([*(axis * math.sin(ang / 2)), math.cos(ang / 2)])
    np.testing.assert_allclose(terms[0, 8:12], np.round((rq - [0, 0, 0, 1]) * SCALE), atol=1)
    assert axis[2] < 0                                # turning +y toward +x is about -z
    assert (terms[0, 12:16] == 0).all()


def test_invalid_bond_skipped_but_deltas_normalise(oracle):
    """:432 skips out-of-range indices; ApplyAdhesionDeltas still renormalises every rotation."""
    O = oracle
    p = _parts(O, 3)
    p["rotation"][2] = (0, 0, 0, 2.0)                 # not unit: ApplyAdhesionDeltas fixes it
    cp = O.contact_params(0.01, spawn_radius=100.0, global_drag=0.0, torque_damping=0.0)
    out, _, terms = O.contact_step_bonds(cp, p, _bond(O, 0, 7))
    assert (terms == 0).all()
    assert out["rotation"][2][3] == pytest.approx(1.0, abs=1e-7)
    out0, _ = O.contact_step(cp, p)                   # without bonds: untouched
    assert out0["rotation"][2][3] == 2.0


def test_no_bonds_equals_plain_step(oracle):
    O = oracle
    rng = np.random.default_rng(3)
    p = _parts(O, 64, spacing=0.5)
    p["velocity"] = rng.normal(size=(64, 3))
    cp = O.contact_params(0.01)
    a, ta = O.contact_step(cp, p)
    b, tb, _ = O.contact_step_bonds(cp, p, np.zeros(0, O.ADHESION84))
    assert a.tobytes() == b.tobytes() and np.array_equal(ta, tb)


def test_terms_order_independent(oracle):
    """int sums: shuffling the bond list changes no particle bit."""
    O = oracle
    from adhesion_cases import bonded_sphere
    parts, conns = bonded_sphere(O.PARTICLE84, O.ADHESION84, 512, seed=4)
    cp = O.contact_params(0.01)
    a, _, ta = O.contact_step_bonds(cp, parts, conns)
    perm = np.random.default_rng(0).permutation(len(conns))
    b, _, tb = O.contact_step_bonds(cp, parts, conns[perm])
    assert a.tobytes() == b.tobytes()
    assert np.array_equal(ta[perm], tb)
