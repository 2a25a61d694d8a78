"""Known-answer tests pinning the CPU oracle to the reference's arithmetic.

The reference has no tests or golden vectors, and its HLSL cannot run here.
These cases are therefore derived by hand from the HLSL text
(/root/reference/Assets/Compute/SimulateParticles.compute) and from SPEC_SPH.md, evaluated
in float64 numpy, and compared with the oracle's fp32 output.
"""
import math

import numpy as np
import pytest


def _parts(O, n):
    p = np.zeros(n, O.PARTICLE84)
    p["rotation"] = (0, 0, 0, 1)
    p["radius"] = 2.0
    p["mass"] = 1.0
    p["momentOfInertia"] = 1.0
    p["drag"] = 1.0
    return p


# ------------------------------------------------------------------ Model R
def test_contact_head_on_repulsion(oracle):
    """compute:248-261 + :302-305 + UpdateMotion :332-337 for one overlapping pair."""
    O = oracle
    p = _parts(O, 2)
    p["position"][1] = (1.5, 0, 0)
    dt = 0.01
    cp = O.contact_params(dt, spawn_radius=15.0, global_drag=1.0, repulsion_strength=200.0)
    out, tq = O.contact_step(cp, p)
    # eff radii 1 + 1 = 2, dist 1.5, overlap 0.5; overlapFalloff = 0.25, falloff = 0.25
    F = 200.0 * 0.25 * 0.25                       # along dir = (posA - posB)/dist
    damp = math.exp(-1.0 * 1.0 * dt)
    vA = -F / 1.0 * dt * damp
    vB = +F / 1.0 * dt * damp
    assert out["velocity"][0][0] == pytest.approx(vA, rel=1e-6)
    assert out["velocity"][1][0] == pytest.approx(vB, rel=1e-6)
    assert out["position"][0][0] == pytest.approx(vA * dt, rel=1e-6)
    assert out["position"][1][0] == pytest.approx(1.5 + vB * dt, rel=1e-6)
    assert np.all(tq == 0)                        # no slip -> no rolling torque (:274)
    assert np.all(out["angularVelocity"] == 0)


def test_contact_no_contact_below_threshold(oracle):
    """overlap must exceed 0.001 (compute:253)."""
    O = oracle
    p = _parts(O, 2)
    p["position"][1] = (1.9995, 0, 0)             # overlap 0.0005
    out, _ = O.contact_step(O.contact_params(0.01), p)
    assert np.all(out["velocity"] == 0)


def test_contact_rolling_friction_and_int_reaction(oracle):
    """Rolling-contact friction (compute:263-294): slip from relative tangential velocity,
    |slip|^1.25 friction, overlapFalloff² torque radius, truncated int3 reaction ×1e4."""
    O = oracle
    p = _parts(O, 2)
    p["position"][1] = (1.5, 0, 0)
    p["velocity"][0] = (0, 1.0, 0)                # A slides along +y relative to B
    dt = 0.01
    cp = O.contact_params(dt, global_drag=0.0, torque_damping=0.0, roll_mult=5.0, torque_factor=1.0)
    out, tq = O.contact_step(cp, p)
    # dir from A's thread = (-1,0,0); slip = (0,1,0) (velocity along y is tangential)
    of = 0.25
    erA = of * of * 1.0 * 5.0
    fmag = 1.0 ** 1.25
    # rollingTorqueA = cross(-dir*erA, -fdir*fmag) = cross((erA,0,0), (0,-1,0)) = (0,0,-erA)
    tauA = np.array([0.0, 0.0, -erA * fmag])
    # B's thread: dir = (+1,0,0), relative slip = (0,-1,0)
    # rollingTorqueB (scattered to A) = cross(dir*erA', fdir*fmag) = cross((erA,0,0),(0,-1,0)) = (0,0,-erA)
    reactA = np.array([0.0, 0.0, -erA * fmag])
    iA = np.trunc(reactA * dt * 10000.0).astype(np.int64)
    assert tq[0].tolist() == iA.tolist()
    # ω_A = τ_A/I·dt + (int τ/1e4)/I   (damping 0)
    expect_w = tauA * dt + iA / 10000.0
    assert np.allclose(out["angularVelocity"][0], expect_w, rtol=1e-5, atol=1e-7)


def test_contact_sphere_boundary_reflect(oracle):
    """UpdateMotion sphere boundary (compute:339-354): project, reflect, friction torque."""
    O = oracle
    p = _parts(O, 1)
    p["position"][0] = (14.99, 0, 0)
    p["velocity"][0] = (10.0, 1.0, 0.0)
    dt = 0.01
    cp = O.contact_params(dt, spawn_radius=15.0, global_drag=0.0, torque_damping=0.0,
                          boundary_friction=0.8, roll_mult=5.0)
    out, _ = O.contact_step(cp, p)
    x = np.array([14.99 + 0.1, 0.01, 0.0])
    n = x / np.linalg.norm(x)
    v = np.array([10.0, 1.0, 0.0])
    v = v - 2 * np.dot(v, n) * n
    assert np.allclose(out["position"][0], n * 15.0, rtol=1e-6)
    assert np.allclose(out["velocity"][0], v, rtol=1e-5)
    t = v - np.dot(v, n) * n
    fdir = (t + 1e-6) / np.linalg.norm(t + 1e-6)
    torque = np.cross(-n * 2.0 * 5.0, -fdir * np.linalg.norm(t) * 0.8)
    assert np.allclose(out["angularVelocity"][0], torque * dt, rtol=1e-4, atol=1e-6)


def test_contact_rotation_integration(oracle):
    """UpdateRotation (compute:385-406): damping then dq(ω·dt)⊗q, normalised."""
    O = oracle
    p = _parts(O, 1)
    p["angularVelocity"][0] = (0, 0, 2.0)
    dt = 0.05
    cp = O.contact_params(dt, global_drag=0.0, torque_damping=0.5)
    out, _ = O.contact_step(cp, p)
    w = 2.0 * math.exp(-0.5 * dt) * math.exp(-0.5 * dt)     # UpdateMotion + UpdateRotation damping
    ang = w * dt
    assert out["angularVelocity"][0][2] == pytest.approx(w, rel=1e-6)
    assert np.allclose(out["rotation"][0], (0, 0, math.sin(ang / 2), math.cos(ang / 2)), atol=1e-6)


def test_contact_drag_input(oracle):
    """ApplyDragForce (compute:316-323) applies to the selected particle only."""
    O = oracle
    p = _parts(O, 2)
    p["position"][1] = (10, 0, 0)
    dt = 0.01
    cp = O.contact_params(dt, global_drag=0.0, drag_id=1, drag_target=(10, 5, 0), drag_strength=100.0)
    out, _ = O.contact_step(cp, p)
    assert np.all(out["velocity"][0] == 0)
    assert out["velocity"][1][1] == pytest.approx(5 * 100.0 * dt / 1.0, rel=1e-6)


def test_contact_grid_clamp_neighbours(oracle):
    """Out-of-grid positions clamp into edge cells (compute:104); pairs there still interact."""
    O = oracle
    p = _parts(O, 2)
    p["position"][0] = (-40.0, 0, 0)
    p["position"][1] = (-41.5, 0, 0)
    out, _ = O.contact_step(O.contact_params(0.001, spawn_radius=100.0, global_drag=0.0), p)
    assert out["velocity"][0][0] > 0 and out["velocity"][1][0] < 0


# ------------------------------------------------------------------ Model S
def _sph(O, dim=3, L=(1.0, 1.0, 1.0)):
    dx = 0.01
    h = 1.2 * dx
    return O.sph_params(dim, dx, h, 1000.0, 20.0, 0.02, 0.5, (0, -9.81, 0), L, 0.5)


def test_sph_isolated_particle(oracle):
    """ρ = m·W(0) = m·σ, Tait P, and a pure-gravity kick-drift (SPEC_SPH.md §2)."""
    O = oracle
    p = _sph(O)
    x = np.array([[0.5, 0.5, 0.5]], np.float32)
    v = np.array([[0.1, 0.0, 0.0]], np.float32)
    dt = 1e-4
    xo, vo, _, rho, prho, _ = O.sph_step(p, x, v, np.array([0], np.int32), dt)
    h = 0.012
    sigma = 1 / (math.pi * h ** 3)
    m = 1000 * 0.01 ** 3
    assert rho[0] == pytest.approx(m * sigma, rel=1e-6)
    B = 20.0 ** 2 * 1000 / 7
    P = B * ((m * sigma / 1000) ** 7 - 1)
    assert prho[0] == pytest.approx(P / (m * sigma) ** 2, rel=1e-5)
    assert vo[0][1] == pytest.approx(-9.81 * dt, rel=1e-6)
    assert xo[0][0] == pytest.approx(0.5 + 0.1 * dt, rel=1e-7)
    assert xo[0][1] == pytest.approx(0.5 - 9.81 * dt * dt, rel=1e-7)


def test_sph_pair_momentum_and_kernel(oracle):
    """Two particles: W(q), symmetric pressure force (Newton's third law) and XSPH."""
    O = oracle
    p = _sph(O)
    r = 0.015                                   # q = 1.25
    x = np.array([[0.5, 0.5, 0.5], [0.5 + r, 0.5, 0.5]], np.float32)
    v = np.zeros_like(x)
    dt = 1e-5
    p.g[1] = 0.0
    xo, vo, ids, rho, prho, _ = O.sph_step(p, x, v, np.array([0, 1], np.int32), dt)
    h = 0.012
    sigma = 1 / (math.pi * h ** 3)
    q = r / h
    W = sigma * 0.25 * (2 - q) ** 3
    m = 1e-3
    assert np.allclose(rho, m * (sigma + W), rtol=1e-6)
    # equal and opposite accelerations (same mass)
    order = np.argsort(ids)
    assert vo[order][0][0] == pytest.approx(-vo[order][1][0], rel=1e-6)
    F = -sigma / h * 0.75 * (2 - q) ** 2 / r
    a0 = -m * (2 * prho[0]) * F * (-r)
    assert vo[order][0][0] == pytest.approx(a0 * dt, rel=1e-4)


def test_sph_diag_support_edge_conditioning(oracle):
    """The diagnostics' conditioning columns (oracle.h or_sph_step_diag): a pair at q = 1.99 has
    Q = 2·S·δq/(2 − q) and Q_x = 3·(XSPH scale)·δq/(2 − q) with δq = 2^-21, and a pair at q < 1 has none; the
    rounding of q by that δq moves the pair's acceleration term by at most Q (finite difference, float64)."""
    O = oracle
    p = _sph(O)
    p.g[1] = 0.0
    h = 0.012
    dq = 2.0 ** -21
    for q, cond in ((1.99, True), (0.7, False)):
        x = np.array([[0.5, 0.5, 0.5], [0.5 + q * h, 0.5, 0.5]], np.float32)
        v = np.array([[0.0, 0.0, 0.0], [0.0, 0.3, 0.0]], np.float32)
        *_, mag = O.sph_step_diag(p, x, v, np.array([0, 1], np.int32), 1e-5)
        assert mag.shape == (2, 5)
        for k in range(2):
            S, Sx, _, Q, Qx = (float(c) for c in mag[k])
            if cond:
                t = 2.0 - float(np.sqrt(np.float64((x[1, 0] - x[0, 0]) ** 2))) / float(np.float32(h))
                assert Q == pytest.approx(2 * S * dq / t, rel=1e-5)
                assert Qx == pytest.approx(3 * Sx * dq / t, rel=1e-5)
                # the pair term is ∝ t²: a q moved by dq moves it by ≈ 2·dq/t of itself
                assert abs((t - dq) ** 2 - t ** 2) / t ** 2 * S <= Q * (1 + 1e-3)
            else:
                assert Q == 0.0 and Qx == 0.0


def test_sph_walls_clamp_and_restitution(oracle):
    O = oracle
    p = _sph(O, L=(1.0, 1.0, 1.0))
    p.g[1] = 0.0
    x = np.array([[0.0001, 0.5, 0.5]], np.float32)
    v = np.array([[-10.0, 0, 0]], np.float32)
    xo, vo, _, _, _, _ = O.sph_step(p, x, v, np.array([0], np.int32), 1e-3)
    assert xo[0][0] == 0.0
    assert vo[0][0] == pytest.approx(5.0, rel=1e-6)     # e = 0.5


def test_grid_sort_and_cell_start(oracle):
    """Stable sort == numpy stable argsort; cell_start == searchsorted(left)."""
    O = oracle
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 1000, 5000).astype(np.uint32)
    perm = O.stable_sort(keys, 1000)
    assert np.array_equal(perm, np.argsort(keys, kind="stable"))
    cs = O.cell_start(keys[perm], 1000)
    assert np.array_equal(cs, np.searchsorted(keys[perm], np.arange(1001), side="left"))


def test_grid_keys_clamp(oracle):
    O = oracle
    p = _sph(O, L=(0.24, 0.24, 0.24))            # cell 0.024 -> 11 cells in x, y; z sub-cells 0.004 -> 60
    G = list(p.grid.G)                           # (0.24f / 0.004f rounds just below 60: floor 59, + 1)
    assert G == [11, 11, 60]
    pos = np.array([[-1, -1, -1], [0.0, 0.0, 0.0], [0.0241, 0.0, 0.0], [5, 5, 5], [np.nan, 0, 0],
                    [0.0, 0.0, 0.0061]], np.float32)
    k = O.grid_keys(p, pos)
    xs = int(p.grid.xsub)                        # x sub-columns per column (SPH_XSUB): keys count them
    assert k.tolist() == [0, 0, xs * 11 * 60, (11 * xs - 1) * 11 * 60 + 10 * 60 + 59, 0, 1]


def test_lattice_deterministic_and_bounded(oracle):
    O = oracle
    a = O.lattice(3, 8, 4, 2, 0.01)
    b = O.lattice(3, 8, 4, 2, 0.01)
    assert np.array_equal(a, b)
    ix = np.arange(64) % 8
    assert np.all(np.abs(a[:, 0] - (ix + 0.5) * 0.01) <= 0.0001 + 1e-9)
    c = O.lattice(3, 8, 4, 2, 0.01, seed=99)
    assert not np.array_equal(a, c)
