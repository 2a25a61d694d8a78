"""GPU parity of the adhesion pass against the CPU oracle, through the C ABI.

Reference: ApplyAdhesionConstraints / ApplyAdhesionDeltas (SimulateParticles.compute:424-607),
dispatched between ApplySPHForces and the drag (ParticleSystemController.cs:284-310).
Bit-exact: the per-bond fixed-point terms (int32, ×1e6, round half to even) and the particle state
match the oracle exactly, because both sides round identically (no contraction; sin / cos / atan2 /
pow / exp in double, rounded once; see vec3.h and oracle/contact_oracle.c).
"""
import numpy as np
import pytest

from adhesion_cases import bonded_sphere

pytestmark = pytest.mark.gpu


def _check_terms(got, ref):
    diff = np.abs(got.astype(np.int64) - ref.astype(np.int64))
    assert diff.max() == 0, f"{(diff > 0).sum()} of {diff.size} terms differ (max {diff.max()})"


def _check_parts(got, ref):
    assert got.tobytes() == ref.tobytes()


class _Manager:
    """Stands in for CellAdhesionManager: GetAdhesionConnectionsForGPU() (CellAdhesionManager.cs:524)."""

    def __init__(self, conns):
        self.conns = conns

    def GetAdhesionConnectionsForGPU(self):
        return self.conns


@pytest.mark.parametrize("n", [256, 4096])
def test_adhesion_one_step(pkg, oracle, n):
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, n, seed=7)
    dt = 0.01
    conns = conns[:4096]                            # maxAdhesionConnections (controller:129,287)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.adhesionManager = _Manager(conns)
    ctl.Start(parts)
    ctl.Update(dt)
    got = ctl.GetParticles()
    terms = ctl.context.adhesion_terms()
    ref, tq_ref, terms_ref = oracle.contact_step_bonds(oracle.contact_params(dt), parts.view(oracle.PARTICLE84),
                                                       conns.view(oracle.ADHESION84))
    assert terms.shape == (len(conns), 16)
    assert np.abs(terms_ref).max() > 1000           # the case exercises every term
    _check_terms(terms, terms_ref)
    _check_parts(got, ref)
    assert np.array_equal(ctl.context.torque_int(), tq_ref)
    ctl.OnDestroy()


def test_adhesion_bond_order_bit_identical(pkg):
    """int sums in any order: a shuffled bond list gives the same particles bit for bit."""
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 2048, seed=8)
    out = []
    for perm in [np.arange(len(conns)), np.random.default_rng(1).permutation(len(conns))]:
        with pkg.Context(pkg.SPH_MODEL_CONTACT, 3, len(parts)) as ctx:
            ctx.upload_aos84(parts)
            ctx.set_adhesion(conns[perm])
            ctx.step(0.01, 3)
            out.append(ctx.download_aos84().tobytes())
    assert out[0] == out[1]


def test_adhesion_cap_and_removal(pkg, oracle):
    """maxAdhesionConnections caps the list (controller:287); an empty list disables the pass
    (no ApplyAdhesionDeltas renormalisation), exactly the plain step."""
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 1024, seed=9)
    parts["rotation"][5] = (0, 0, 0, 1.5)           # not unit: ApplyAdhesionDeltas renormalises it
    dt = 0.01
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    mgr = _Manager(conns)
    ctl.adhesionManager = mgr
    ctl.maxAdhesionConnections = 100
    ctl.Start(parts)
    ctl.Update(dt)
    ref, _, _ = oracle.contact_step_bonds(oracle.contact_params(dt), parts.view(oracle.PARTICLE84),
                                          conns[:100].view(oracle.ADHESION84))
    got = ctl.GetParticles()
    _check_parts(got, ref)
    mgr.conns = conns[:0]
    ctl.SetParticles(parts)
    ctl.Update(dt)
    plain, _ = oracle.contact_step(oracle.contact_params(dt), parts.view(oracle.PARTICLE84))
    got = ctl.GetParticles()
    _check_parts(got, plain)
    ctl.OnDestroy()


def test_adhesion_invalid_indices_and_inactive(pkg):
    """compute:432 skips out-of-range ends; bonds to inactive particles act on the active end
    only (ApplyAdhesionDeltas skips id >= activeParticleCount, :589)."""
    n, act = 600, 500
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, n, seed=10)
    bad = conns[:3].copy()
    bad["particleA"] = [-1, n, 5]
    bad["particleB"] = [3, 4, n + 10]
    allc = np.concatenate([conns, bad])
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.adhesionManager = _Manager(allc)
    ctl.Start(parts)
    ctl.activeParticleCount = act
    ctl.Update(0.01)
    terms = ctl.context.adhesion_terms()
    assert (terms[len(conns):] == 0).all()
    got = ctl.GetParticles()
    assert got[act:].tobytes() == parts[act:].tobytes()   # inactive: untouched
    cross = (conns["particleA"] >= act) ^ (conns["particleB"] >= act)
    assert cross.any() and (terms[:len(conns)][cross] != 0).any()
    ctl.OnDestroy()


def test_adhesion_long_run_invariants(pkg):
    parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 8192, seed=11)
    with pkg.Context(pkg.SPH_MODEL_CONTACT, 3, len(parts)) as ctx:
        ctx.upload_aos84(parts)
        ctx.set_adhesion(conns)
        ctx.step(0.005, 50)
        got = ctx.download_aos84()
    assert np.isfinite(got["position"]).all() and np.isfinite(got["velocity"]).all()
    assert (np.linalg.norm(got["position"], axis=1) <= 15.0 * (1 + 1e-5)).all()
    assert np.allclose(np.linalg.norm(got["rotation"], axis=1), 1.0, atol=1e-5)
    # bonded pairs are pulled toward their rest length (on average the spread shrinks)
    x = got["position"]
    L = np.linalg.norm(x[conns["particleB"]] - x[conns["particleA"]], axis=1)
    L0 = np.linalg.norm(parts["position"][conns["particleB"]] - parts["position"][conns["particleA"]], axis=1)
    err, err0 = np.abs(L - conns["restLength"]), np.abs(L0 - conns["restLength"])
    assert err.mean() < err0.mean() * 1.5


def test_drag_on_inactive_particle(pkg):
    """ApplyDragForce (compute:311-324) checks only particleBuffer.Length, so a selected inactive
    particle still gets the drag impulse; UpdateMotion (:329) then leaves it in place."""
    n, act = 300, 200
    parts, _ = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, n, seed=12)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ctl.activeParticleCount = act
    sel = 250
    ctl.drag.selectedID = sel
    ctl.drag.targetPosition = (3.0, -2.0, 1.0)
    ctl.drag.strength = 100.0
    ctl.Update(0.01)
    got = ctl.GetParticles()
    p = parts[sel]
    f32 = np.float32
    force = (np.array([3.0, -2.0, 1.0], f32) - p["position"]) * f32(100.0) * f32(0.01)
    np.testing.assert_allclose(got["velocity"][sel], p["velocity"] + force / p["mass"], rtol=1e-6)
    assert got["position"][sel].tobytes() == p["position"].tobytes()
    keep = np.ones(n - act, bool)
    keep[sel - act] = False
    assert got[act:][keep].tobytes() == parts[act:][keep].tobytes()
    ctl.OnDestroy()


def test_gpu_vs_golden_adhesion(pkg):
    """The committed oracle fixture (tests/golden/adhesion_n512_s1.npz, make_golden.py)."""
    from pathlib import Path
    d = np.load(Path(__file__).resolve().parent / "golden" / "adhesion_n512_s1.npz")
    inp = d["input"].view(pkg.PARTICLE84)
    conns = d["conns"].view(pkg.ADHESION84)
    ref = d["output"].view(pkg.PARTICLE84)
    ctl = pkg.ParticleSystemController(particleCount=len(inp))
    ctl.globalDragMultiplier = 10.0
    ctl.adhesionManager = _Manager(conns)
    ctl.Start(inp)
    ctl.Update(0.01)
    _check_terms(ctl.context.adhesion_terms(), d["terms"])
    _check_parts(ctl.GetParticles(), ref)
    ctl.OnDestroy()
