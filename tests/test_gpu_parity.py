"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances (SPEC_SPH.md §1-2):
  * integer / index work (cell keys, radix-sort permutation, cell_start, sorted ids): bit-exact;
  * Model S after 1 step: ρ rtol 1e-5 (the strict per-pass bounds are in test_gpu_parity_headline.py); x atol 1e-6 (·1 m); v atol 1e-4·c0·dt·max(1,|a|dt) —
    differences come from fp contraction and v_sqrt/v_rcp rounding, not the summation order,
    which is the same §0 order on both sides;
  * Model R after 1 step: v, ω rtol 1e-4 (+atol), x rtol 1e-5; int torque sums exact except
    when a per-pair float lies within an ulp of an integer boundary (counted and bounded).
"""
import numpy as np
import pytest

from conftest import oracle_sph_params

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ sort / grid
@pytest.mark.parametrize("n,bits", [(1, 8), (2047, 8), (2048, 15), (2049, 16), (5000, 12), (16_384, 16),
                                    (16_385, 16), (100_000, 20), (1_048_576, 20), (333_333, 24), (65_536, 32)])
def test_radix_sort_bit_exact(pkg, n, bits):
    rng = np.random.default_rng(n + bits)
    keys = rng.integers(0, 2 ** bits, n, dtype=np.uint64).astype(np.uint32)
    with pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 16) as ctx:
        perm, sk = ctx.radix_sort(keys, bits)
    ref = np.argsort(keys, kind="stable")
    assert np.array_equal(perm, ref)
    assert np.array_equal(sk, keys[ref])


@pytest.mark.parametrize("n,hi", [(16_384, 7), (4096, 32_769), (1000, 1)])
def test_radix_sort_small_ties(pkg, n, hi):
    """The one-workgroup sort (n <= 16,384, keys <= 16 bits): long runs of equal keys keep their
    index order, and Model R's sentinel key 32,768 sorts last."""
    rng = np.random.default_rng(n)
    keys = rng.integers(0, hi, n).astype(np.uint32)
    with pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 16) as ctx:
        perm, sk = ctx.radix_sort(keys, 16)
    ref = np.argsort(keys, kind="stable")
    assert np.array_equal(perm, ref)
    assert np.array_equal(sk, keys[ref])


def test_radix_sort_nearly_sorted_and_ties(pkg):
    """The step's real input: the previous step's order with a few keys changed."""
    rng = np.random.default_rng(3)
    keys = np.sort(rng.integers(0, 600_000, 500_000)).astype(np.uint32)
    flip = rng.integers(0, len(keys), 5000)
    keys[flip] += rng.integers(-3, 4, len(flip)).astype(np.int64).clip(0).astype(np.uint32)
    keys[:1000] = 7                              # long run of ties
    with pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 16) as ctx:
        perm, _ = ctx.radix_sort(keys, 20)
    assert np.array_equal(perm, np.argsort(keys, kind="stable"))


# ------------------------------------------------------------------ Model S
def _sim_and_oracle(pkg, oracle, name_or_sc):
    sc = pkg.config_scenario(name_or_sc) if isinstance(name_or_sc, str) else name_or_sc
    sim = pkg.SPHSim(sc)
    op = oracle_sph_params(oracle, sim.params, sc.dim)
    return sim, op


def test_lattice_init_bit_exact(pkg, oracle):
    sim, _ = _sim_and_oracle(pkg, oracle, "C1")
    x = sim.positions()
    ref = oracle.lattice(2, 64, 64, 1, 0.01, seed=1234)
    assert np.array_equal(x, ref)
    sim.close()
    sc = pkg.make_scenario(0, 3, 9, 7, 5, 32, 32, 32, seed=77)
    sim = pkg.SPHSim(sc)
    assert np.array_equal(sim.positions(), oracle.lattice(3, 9, 7, 5, 0.01, seed=77))
    sim.close()


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_wcsph_one_step(pkg, oracle, cfg):
    sim, op = _sim_and_oracle(pkg, oracle, cfg)
    x0 = sim.positions()
    n = len(x0)
    sim.step(1)
    xg, vg, rg = sim.positions(), sim.velocities(), sim.density()
    ids_g = sim.ctx.sorted_ids()
    cs_g = sim.ctx.cell_start()
    xo, vo, io, ro, _, cso = oracle.sph_step(op, x0, np.zeros_like(x0), np.arange(n, dtype=np.int32), sim.dt, 0.0)
    # integer work: identical sort permutation and cell table
    assert np.array_equal(ids_g, io)
    assert np.array_equal(cs_g, cso)
    order = np.argsort(io)
    np.testing.assert_allclose(rg, ro[order], rtol=1e-5, atol=0)
    np.testing.assert_allclose(xg, xo[order], rtol=0, atol=1e-6)
    vscale = float(sim.params.c0) * sim.dt * 10
    np.testing.assert_allclose(vg, vo[order], rtol=1e-3, atol=1e-4 * vscale)
    sim.close()


def test_wcsph_ten_steps_c1(pkg, oracle):
    sim, op = _sim_and_oracle(pkg, oracle, "C1")
    x = sim.positions()
    n = len(x)
    v = np.zeros_like(x)
    ids = np.arange(n, dtype=np.int32)
    for s in range(10):
        x, v, ids, rho, _, _ = oracle.sph_step(op, x, v, ids, sim.dt, np.float32(s * sim.dt))
    sim.step(10)
    order = np.argsort(ids)
    np.testing.assert_allclose(sim.positions(), x[order], rtol=0, atol=2e-6)
    np.testing.assert_allclose(sim.density(), rho[order], rtol=2e-4)
    sim.close()


def test_wcsph_sloshing_forcing(pkg, oracle):
    """C4-shaped (scaled down) sloshing: the lateral forcing term f_ext(t)."""
    sc = pkg.make_scenario(1, 3, 32, 8, 16, 32, 16, 16)
    sim, op = _sim_and_oracle(pkg, oracle, sc)
    assert sim.params.forcing_amp > 0
    x = sim.positions()
    v = np.zeros_like(x)
    ids = np.arange(len(x), dtype=np.int32)
    for s in range(3):
        x, v, ids, _, _, _ = oracle.sph_step(op, x, v, ids, sim.dt, np.float32(s * sim.dt))
    sim.step(3)
    order = np.argsort(ids)
    np.testing.assert_allclose(sim.velocities(), v[order], rtol=1e-3, atol=1e-3)
    sim.close()


def test_wcsph_c3_invariants(pkg):
    """Full C3 size (1,048,576): size-independent properties over 20 steps."""
    sim = pkg.SPHSim.from_config("C3")
    n = sim.n
    assert n == 1_048_576
    sim.step(20)
    x, v, rho = sim.positions(), sim.velocities(), sim.density()
    box = np.array(sim.params.box)
    assert np.isfinite(x).all() and np.isfinite(v).all() and np.isfinite(rho).all()
    assert (x >= 0).all() and (x <= box).all()
    ids = sim.ctx.sorted_ids()
    assert np.array_equal(np.sort(ids), np.arange(n))        # a permutation: no particle lost
    cs = sim.ctx.cell_start()
    assert cs[0] == 0 and cs[-1] == n and np.all(np.diff(cs.astype(np.int64)) >= 0)
    assert 500 < np.median(rho) < 1100
    sim.close()


@pytest.mark.parametrize("cfg,steps", [("C4", 10), ("C5", 4)])
def test_wcsph_full_size_configs(pkg, cfg, steps):
    """BASELINE.json's multi-GPU configs at full size on one GPU (4,194,304 sloshing, 16,777,216
    dam-break): finite, in the box, no particle lost, sorted cell table, sane density."""
    sim = pkg.SPHSim.from_config(cfg)
    n = sim.n
    assert n == {"C4": 4_194_304, "C5": 16_777_216}[cfg]
    if cfg == "C4":
        assert sim.params.forcing_amp > 0
    sim.step(steps)
    x, v, rho = sim.positions(), sim.velocities(), sim.density()
    box = np.array(sim.params.box)
    assert np.isfinite(x).all() and np.isfinite(v).all() and np.isfinite(rho).all()
    assert (x >= 0).all() and (x <= box).all()
    ids = sim.ctx.sorted_ids()
    assert np.array_equal(np.sort(ids), np.arange(n))
    cs = sim.ctx.cell_start()
    assert cs[0] == 0 and cs[-1] == n and np.all(np.diff(cs.astype(np.int64)) >= 0)
    assert 500 < np.median(rho) < 1100
    sim.close()


def test_wcsph_upload_state_and_empty(pkg, oracle):
    sc = pkg.config_scenario("C1")
    p, dt = pkg.scenario_params(sc)
    with pkg.Context(pkg.SPH_MODEL_WCSPH, 2, 100) as ctx:
        ctx.set_params(p)
        ctx.upload_state(np.zeros((0, 3), np.float32))
        ctx.step(dt, 3)                                 # empty: a no-op, not an error
        x = np.array([[0.3, 0.3, 0.0]], np.float32)
        ctx.upload_state(x, np.zeros_like(x))
        ctx.step(dt, 1)
        assert ctx.positions()[0][1] == pytest.approx(0.3 - 9.81 * dt * dt, rel=1e-6)
        from sph_test_amd import _abi as A
        with pytest.raises(A.SphError) as e:
            ctx.upload_state(np.zeros((101, 3), np.float32))
        assert e.value.status == A.SPH_ERR_CAPACITY


# ------------------------------------------------------------------ Model R
def random_sphere(PARTICLE84, n, seed=1234, R=15.0):
    """SURVEY §8c fixture recipe: positions in a sphere, radii U[1.5,2], v,ω ~ N(0,1), q = identity."""
    rng = np.random.default_rng(seed)
    p = np.zeros(n, PARTICLE84)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    p["position"] = d * (R * rng.random((n, 1)) ** (1 / 3))
    p["radius"] = rng.uniform(1.5, 2.0, n)
    p["velocity"] = rng.normal(size=(n, 3))
    p["mass"] = 0.1 * 4.0 / 3.0 * 3.1415926 * p["radius"] ** 3
    p["angularVelocity"] = rng.normal(size=(n, 3))
    p["momentOfInertia"] = 0.4 * p["mass"] * p["radius"] ** 2
    p["drag"] = rng.uniform(0.5, 1.0, n)
    p["repulsionStrength"] = 1.0
    p["rotation"] = (0, 0, 0, 1)
    p["modeIndex"] = -1
    return p


def test_aos84_round_trip_bit_exact(pkg):
    parts = random_sphere(pkg.PARTICLE84, 1000)
    parts["genomeFlags"] = np.arange(1000)
    parts["modeIndex"] = np.arange(1000) % 7
    with pkg.Context(pkg.SPH_MODEL_CONTACT, 3, 1000) as ctx:
        ctx.upload_aos84(parts)
        back = ctx.download_aos84()
    assert back.tobytes() == parts.tobytes()


@pytest.mark.parametrize("n,steps", [(64, 1), (4096, 1), (32768, 1), (262_144, 1), (4096, 10), (32768, 5)])
def test_contact_bit_exact(pkg, oracle, n, steps):
    """Model R against the C restatement, BIT-EXACT: the same roundings on both sides (no contraction,
    pow / exp / sin / cos evaluated in double and rounded once, serial-order sums, int torque gather).
    262,144 particles in R = 15 is the SURVEY §8c stress case (~30,000 candidates per particle).
    Over several steps the neighbour visit order depends on the tie order of the stable sort (the
    previous step's slots, SPEC_SPH.md §0), so the oracle gets its input in the GPU's slot order."""
    parts = random_sphere(pkg.PARTICLE84, n)
    dt = 0.01
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ref = parts.view(oracle.PARTICLE84).copy()
    order = np.arange(n)
    for _ in range(steps):
        out, tq_slot = oracle.contact_step(oracle.contact_params(dt), ref[order])
        ref[order] = out
        tq_ref = np.empty_like(tq_slot)
        tq_ref[order] = tq_slot
        ctl.Update(dt)
        order = ctl.context.sorted_ids()
    got = ctl.GetParticles()
    assert np.array_equal(ctl.context.torque_int(), tq_ref)
    assert got.tobytes() == ref.tobytes()
    ctl.OnDestroy()


@pytest.mark.parametrize("case", ["outside", "big_radius", "shrink"])
def test_contact_cell_skipping_edge_states(pkg, oracle, case):
    """The contact pass skips the cells of its 27 that lie beyond rA/2 + rmax/2 (contact.hip cell_reach / reach_row, r6);
    the oracle scans all 27 (SimulateParticles.compute:228-233), so any wrongly skipped contact shows as a bit difference.
    The states where the bound could go wrong: particles far outside the 128-unit grid, clamped into its edge cells
    (there the per-axis bound only grows), a few of them touching each other there; one radius far above the rest (the
    bound then skips little); radii shrunk between steps by a range write (the bound must follow on the full sort the
    write forces, and a too-small stale bound would drop contacts of the grown ones: here the first 1,000 shrink and
    the next 200 grow). Bit-exact over several steps, the oracle fed in the GPU's slot order."""
    n = 4096
    parts = random_sphere(pkg.PARTICLE84, n, seed=77)
    if case == "outside":
        rng = np.random.default_rng(3)
        parts["position"][:200] *= 6.0                                                   # spread far outside the grid
        parts["position"][200:260] = (-40.0, -40.0, -40.0) + rng.uniform(-1.5, 1.5, (60, 3))   # a clamped cluster
        parts["position"][260:320] = (60.0, 9.0, -1.0) + rng.uniform(-1.5, 1.5, (60, 3))      # beyond +x, in contact
    if case == "big_radius":
        parts["radius"][5] = 12.0
        parts["mass"][5] = 0.1 * 4.0 / 3.0 * 3.1415926 * 12.0 ** 3
        parts["momentOfInertia"][5] = 0.4 * parts["mass"][5] * 144.0
    dt = 0.01
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ref = parts.view(oracle.PARTICLE84).copy()
    order = np.arange(n)
    for s in range(6):
        if case == "shrink" and s == 3:
            cur = ctl.context.get_particles(0, 1200)
            cur["radius"][:1000] *= np.float32(0.5)
            cur["radius"][1000:1200] *= np.float32(1.6)
            ctl.context.set_particles(0, cur)
            ref_idx = ref.copy()
            ref_idx["radius"][:1000] *= np.float32(0.5)
            ref_idx["radius"][1000:1200] *= np.float32(1.6)
            ref = ref_idx
        out, tq_slot = oracle.contact_step(oracle.contact_params(dt), ref[order])
        ref[order] = out
        tq_ref = np.empty_like(tq_slot)
        tq_ref[order] = tq_slot
        ctl.Update(dt)
        order = ctl.context.sorted_ids()
    got = ctl.GetParticles()
    assert np.array_equal(ctl.context.torque_int(), tq_ref), case
    assert got.tobytes() == ref.tobytes(), case
    ctl.OnDestroy()


def test_contact_drag_and_inactive(pkg, oracle):
    n = 2000
    parts = random_sphere(pkg.PARTICLE84, n, seed=5)
    act = 1500
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ctl.activeParticleCount = act
    ctl.drag.selectedID = 17
    ctl.drag.targetPosition = (3.0, -2.0, 1.0)
    ctl.drag.strength = 100.0
    ctl.Update(0.01)
    got = ctl.GetParticles()
    cp = oracle.contact_params(0.01, drag_id=17, drag_target=(3.0, -2.0, 1.0), drag_strength=100.0)
    ref, _ = oracle.contact_step(cp, parts[:act].view(oracle.PARTICLE84))
    assert got[:act].tobytes() == ref.tobytes()                  # bit-exact, drag included
    assert got[act:].tobytes() == parts[act:].tobytes()     # inactive particles untouched
    ctl.OnDestroy()


def test_contact_long_run_invariants(pkg):
    n = 10000
    parts = random_sphere(pkg.PARTICLE84, n, seed=9)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    for _ in range(50):
        ctl.Update(0.005)
    got = ctl.GetParticles()
    assert np.isfinite(got["position"]).all() and np.isfinite(got["angularVelocity"]).all()
    r = np.linalg.norm(got["position"], axis=1)
    assert (r <= 15.0 * (1 + 1e-5)).all()
    qn = np.linalg.norm(got["rotation"], axis=1)
    assert np.allclose(qn, 1.0, atol=1e-5)
    ctl.OnDestroy()


def test_contact_resize_keeps_state(pkg):
    n = 300
    parts = random_sphere(pkg.PARTICLE84, n, seed=11)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ctl.Update(0.01)
    before = ctl.GetParticles()
    ctl.ResizeParticleBuffers(1000)
    assert ctl.GetParticles().tobytes() == before.tobytes()
    ctl.Update(0.01)
    ctl.OnDestroy()


# ------------------------------------------------------------------ committed fixtures
def test_gpu_vs_golden_wcsph_c1(pkg):
    from pathlib import Path
    d = np.load(Path(__file__).resolve().parent / "golden" / "wcsph_c1_s10.npz")
    sim = pkg.SPHSim.from_config("C1")
    assert np.array_equal(sim.positions(), d["x0"])
    sim.step(10)
    np.testing.assert_allclose(sim.positions(), d["x"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(sim.density(), d["rho"], rtol=2e-4)
    sim.close()


def test_gpu_vs_golden_contact_n4096(pkg):
    from pathlib import Path
    d = np.load(Path(__file__).resolve().parent / "golden" / "contact_n4096_s1.npz")
    inp = d["input"].view(pkg.PARTICLE84)
    ref = d["output"].view(pkg.PARTICLE84)
    ctl = pkg.ParticleSystemController(particleCount=len(inp))
    ctl.globalDragMultiplier = 10.0
    ctl.Start(inp)
    ctl.Update(0.01)
    got = ctl.GetParticles()
    assert np.array_equal(ctl.context.torque_int(), d["torque"])
    assert got.tobytes() == ref.tobytes()
    ctl.OnDestroy()
