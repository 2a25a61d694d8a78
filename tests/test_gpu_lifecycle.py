"""GPU parity of the Model R particle lifecycle against the oracle, through the C ABI.

InitParticles (compute:118-194): bit-exact (both sides take the HLSL sin / pow as the correctly
rounded float value and contract nothing); a double-precision sin that lands within one double
ulp of a float rounding boundary could flip one value, so the test allows 1e-4 of the particles.
Splits (controller:832-959), index-range get/set and device-side resizes are data movement:
bit-exact.
"""
import numpy as np
import pytest

from shipped_scene import shipped_controller

pytestmark = pytest.mark.gpu


def _ctx(pkg, cap):
    return pkg.Context(pkg.SPH_MODEL_CONTACT, 3, cap)


@pytest.mark.parametrize("n,modes,default", [(1, 0, 0), (4096, 0, 0), (65536, 3, 1), (1048576, 5, 4)])
def test_init_particles_bit_exact(pkg, oracle, n, modes, default):
    with _ctx(pkg, n) as ctx:
        ctx.init_particles(n, n, modes, default)
        got = ctx.download_aos84()
    ref = oracle.init_particles(n, n, genome_modes=modes, default_mode=default)
    bad = np.frombuffer(got.tobytes(), np.uint8).reshape(n, 84) != np.frombuffer(ref.tobytes(), np.uint8).reshape(n, 84)
    assert bad.any(axis=1).mean() <= 1e-4, f"{bad.any(axis=1).sum()} particles differ"


def test_init_particles_partial_active(pkg, oracle):
    n, act = 1000, 1
    with _ctx(pkg, 2000) as ctx:
        ctx.init_particles(n, act)
        assert ctx.get_params().active_particle_count == act
        got = ctx.download_aos84()
    assert got.tobytes() == oracle.init_particles(n, act).tobytes()


def _random_splits(pkg, rng, parents):
    sp = np.zeros(len(parents), pkg.SPLIT92)
    sp["parentIndex"] = parents
    for f in ["positionA", "positionB", "velocityA", "velocityB"]:
        sp[f] = rng.normal(size=(len(parents), 3))
    for f in ["rotationA", "rotationB"]:
        q = rng.normal(size=(len(parents), 4))
        sp[f] = q / np.linalg.norm(q, axis=1, keepdims=True)
    sp["childAModeIndex"] = rng.integers(0, 5, len(parents))
    sp["childBModeIndex"] = rng.integers(0, 5, len(parents))
    return sp


@pytest.mark.parametrize("cap,n,act,k", [(5000, 5000, 3000, 700), (4096, 4096, 4000, 500), (64, 8, 8, 8)])
def test_split_matches_oracle(pkg, oracle, cap, n, act, k):
    """After a few steps (cell-sorted slots), splits overwrite parents and fill index active+k;
    past the capacity the device grows to max(need, 2·capacity) (controller:788-792)."""
    rng = np.random.default_rng(cap + k)
    with _ctx(pkg, cap) as ctx:
        ctx.init_particles(n, act)
        p = ctx.get_params()
        p.active_particle_count = act
        ctx.set_params(p)
        ctx.step(0.01, 3)
        before = ctx.download_aos84()
        sp = _random_splits(pkg, rng, rng.choice(act, size=k, replace=False))
        new_act = ctx.split_particles(sp)
        st = ctx.stats()
        got = ctx.download_aos84()
        assert new_act == act + k == ctx.get_params().active_particle_count
        if act + k > cap:
            assert st.capacity == max(act + k, 2 * cap)
        ctx.step(0.01, 2)                                  # the grown state steps
        assert np.isfinite(ctx.download_aos84()["position"]).all()
    ref, ref_act = oracle.split_particles(before.view(oracle.PARTICLE84), act, sp.view(oracle.SPLIT92))
    assert ref_act == new_act
    assert got.tobytes() == ref[: len(got)].tobytes()
    assert len(got) == max(n, act + k)


def test_split_rejects_bad_parents(pkg):
    rng = np.random.default_rng(0)
    with _ctx(pkg, 100) as ctx:
        ctx.init_particles(100, 50)
        from sph_test_amd import _abi as A
        for parents in ([3, 3], [50], [-1]):
            with pytest.raises(A.SphError) as e:
                ctx.split_particles(_random_splits(pkg, rng, np.array(parents)))
            assert e.value.status == A.SPH_ERR_INVALID
        assert ctx.get_params().active_particle_count == 50


def test_get_set_range_round_trip(pkg, oracle):
    n = 3000
    with _ctx(pkg, n) as ctx:
        ctx.init_particles(n, n)
        ctx.step(0.01, 2)                                  # slots are cell-sorted now
        full = ctx.download_aos84()
        part = ctx.get_particles(1000, 500)
        assert part.tobytes() == full[1000:1500].tobytes()
        new = part.copy()
        new["velocity"] += 1.0
        new["modeIndex"] = 7
        ctx.set_particles(1000, new)
        after = ctx.download_aos84()
        assert after[1000:1500].tobytes() == new.tobytes()
        assert after[:1000].tobytes() == full[:1000].tobytes() and after[1500:].tobytes() == full[1500:].tobytes()
        from sph_test_amd import _abi as A
        with pytest.raises(A.SphError):
            ctx.get_particles(2900, 200)


def test_resize_on_device_keeps_state_and_time(pkg):
    n = 2000
    with _ctx(pkg, n) as ctx:
        ctx.init_particles(n, n)
        ctx.step(0.01, 3)
        before = ctx.download_aos84()
        steps = ctx.stats().steps
        ctx.resize(5000)
        assert ctx.download_aos84().tobytes() == before.tobytes()
        assert ctx.stats().capacity == 5000 and ctx.stats().steps == steps
        ctx.step(0.01, 1)


def test_shipped_scene_headless(pkg):
    """The reference's own scenario (Particle Simulation.unity + NewCellGenome.asset): one cell at the
    centre divides every splitInterval = 5 s of simulated time until the 4-particle buffer is full
    (UpdateCellDivisionTimers stops when particleCount − activeParticleCount = 0, controller:648-649)."""
    ctl = shipped_controller(pkg)
    ctl.Start()
    assert ctl.activeParticleCount == 1
    first = ctl.context.get_particles(0, 1)[0]
    assert first["modeIndex"] == 0 and first["radius"] == 2.0       # minRadius == maxRadius == 2
    dt = 1.0 / 60.0
    history = []
    for frame in range(60 * 16):
        ctl.Update(dt)
        history.append(ctl.activeParticleCount)
    # divisions at t ≈ 5, 10, 15 s (the split is applied at the start of the next frame)
    assert history[60 * 5 - 5] == 1 and history[60 * 5 + 5] == 2 and history[60 * 10 + 5] == 4
    assert history[-1] == 4 and ctl.particleCount == 4
    ids = [ctl.ParticleIDs[i].GetFormattedID() for i in range(4)]
    assert len(set(ids)) == 4 and all(s != "Unknown" for s in ids)
    assert ctl.nextUniqueIDCounter == 7                              # 3 splits, 2 ids each, from 1
    parts = ctl.GetParticles()[:4]
    assert np.isfinite(parts["position"]).all()
    assert (np.linalg.norm(parts["position"], axis=1) <= 15.0 * (1 + 1e-5)).all()
    assert (parts["modeIndex"] == 0).all()
    ctl.OnDestroy()
