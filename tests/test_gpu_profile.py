"""Per-kernel timing through the C ABI (SPH_FLAG_PROFILE, sph_get_kernel_stat, sph_set_profile_every):
the scopes of the Model S step carry their events in the kernels' dispatch packets, and a sampling stride
times one step in `every` while every launch is still counted."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(pkg, every, steps):
    sim = pkg.SPHSim.from_config("C2", profile=True)
    try:
        sim.step(3)                      # past the first step's full sort: steady-state scopes only
        sim.ctx.set_profile_every(every)
        sim.ctx.reset_kernel_stats()
        sim.step(steps)
        return sim.ctx.kernel_stats(), sim.positions()
    finally:
        sim.close()


def test_profile_every_step_times_every_launch(pkg):
    ks, _ = _run(pkg, 1, 8)
    for name in ("density", "force_integrate", "resort"):
        assert ks[name]["launches"] == 8, (name, ks[name])
        assert ks[name]["timed"] == 8, (name, ks[name])
        assert ks[name]["total_ms"] > 0.0
    # the C2 force pass takes tens of microseconds: the packet events bracket the kernel, not the host
    mean_us = ks["force_integrate"]["total_ms"] / ks["force_integrate"]["timed"] * 1e3
    assert 5.0 < mean_us < 5000.0, mean_us


def test_profile_sampling_counts_all_times_some(pkg):
    ks, _ = _run(pkg, 4, 12)
    for name in ("density", "force_integrate", "resort"):
        assert ks[name]["launches"] == 12, (name, ks[name])
        assert ks[name]["timed"] == 3, (name, ks[name])
        assert ks[name]["total_ms"] > 0.0


def test_profile_sampling_does_not_change_results(pkg):
    """Timing is observation only: the same steps with and without events give the same bits."""
    out = []
    for prof in (False, True):
        sim = pkg.SPHSim.from_config("C2", profile=prof)
        try:
            if prof:
                sim.ctx.set_profile_every(3)
            sim.step(10)
            out.append((sim.positions(), sim.velocities(), sim.density()))
        finally:
            sim.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)


def test_profile_every_rejects_zero(pkg):
    sim = pkg.SPHSim.from_config("C1", profile=True)
    try:
        with pytest.raises(Exception):
            sim.ctx.set_profile_every(0)
    finally:
        sim.close()
