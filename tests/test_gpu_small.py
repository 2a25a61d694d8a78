"""Model S's small-N form (wcsph_tiled.hip k_density_small / k_force_small: one wave per target, the candidates of
the nine trimmed row windows spread over the lanes, the sums taken in visit order) against the LDS-tiled passes:
every float operation and its order are the tiled passes', so whole runs must agree BIT FOR BIT. SPH_SMALL (read at
context creation): 0 the tiled passes, 2 the small form at any size, 1 (default) the small form up to SMALL_N.
The states cover 2D (C1) and 3D, a dam-break from rest and a violent state (random velocities, wall clamps), and a
compressed block whose targets have more candidates than the tiled pass 2's hit mask covers (its distance scans)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(pkg, monkeypatch, make):
    out = []
    for flag in ("0", "2"):
        monkeypatch.setenv("SPH_SMALL", flag)
        out.append(make())
    monkeypatch.delenv("SPH_SMALL")
    return out


def _same(a, b, what):
    for f in ("positions", "velocities", "density", "sorted_ids"):
        x, y = getattr(a, f)(), getattr(b, f)()
        assert np.array_equal(x, y, equal_nan=True), f"{what}: {f} differs"


@pytest.mark.parametrize("case", ["C1", "3d", "violent", "compressed"])
def test_small_form_bit_identical_to_tiled(pkg, monkeypatch, case):
    def make():
        if case == "C1":
            return pkg.SPHSim.from_config("C1")
        sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24, 20, 16, 40, 40, 40, dx=0.01, seed=5)
        s = pkg.SPHSim(sc, capacity=40_000)
        if case == "violent":
            rng = np.random.default_rng(11)
            x = s.positions()
            v = rng.uniform(-1.0, 1.0, x.shape).astype(np.float32) * (2 * s.params.h / 6 / s.dt)
            s.ctx.upload_state(x, v)
        elif case == "compressed":   # test_hit_mask_budget_fallback's state: ~2.4x the candidates per target
            def block(x0, n, sp, ny, nz):
                g = np.stack(np.meshgrid(np.arange(n), np.arange(ny), np.arange(nz), indexing="ij"), -1).reshape(-1, 3)
                return (g * sp + sp / 2 + np.array([x0, 0.0, 0.0])).astype(np.float32)
            x = np.concatenate([block(0.0, 16, 0.0075, 24, 16), block(0.12, 12, 0.01, 18, 12)])
            s.ctx.upload_state(x, np.zeros_like(x))
        return s

    tiled, small = _pair(pkg, monkeypatch, make)
    try:
        for k in (1, 2, 7, 20):
            tiled.step(k)
            small.step(k)
            _same(tiled.ctx, small.ctx, f"{case}, after {k} more steps")
    finally:
        tiled.close()
        small.close()


@pytest.mark.parametrize("case", ["C1", "3d", "violent"])
def test_two_launch_step_bit_identical(pkg, monkeypatch, case):
    """Model S at n <= 4,096: the re-sort fused into pass 1 (wcsph_tiled.hip k_density_fused, then k_force_small on
    the sorted arrays it wrote; two launches per step) against the re-sort kernel + the small form (SPH_FUSED=0)."""
    def make(flag):
        monkeypatch.setenv("SPH_FUSED", flag)
        if case == "C1":
            s = pkg.SPHSim.from_config("C1")
        else:
            sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 16, 16, 16, 32, 32, 32, dx=0.01, seed=9)
            s = pkg.SPHSim(sc, capacity=4096)
            if case == "violent":
                rng = np.random.default_rng(13)
                x = s.positions()
                v = rng.uniform(-1.0, 1.0, x.shape).astype(np.float32) * (2 * s.params.h / 6 / s.dt)
                s.ctx.upload_state(x, v)
        monkeypatch.delenv("SPH_FUSED")
        return s

    three, two = make("0"), make("1")
    try:
        for k in (1, 2, 7, 40):
            three.step(k)
            two.step(k)
            _same(three.ctx, two.ctx, f"{case}, after {k} more steps")
    finally:
        three.close()
        two.close()
