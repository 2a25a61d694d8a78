"""Incremental re-sort (sph-test_amd/csrc/resort.hip) against the full radix sort.

Both realise the stable (cell key, slot index) order of SPEC_SPH.md §0, so the slot
permutation is identical. Every later float operation then runs on the same data in the same
order, and whole runs must agree BIT FOR BIT: positions, velocities, density, sorted ids, cell
starts. SPH_RESORT (read at context creation): 0 forces the full sort every step, 2 the
incremental re-sort whenever possible, 1 (default) switches to the full sort while the last
mover count the host has seen exceeds the crossover (sph_abi.cpp resort_limit).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(monkeypatch, make, flags=("0", "2")):
    out = []
    for flag in flags:
        monkeypatch.setenv("SPH_RESORT", flag)
        out.append(make())
    monkeypatch.delenv("SPH_RESORT")
    return out


def _assert_same(a, b, what):
    for f in ("positions", "velocities", "density", "sorted_ids", "cell_start"):
        x, y = getattr(a, f)(), getattr(b, f)()
        assert np.array_equal(x, y, equal_nan=True), f"{what}: {f} differs"


def test_resort_bitwise_dambreak(pkg, monkeypatch):
    full, inc = _pair(monkeypatch, lambda: pkg.SPHSim.from_config("C2", profile=True))
    try:
        for k in (1, 9, 40):
            full.step(k)
            inc.step(k)
            _assert_same(full.ctx, inc.ctx, f"after {k} more steps")
        ks_inc, ks_full = inc.ctx.kernel_stats(), full.ctx.kernel_stats()
        # the incremental path ran on every step after the first; the full path never did
        assert ks_inc["resort"]["launches"] == 49 and ks_inc["radix_sort"]["launches"] == 1
        assert "resort" not in ks_full and ks_full["radix_sort"]["launches"] == 50
    finally:
        full.close()
        inc.close()


def test_resort_bitwise_many_movers(pkg, monkeypatch):
    """A violent state: random velocities that move ~half the particles across a sub-cell per
    step, in every direction, including wall clamps (keys far from their old ones)."""
    sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24, 20, 16, 40, 40, 40, dx=0.01, seed=5)

    def make():
        s = pkg.SPHSim(sc, profile=True)
        rng = np.random.default_rng(11)
        x = s.positions()
        sub = 2 * s.params.h / 6                  # z sub-cell (SPEC_SPH.md §0)
        v = rng.uniform(-1.0, 1.0, x.shape).astype(np.float32) * (sub / s.dt)
        s.ctx.upload_state(x, v)
        return s

    full, inc = _pair(monkeypatch, make)
    try:
        for k in (1, 1, 3, 5):
            full.step(k)
            inc.step(k)
            _assert_same(full.ctx, inc.ctx, "violent state")
        assert inc.ctx.kernel_stats()["resort"]["launches"] == 9
    finally:
        full.close()
        inc.close()


def test_resort_after_state_changes(pkg, monkeypatch):
    """Uploads, parameter changes and resizes invalidate the sorted keys: the next step falls
    back to the full sort, and both paths still agree."""
    full, inc = _pair(monkeypatch, lambda: pkg.SPHSim.from_config("C1", profile=True))
    try:
        for s in (full, inc):
            s.step(5)
            x, v = s.positions(), s.velocities()
            s.ctx.upload_state(x[::-1].copy(), v[::-1].copy())   # new slot order
            s.step(3)
            s.ctx.resize(s.n + 100)
            s.step(3)
            s.ctx.set_params(s.params)
            s.step(3)
        _assert_same(full.ctx, inc.ctx, "after state changes")
        ks = inc.ctx.kernel_stats()
        # C1 is within the two-launch step's size: there the re-sort runs inside k_density_fused
        incremental = sum(ks.get(k, {}).get("launches", 0) for k in ("resort", "density_fused"))
        assert ks["radix_sort"]["launches"] == 4 and incremental == 10, ks
    finally:
        full.close()
        inc.close()


def test_resort_adaptive_falls_back_when_many_move(pkg, monkeypatch):
    """Default mode: a violent state (about half the particles change sub-cell per step, far above
    the crossover) goes back to the full sort once the host has seen the mover count; the quiet
    dam-break keeps the incremental path. Results stay bit-identical to the full sort."""
    sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 32, 32, 32, 48, 48, 48, dx=0.01, seed=5)

    def make():
        s = pkg.SPHSim(sc, profile=True)
        rng = np.random.default_rng(12)
        x = s.positions()
        sub = 2 * s.params.h / 6
        v = rng.uniform(-1.0, 1.0, x.shape).astype(np.float32) * (sub / s.dt)
        s.ctx.upload_state(x, v)
        return s

    full, ada = _pair(monkeypatch, make, flags=("0", "1"))
    try:
        for k in (1, 1, 1, 3):
            full.step(k)
            ada.step(k)
            _assert_same(full.ctx, ada.ctx, "adaptive, violent state")   # also syncs: the count is seen
        ks = ada.ctx.kernel_stats()
        assert ks["radix_sort"]["launches"] >= 4, ks      # fell back after the first incremental step
    finally:
        full.close()
        ada.close()
    quiet = pkg.SPHSim.from_config("C2", profile=True)
    try:
        quiet.step(1)
        quiet.ctx.synchronize()
        quiet.step(20)
        ks = quiet.ctx.kernel_stats()
        assert ks["resort"]["launches"] == 20 and ks["radix_sort"]["launches"] == 1
    finally:
        quiet.close()


@pytest.mark.parametrize("shape", ["C5", "C5_rank8"])
def test_resort_ranges_never_count_against_the_whole_list(pkg, shape):
    """C5 (16.8M particles) and the per-rank shape of C5 on 8 GPUs (its 256 x 512 cross-section, 16 lattice
    layers in x, as profiles/pmc_slab8.json), 300 steps each through the start of the collapse. From step ~60
    the front carries more particles per step into empty columns than one range stages in LDS (the last range's
    key interval holds every empty column); r5 counted such a range against the whole mover list, O(slots x
    movers), 7.75 against 4.19 ms per C5 step. The multi-pass path (resort.hip) must take every such range:
    the whole-list counters stay 0 (sph_read_resort_counts)."""
    if shape == "C5":
        sim = pkg.SPHSim.from_config("C5", profile=True)
    else:
        sim = pkg.SPHSim(pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 16, 256, 512, 64, 512, 512, dx=0.01,
                                           seed=1234), profile=True)
    try:
        sim.ctx.resort_counts(reset=True)
        tot = np.zeros(6, np.int64)
        for _ in range(6):
            sim.step(50)
            c = sim.ctx.resort_counts(reset=True).astype(np.int64)
            tot[:4] += c[:4]
            tot[4] = max(tot[4], c[4])
            tot[5] += c[5]
        ks = sim.ctx.kernel_stats()
        print({"shape": shape, "whole": int(tot[0]), "whole_lanes": int(tot[1]), "multi_pass_ranges": int(tot[2]),
               "passes": int(tot[3]), "max_range_entries": int(tot[4]), "share_restreams": int(tot[5]),
               "resort_launches": ks.get("resort", {}).get("launches", 0),
               "radix_sort_launches": ks.get("radix_sort", {}).get("launches", 0)})
        assert tot[0] == 0 and tot[1] == 0, tot
        assert ks["resort"]["launches"] >= 250, ks   # the incremental path ran (the adaptive mode's default)
    finally:
        sim.close()


# ------------------------------------------------------------------ Model R
def _contact_run(pkg, monkeypatch, flag, parts, steps, conns=None, change_active=None):
    from test_gpu_contact_team import _Manager
    monkeypatch.setenv("SPH_RESORT", flag)
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    if conns is not None:
        ctl.adhesionManager = _Manager(conns)
    ctl.Start(parts.copy())
    ctl.drag.selectedID = 3
    ctl.drag.targetPosition = (2.0, 1.0, -1.0)
    ctl.drag.strength = 50.0
    for s in range(steps):
        if change_active is not None and s == steps // 2:
            ctl.activeParticleCount = change_active
        ctl.Update(0.01)
    out = (ctl.GetParticles().tobytes(), ctl.context.torque_int().tobytes(), ctl.context.sorted_ids().tobytes(),
           ctl.context.cell_start().tobytes(), ctl.context.kernel_stats() if hasattr(ctl.context, "kernel_stats") else {})
    ctl.OnDestroy()
    monkeypatch.delenv("SPH_RESORT")
    return out


@pytest.mark.parametrize("case", ["plain", "bonds", "active_change"])
def test_resort_bitwise_contact(pkg, monkeypatch, case):
    """Model R: the incremental re-sort (movers appended by the contact pass; all seven slot arrays
    moved) against the full sort, bit for bit over 20 steps, with drag, adhesion bonds, and a change
    of activeParticleCount mid-run (which forces one full sort)."""
    from adhesion_cases import bonded_sphere
    from test_gpu_parity import random_sphere
    conns = None
    if case == "bonds":
        parts, conns = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 2048, seed=21)
    else:
        parts = random_sphere(pkg.PARTICLE84, 4096, seed=21)
    act = 3000 if case == "active_change" else None
    full = _contact_run(pkg, monkeypatch, "0", parts, 20, conns, act)
    inc = _contact_run(pkg, monkeypatch, "2", parts, 20, conns, act)
    for a, b, what in zip(full[:4], inc[:4], ("particles", "torque", "sorted ids", "cell starts")):
        assert a == b, what
