"""The decomposed step inside the library (sph_config.ndev > 1 / sph_comm_init; abi_multi.cpp).

On the one-GPU test box every slab context of a local group sits on device 0 (the halo copies are
then plain device copies instead of xGMI peer copies; the step is otherwise the same code).

  * ndev = 2 / 3 / 4 against the single-context step, dam-break and sloshing (the decomposition changes
    only who computes what: positions within 2e-6, as tests/test_gpu_slab.py);
  * ndev = 3 with re-balancing against the per-phase slab ABI driven from Python over gloo
    (tests/test_gpu_slab.py's harness, sph_test_amd.slab.SlabRunner): the same kernels on the same data
    in the same order, so every rank's owned particles are BIT-identical, over 60 steps that take the
    exact-size steps (after each re-cut) and the lag-sized steps (device sizes, no host read);
  * an RCCL communicator of one rank (sph_comm_init): the in-library step equals the single context bit
    for bit (world 1 has no halo; RCCL between ranks needs two GPUs and runs in the driver's 8-GPU bench).
"""
import numpy as np
import pytest

from test_gpu_slab import _run_ranks, _scenario, _single

pytestmark = pytest.mark.gpu


def _check(x, v, xs, vs):
    np.testing.assert_allclose(x, xs, rtol=0, atol=2e-6)
    np.testing.assert_allclose(v, vs, rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("ndev,kind", [(2, 0), (3, 0), (4, 0), (3, 1)])
def test_group_matches_single(pkg, ndev, kind):
    """kind 0: dam-break; 1: sloshing (the lateral forcing follows every slab's simulated time)."""
    sc = _scenario(pkg, kind)
    xs, vs = _single(pkg, sc)
    sim = pkg.SPHSim(sc, ndev=ndev, rebalance_every=0)
    try:
        d = sim.ctx.decomposition()
        assert d.world == ndev and d.local_ranks == ndev and d.total == len(xs)
        sim.step(8)
        _check(sim.positions(), sim.velocities(), xs, vs)
        st = sim.ctx.stats()
        assert st.active == len(xs) and st.steps == 8
        assert sim.ctx.decomposition().owned == len(xs)   # every particle owned once
    finally:
        sim.close()


def test_group_bitwise_vs_python_slab_path(pkg, tmp_path):
    """The in-library step (device sizes, lagged message capacities, RCCL-free local copies) against
    SlabRunner's per-phase ABI over gloo: bit-identical owned particles after 60 steps with re-balancing
    every 20 steps (3 re-cuts, each followed by two exact-size steps)."""
    sc = _scenario(pkg)
    steps, every = 60, 20
    rec = _run_ranks(3, tmp_path, rebalance_every=every, steps=steps)
    ref = {int(i): r for i, r in zip(rec[:, 6].view(np.int32), rec)}
    sim = pkg.SPHSim(sc, ndev=3, rebalance_every=every, profile=True)
    try:
        sim.step(steps)
        x, v, rho = sim.positions(), sim.velocities(), sim.density()
        ids = np.arange(len(x))
        want = np.stack([ref[i] for i in ids])
        assert x.tobytes() == np.ascontiguousarray(want[:, 0:3]).tobytes()
        assert v.tobytes() == np.ascontiguousarray(want[:, 3:6]).tobytes()
        assert rho.tobytes() == np.ascontiguousarray(want[:, 7]).tobytes()
        cuts = [tuple(int(v) for v in c) for c in np.load(tmp_path / "cuts0.npy")]
        d = sim.ctx.decomposition()
        assert (d.cut.cx_lo, d.cut.cx_hi) == cuts[0]   # rank 0's slab after re-balancing, as the Python run's
        ks = sim.ctx.kernel_stats()
        assert ks["resort"]["launches"] > 0          # the device-sized incremental re-sort ran
    finally:
        sim.close()


@pytest.mark.parametrize("switch", ["SPH_NO_PRE_REC", "SPH_NO_EARLY_SENDS"])
def test_group_step_placement_is_bitwise_neutral(pkg, monkeypatch, switch):
    """Where the slab step runs its work never changes results: a 3-slab group with re-balancing every 40
    steps, 160 steps with the next step's record kernel on the comm stream and early sends (the default),
    against the same run with the record kernel at each step's start (SPH_NO_PRE_REC) or without early sends
    (SPH_NO_EARLY_SENDS): bit-identical positions, velocities and densities."""
    sc = _scenario(pkg)

    def run():
        sim = pkg.SPHSim(sc, ndev=3, rebalance_every=40)
        try:
            sim.step(160)
            return sim.positions(), sim.velocities(), sim.density()
        finally:
            sim.close()

    base = run()
    monkeypatch.setenv(switch, "1")
    alt = run()
    for a, b in zip(base, alt):
        assert a.tobytes() == b.tobytes()


def test_group_long_run_lag_sizes(pkg):
    """300 steps of a 2-slab group with re-balancing every 50: the lag-sized messages never overflow
    (a flagged overflow would fail sph_step with SPH_ERR_CAPACITY), no particle is lost, and the result
    stays within the decomposition tolerance of the single context after the first 8 steps."""
    sc = _scenario(pkg)
    sim = pkg.SPHSim(sc, ndev=2, rebalance_every=50, validate=True)
    try:
        sim.step(300)
        x = sim.positions()
        assert np.isfinite(x).all()
        assert (x >= 0).all() and (x <= np.array(sim.params.box, np.float32)).all()
        assert sim.ctx.decomposition().owned == len(x)
    finally:
        sim.close()


def test_rccl_world1_bitwise(pkg):
    """One RCCL rank: sph_comm_init + sph_init_scenario + sph_step give the single context's bits."""
    from sph_test_amd.context import comm_unique_id
    sc = _scenario(pkg)
    xs, vs = _single(pkg, sc, 50)
    p, dt = pkg.scenario_params(sc)
    ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 1000)
    try:
        ctx.comm_init(comm_unique_id(), 1, 0)
        ctx.set_params(p)
        ctx.init_scenario(sc)
        ctx.step(dt, 50)
        d = ctx.decomposition()
        assert d.world == 1 and d.owned == len(xs)
        rec = np.empty((ctx.stats().capacity, 8), np.float32)
        import ctypes as C
        from sph_test_amd import _abi as A
        n = C.c_int32()
        A.check("sph_slab_read_owned", ctx._L.sph_slab_read_owned(ctx.handle, A.ptr(rec), len(rec), C.byref(n)), ctx.handle)
        rec = rec[: n.value]
        order = np.argsort(rec[:, 6].view(np.int32))
        assert np.array_equal(rec[order, 0:3], xs)
        assert np.array_equal(rec[order, 3:6], vs)
    finally:
        ctx.close()


def test_group_overflow_stops_the_group(pkg, monkeypatch):
    """A forced tiny halo-message capacity (SPH_DEBUG_MSG_CAP: every lag-sized message holds 256
    records, far fewer than a ghost column) overflows on the receiving side. The overflow is flagged
    on the device, the step still completes on clamped sizes (no rank returns alone), and sph_step
    fails with SPH_ERR_CAPACITY for the whole group at the step the flag is read: the first lag-sized
    step is 3 (three exact-size steps after the initial cut), its flags are read two steps on."""
    sc = _scenario(pkg)
    # read once when the scenario is cut (abi_multi.cpp read_switches: over RCCL every rank must agree on it)
    monkeypatch.setenv("SPH_DEBUG_MSG_CAP", "256")
    sim = pkg.SPHSim(sc, ndev=3, rebalance_every=0)
    try:
        with pytest.raises(pkg.SphError) as ei:
            sim.step(20)
        msg = str(ei.value)
        assert ei.value.status == -3, msg
        assert "slab step 5:" in msg and "halo message overflow" in msg, msg
    finally:
        monkeypatch.delenv("SPH_DEBUG_MSG_CAP", raising=False)
        sim.close()


def test_force_without_density_scans_by_distance(pkg):
    """The per-phase ABI lets a caller run the force pass after a new assemble without a density pass
    in between: the hit mask then describes the previous slot order, so the force pass must not read
    it (every wave-plane scans by distance; sph_read_hit_mask_counts), while after a density pass it
    takes its hits from the mask."""
    import ctypes as C
    from sph_test_amd import _abi as A
    from sph_test_amd import slab
    sc = _scenario(pkg)
    p, dt = pkg.scenario_params(sc)
    n = sc.nx * sc.ny * sc.nz
    ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, 3, n + 4096)
    L, h = ctx._L, ctx.handle
    try:
        ctx.set_params(p)
        A.check("sph_slab_set", L.sph_slab_set(h, C.byref(A.SphSlab(0, slab.global_columns(p)))), h)
        A.check("sph_slab_init_scenario", L.sph_slab_init_scenario(h, C.byref(sc)), h)
        cnt = (C.c_int32 * 2)()
        rng = (C.c_int32 * 10)()

        def step(density: bool):
            A.check("sph_slab_count_sends", L.sph_slab_count_sends(h, cnt), h)
            A.check("sph_slab_assemble", L.sph_slab_assemble(h, None, 0, None, 0), h)
            if density:
                A.check("sph_slab_density", L.sph_slab_density(h), h)
            A.check("sph_slab_ranges", L.sph_slab_ranges(h, rng), h)
            A.check("sph_slab_force", L.sph_slab_force(h, dt, 0), h)
            A.check("sph_slab_finish_step", L.sph_slab_finish_step(h, dt), h)
            ctx.synchronize()

        xsub = ctx.stats().grid[0] // slab.global_columns(p)   # x sub-columns: 2 * xsub + 1 planes per wave
        npl = 2 * xsub + 1
        ctx.hit_mask_counts(reset=True)     # arm the counters
        for _ in range(3):
            step(True)
        dist_planes, waves = (int(c) for c in ctx.hit_mask_counts(reset=True))
        assert waves > 0 and dist_planes < npl * waves      # the mask was used
        step(False)
        dist_planes, waves = (int(c) for c in ctx.hit_mask_counts(reset=True))
        assert waves > 0 and dist_planes == npl * waves     # stale mask: never read
    finally:
        ctx.close()


@pytest.mark.parametrize("ndev", [2, 4, 8])
def test_bench_check_tolerance_on_groups(pkg, ndev):
    """bench.py's N > 1 correctness check (slab_check: CHECK_STEPS steps of check_scenario with
    re-balancing every CHECK_REBALANCE, owned positions against one context, |dx| <= CHECK_MAX_DX) run
    on local groups of the same slab counts: the driver's 2/4/8-GPU bench must not fail its own check
    on a correct decomposition. The measured difference is printed."""
    import bench
    sc = bench.check_scenario(pkg, ndev)
    xs, vs = _single(pkg, sc, bench.CHECK_STEPS)
    sim = pkg.SPHSim(sc, ndev=ndev, rebalance_every=bench.CHECK_REBALANCE)
    try:
        sim.step(bench.CHECK_STEPS)
        x, v = sim.positions(), sim.velocities()
        dx = float(np.abs(x - xs).max())
        print({"ndev": ndev, "max_dx": dx, "max_dv": float(np.abs(v - vs).max()),
               "rebalances": sim.ctx.decomposition().rebalances, "limit": bench.CHECK_MAX_DX})
        assert dx <= bench.CHECK_MAX_DX
        assert dx == 0.0 and np.array_equal(v, vs)     # the slabs keep the single domain's slot order
        assert sim.ctx.decomposition().rebalances > 0
    finally:
        sim.close()


def _top_of_column(x, colw, col, up):
    """The highest particle of global column `col` (a free-surface particle: few neighbours to brake it)."""
    sel = np.where(np.floor(x[:, 0] / colw).astype(np.int64) == col)[0]
    assert len(sel) > 0, col
    return int(sel[np.argmax(x[sel, up])])


@pytest.mark.parametrize("resort,early", [("1", True), ("1", False), ("0", True)])
def test_group_column_jump_falls_back_to_full_sends(pkg, monkeypatch, resort, early):
    """A particle of rank 0 kicked from column c1 − 3 across two columns in one step, into its last own
    column or the halo column c1 (rank 0 owns [0, c1)): it must be sent to rank 1, although the steady-
    state sends scan only the old columns c1 − 2 and c1 − 1. With the incremental re-sort (SPH_RESORT=1)
    the force pass's column-jump guard flags the move and the next sends scan every own slot; with the
    full sort (SPH_RESORT=0) the guard cannot run (it reads the previous order's keys) and the sends scan
    every own slot on every step (abi_multi.cpp steady_sends). Either way the group stays bit-identical
    to one context. The kick is taken back after the jump, so the run goes on in the steady state.
    A kick drops the messages sent early (during the step before it) and holds the early sends for one
    step, so the jump step keeps the graceful guard; early=False runs the whole test without early sends."""
    monkeypatch.setenv("SPH_RESORT", resort)
    if not early:
        monkeypatch.setenv("SPH_NO_EARLY_SENDS", "1")
    sc = _scenario(pkg)
    p, dt = pkg.scenario_params(sc)
    colw = float(np.float32(2.0) * np.float32(p.h))
    up = int(np.argmax(np.abs(np.array(p.gravity))))
    single = pkg.SPHSim(sc)
    group = pkg.SPHSim(sc, ndev=3, rebalance_every=0)
    try:
        for s in (single, group):
            s.step(10)
        c1 = int(group.ctx.decomposition().cut.cx_hi)
        x = single.positions()
        pid = _top_of_column(x, colw, c1 - 3, up)
        f = float(x[pid, 0]) / colw - (c1 - 3)
        kick = np.array([(3.0 - f) * colw / float(dt), 0.0, 0.0], np.float32)   # XSPH / viscosity take some back
        for s in (single, group):
            s.ctx.debug_kick(pid, kick)
            s.step(1)
        x1 = single.positions()
        col1 = int(np.floor(float(x1[pid, 0]) / colw))
        print({"resort": resort, "c1": c1, "pid": pid, "f": f, "landed_column": col1,
               "moved_columns": float(x1[pid, 0] - x[pid, 0]) / colw})
        assert col1 in (c1 - 1, c1), (col1, c1)             # moved two or three columns, still in the window
        assert np.array_equal(group.positions(), x1) and np.array_equal(group.velocities(), single.velocities())
        v1 = single.velocities()[pid]
        for s in (single, group):
            s.ctx.debug_kick(pid, -v1)                       # stop it: the run continues in the steady state
            s.step(6)
        assert np.array_equal(group.positions(), single.positions())
        assert np.array_equal(group.velocities(), single.velocities())
    finally:
        single.close()
        group.close()


def test_group_window_exit_stops_the_group(pkg, monkeypatch):
    """A particle of rank 0 kicked from its last own column c1 − 1 past the halo column c1 in one step has
    left the columns rank 0 holds: no neighbour receives it from the boundary columns, so the force pass
    raises SZ_JUMP and sph_step fails for the whole group (the flags are read two steps on), naming it."""
    monkeypatch.setenv("SPH_RESORT", "1")
    sc = _scenario(pkg)
    p, dt = pkg.scenario_params(sc)
    colw = float(np.float32(2.0) * np.float32(p.h))
    up = int(np.argmax(np.abs(np.array(p.gravity))))
    group = pkg.SPHSim(sc, ndev=3, rebalance_every=0)
    try:
        group.step(10)
        c1 = int(group.ctx.decomposition().cut.cx_hi)
        x = group.positions()
        pid = _top_of_column(x, colw, c1 - 1, up)
        f = float(x[pid, 0]) / colw - (c1 - 1)
        group.ctx.debug_kick(pid, np.array([(3.5 - f) * colw / float(dt), 0.0, 0.0], np.float32))
        with pytest.raises(pkg.SphError) as ei:
            group.step(4)
        assert ei.value.status == -3 and "left the held columns" in str(ei.value), str(ei.value)
    finally:
        group.close()


def test_group_early_sends_two_column_jump_stops_the_group(pkg, monkeypatch):
    """Early sends (the next step's halo messages packed during this step, abi_multi.cpp phase_boundary) scan
    only the two columns at each side; a particle that moves two or more columns while they are packed could be
    missed, so the force pass raises SZ_JUMP_EARLY and the group stops, naming it. A particle of rank 0 kicked
    to about 2.8 columns per step from column c1 − 7: the kick step runs without early sends (the graceful guard,
    test above), the step after it with them, and its second jump stops the group."""
    monkeypatch.setenv("SPH_RESORT", "1")
    sc = _scenario(pkg)
    p, dt = pkg.scenario_params(sc)
    colw = float(np.float32(2.0) * np.float32(p.h))
    up = int(np.argmax(np.abs(np.array(p.gravity))))
    group = pkg.SPHSim(sc, ndev=2, rebalance_every=0)   # two slabs: rank 0 holds about nine columns
    try:
        group.step(10)
        c1 = int(group.ctx.decomposition().cut.cx_hi)
        if c1 < 8:
            pytest.skip(f"rank 0 holds {c1} columns")
        x = group.positions()
        pid = _top_of_column(x, colw, c1 - 7, up)
        group.ctx.debug_kick(pid, np.array([2.8 * colw / float(dt), 0.0, 0.0], np.float32))
        group.step(1)   # the kick step: graceful
        x1 = group.positions()
        print({"c1": c1, "pid": pid, "col0": float(x[pid, 0]) / colw, "col1": float(x1[pid, 0]) / colw})
        with pytest.raises(pkg.SphError) as ei:
            group.step(4)
        assert ei.value.status == -3 and "two or more columns" in str(ei.value), str(ei.value)
    finally:
        group.close()


@pytest.mark.parametrize("cfg,ndev,steps", [("C4", 4, 120), ("C5", 8, 100)])
def test_baseline_config_decomposed_full_size(pkg, oracle, monkeypatch, cfg, ndev, steps):
    """BASELINE's own multi-GPU configurations decomposed as they run on 4 / 8 GPUs, at full size, as a local
    group on the test box's one device: C4 (4,194,304 particles, sloshing) in 4 slabs, C5 (16,777,216) in 8,
    re-balanced every 20 steps. The cuts start one column right of the equal-count position
    (SPH_DEBUG_CUT_SKEW=1), so the first re-balancing re-cuts every slab at full size (a full radix sort and three
    exact-size steps follow). Every step's halo must reproduce the 27-cell neighbourhood at every cut
    (SimulateParticles.compute:228-233), so the group is bit-identical to one context; then one step from the
    decomposed state meets the oracle tolerances of test_gpu_parity_headline.compare_one_step."""
    from test_gpu_parity_headline import compare_one_step
    sc = pkg.config_scenario(cfg)
    monkeypatch.setenv("SPH_DEBUG_CUT_SKEW", "1")
    group = pkg.SPHSim(sc, ndev=ndev, rebalance_every=20)
    monkeypatch.delenv("SPH_DEBUG_CUT_SKEW")
    try:
        group.step(steps)
        xg, vg = group.positions(), group.velocities()
        d = group.ctx.decomposition()
        assert d.world == ndev and d.owned == group.n == len(xg)
        rebalances = d.rebalances
        assert rebalances > 0
    finally:
        group.close()
    single = pkg.SPHSim(sc)
    try:
        single.step(steps)
        xs, vs = single.positions(), single.velocities()
        same = bool(np.array_equal(xg, xs) and np.array_equal(vg, vs))
        print({"cfg": cfg, "ndev": ndev, "steps": steps, "rebalances": rebalances, "bitwise": same,
               "max_dx": float(np.abs(xg - xs).max())})
        assert same
        t = float(np.float32(single.ctx.stats().sim_time))
        compare_one_step(pkg, oracle, single, xg, vg, f"{cfg} decomposed x{ndev}", t=t)
    finally:
        single.close()


def test_group_through_the_collapse_bitwise(pkg):
    """C3 x 4 (4,194,304 particles, dam-break) in 4 slabs for 5,000 steps, re-balanced every 50: from rest through
    the collapse to the surge front running along the floor (bench.py's mid-collapse state), so the steady-state
    steps with early sends meet the splash, thousands of movers per step (steps past the re-sort's
    mover limit take the full sort and send from every own slot) and the re-cuts that follow the moving fluid. The
    group stays bit-identical to one context."""
    from sph_test_amd import slab
    sc = slab.weak_scenario("C3", 4)
    steps = 5000
    group = pkg.SPHSim(sc, ndev=4, rebalance_every=50)
    try:
        group.step(steps)
        xg, vg = group.positions(), group.velocities()
        rebalances = group.ctx.decomposition().rebalances
    finally:
        group.close()
    single = pkg.SPHSim(sc)
    try:
        single.step(steps)
        xs, vs = single.positions(), single.velocities()
    finally:
        single.close()
    same = bool(np.array_equal(xg, xs) and np.array_equal(vg, vs))
    print({"steps": steps, "rebalances": rebalances, "bitwise": same, "max_dx": float(np.abs(xg - xs).max())})
    assert rebalances > 0 and same


def test_group_sloshing_long_run_bitwise(pkg):
    """BASELINE's C4 (4,194,304 particles, sloshing: lateral forcing, the fastest x motion of the configurations) in 4
    slabs for 2,000 steps, re-balanced every 50: the early sends' two-column scan never misses a particle (a miss would
    stop the group with SZ_JUMP_EARLY or break the identity), and the group stays bit-identical to one context."""
    sc = pkg.config_scenario("C4")
    steps = 2000
    group = pkg.SPHSim(sc, ndev=4, rebalance_every=50)
    try:
        group.step(steps)
        xg, vg = group.positions(), group.velocities()
        rebalances = group.ctx.decomposition().rebalances
    finally:
        group.close()
    single = pkg.SPHSim(sc)
    try:
        single.step(steps)
        xs, vs = single.positions(), single.velocities()
    finally:
        single.close()
    same = bool(np.array_equal(xg, xs) and np.array_equal(vg, vs))
    print({"steps": steps, "rebalances": rebalances, "bitwise": same, "max_dx": float(np.abs(xg - xs).max())})
    assert same
