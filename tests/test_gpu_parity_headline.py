"""Model S GPU-vs-oracle parity where the headline runs.

One step of the HIP path (through the C ABI) against oracle.sph_step_diag on the SAME input, for:
  * full C3 (1,048,576 particles) from the resting lattice;
  * C3 mid-collapse: 5,000 steps advanced on the GPU, then the state uploaded to both sides;
  * a wall-driven state (every wall clamps and reflects in the compared step);
  * a splash state whose sparse workgroups provably take the chunked and the global-gather
    paths of wcsph_tiled.hip (sph_read_path_counts > 0 on both passes).

Tolerances (SURVEY.md §8c Model S, SPEC_SPH.md §2), all per particle:
  * sorted ids and the cell-start table: bit-exact;
  * pass 1: |ρ_gpu − ρ_oracle| ≤ 1e-5·ρ_oracle;
  * pass 2 on the same inputs: the oracle's pass 2 runs on the GPU's own (ρ, P/ρ²), so only pass-2
    arithmetic differs. The kick is v1 = v0 + (a + g)·dt on both sides, so the acceleration error is
    |v1_gpu − v1_oracle|/dt, bounded by 1e-4·S with S = Σ_j m|F|r(|Pρ_i| + |Pρ_j| + |Π_ij|), the pair
    terms before they cancel (the net acceleration of a fluid particle is ~g while its ~50 pressure terms
    are orders larger, so a bound relative to the net value is meaningless), plus the support-edge
    conditioning Q = Σ_{q>=1} 2·T_ij·δq/(2 − q) with δq = 2^-21 (four ulp of q; oracle.h or_sph_step_diag):
    for q >= 1 a pair term T ∝ (2 − q)², so a q rounded differently by δq (the GPU's fma chain and rsq
    against the oracle's products and sqrt) moves T by 2δq/(2 − q) of itself. It matters only where a
    particle's S is held by pairs at the support edge: the splash state's largest err/S (7.8e-5 in r5 and
    r6) are particles with ONE neighbour at 2 − q = 0.002–0.009 (scripts/pass2_margin.py,
    profiles/r06_pass2_margin.log), whose error is 0.18–0.48 of Q; plus the fp32 rounding of
    v1 (2 ulp) and of (a + g)·dt (2 ulp);
  * the whole step against the oracle's whole step: the same bound plus the propagation of the pass-1
    difference through the stiff Tait EOS, E·max_i|δρ_i/ρ_i| with E = Σ_j m|F|r(E_i + E_j),
    E = (B/ρ²)(5(ρ/ρ0)^7 + 2) (oracle.h): a 1e-6 relative density difference moves P by ~7e-6·B;
  * position: x1 = x0 + (v1 + δv)·dt, so |Δx1| ≤ (|Δv1| + 1e-4·Σ_j|XSPH term_ij| + Q_x)·dt + 3 ulp(max(x0, x1)),
    Q_x = Σ_{q>=1} 3·|XSPH term_ij|·δq/(2 − q) (W ∝ (2 − q)³)
    (the GPU may fuse the drift into one rounding where the oracle rounds twice);
  * walls: where the reference's new position lies within the position tolerance of a wall, the two
    sides may fall on opposite sides of it, so the velocity may be the reflected one (−e·v) on one side
    only; such particles are counted and must stay below 1e-4 of N.
The acceleration error beyond the fp32 rounding of the kick, over S and over the whole bound (1e-4·S + Q + the
EOS term), and the other maxima are printed (pytest -s / the GPU log) so the margins are on record.
"""
import numpy as np
import pytest

from conftest import oracle_sph_params
from sph_states import block_paths, splash_state, wall_state

pytestmark = pytest.mark.gpu

RHO_RTOL = 1e-5
ACC_RTOL = 1e-4


def _ulp(a):
    a = np.abs(np.asarray(a, np.float32))
    return np.spacing(np.maximum(a, np.float32(1e-30))).astype(np.float64)


def _check(label, dt, e, L, x0, xg, vg, xr, vr, S, Q, extra, n):
    """x, v of the GPU against a reference step (xr, vr) from x0; returns (summary, failures). S: the
    acceleration and XSPH scales and |a + g|; Q: their support-edge conditioning terms (module docstring)."""
    dv = np.abs(vg.astype(np.float64) - vr.astype(np.float64))
    rnd = 2 * _ulp(np.maximum(np.abs(vr), np.abs(vg))) + 2 * _ulp(S[:, 2:5]) * dt   # fp32 rounding of the kick
    abound = ACC_RTOL * S[:, 0:1] + Q[:, 0:1] + extra
    vtol = abound * dt + rnd
    # x1 = x0 + (v1 + δv)·dt: the GPU may round the drift once (fused), the oracle twice
    xtol = ((dv + ACC_RTOL * S[:, 1:2] + Q[:, 1:2]) * dt
            + 3 * _ulp(np.maximum(np.maximum(np.abs(xr), np.abs(xg)), np.abs(x0))))
    xtol_w = np.maximum(xtol, 1e-6 * dt) + _ulp(L)[None, :]
    near = (np.abs(xr) <= xtol_w) | (np.abs(xr - L[None, :]) <= xtol_w)
    alt = np.minimum(np.abs(vg + e * vr), np.abs(vg + vr / e))
    vbad = dv > vtol
    amb = vbad & near & (alt <= vtol * (1 + 1 / e))
    vfail = vbad & ~amb
    xerr = np.abs(xg.astype(np.float64) - xr.astype(np.float64))
    xfail = (xerr > xtol) & ~near
    scale = np.maximum(S[:, 0:1], 1e-30)
    # margins over the particles the velocity check holds (a wall-ambiguous particle is checked against the
    # reflected velocity instead)
    aerr = np.where(amb, 0.0, np.maximum(dv - rnd, 0.0) / dt)
    summ = {f"{label}_acc_err_over_S_max": float((aerr / scale).max()),
            f"{label}_acc_err_over_bound_max": float((aerr / np.maximum(abound, 1e-30)).max()),
            f"{label}_acc_err_max": float((dv / dt).max()),
            f"{label}_v_fail": int(vfail.sum()), f"{label}_wall_ambiguous": int(amb.any(axis=1).sum()),
            f"{label}_x_err_max": float(xerr.max()), f"{label}_x_fail": int(xfail.sum())}
    bad = []
    if vfail.any():
        bad.append((label, "v", np.argwhere(vfail)[:5].tolist()))
    if amb.any(axis=1).sum() > max(1, n // 10000):
        bad.append((label, "wall-ambiguous count"))
    if xfail.any():
        bad.append((label, "x", np.argwhere(xfail)[:5].tolist()))
    return summ, bad


def compare_one_step(pkg, O, sim, x0, v0, label, t=0.0):
    """Upload (x0, v0) to the GPU context at simulated time t (the sloshing forcing reads it), step
    once; run the oracle on the same input at the same t; assert the tolerances above. Returns
    (summary, sparse-path counts of the GPU step)."""
    op = oracle_sph_params(O, sim.params, sim.scenario.dim)
    n = len(x0)
    sim.ctx.upload_state(x0, v0)
    t = float(np.float32(t))
    if t != 0.0:
        sim.ctx.set_sim_time(t)
    sim.ctx.path_counts(reset=True)
    sim.step(1)
    paths = sim.ctx.path_counts(reset=True)
    xg, vg, rg, pg = sim.positions(), sim.velocities(), sim.density(), sim.ctx.pressure_term()
    ids_g, cs_g = sim.ctx.sorted_ids(), sim.ctx.cell_start()
    xo, vo, io, ro, _, cso, acc, mag = O.sph_step_diag(op, x0, v0, np.arange(n, dtype=np.int32), sim.dt, t)
    assert np.array_equal(ids_g, io), f"{label}: sort permutation differs"
    assert np.array_equal(cs_g, cso), f"{label}: cell-start table differs"
    # pass 2 alone: the oracle's force pass on the GPU's pass-1 output (sorted order = io)
    sk = O.grid_keys(op, x0)[io]
    x2, v2, acc2, mag2 = O.force_range_diag(op, x0[io], v0[io], rg[io], pg[io], sk, cso, sim.dt, t)
    order = np.argsort(io)
    xo, vo, ro, acc, mag = xo[order], vo[order], ro[order], acc[order], mag[order]
    x2, v2, acc2, mag2 = x2[order], v2[order], acc2[order], mag2[order]
    dt = float(sim.dt)
    g = np.array(sim.params.gravity, np.float64)
    L = np.array(sim.params.box, np.float64)
    e = float(sim.params.wall_restitution)
    rerr = np.abs(rg.astype(np.float64) - ro) / ro
    S1 = np.concatenate([mag2[:, :2], np.abs(acc2 + g[None, :])], axis=1).astype(np.float64)
    S2 = np.concatenate([mag[:, :2], np.abs(acc + g[None, :])], axis=1).astype(np.float64)
    s1, bad1 = _check("pass2", dt, e, L, x0, xg, vg, x2, v2, S1, mag2[:, 3:5].astype(np.float64), 0.0, n)
    s2, bad2 = _check("step", dt, e, L, x0, xg, vg, xo, vo, S2, mag[:, 3:5].astype(np.float64),
                      mag[:, 2:3].astype(np.float64) * rerr.max(), n)
    summary = {"label": label, "n": n, "paths": paths.tolist(), "rho_rel_max": float(rerr.max()), **s1, **s2,
               "wall_clamped": int(((xo == 0) | (xo == L[None, :].astype(np.float32))).any(axis=1).sum())}
    print(summary)
    assert rerr.max() <= RHO_RTOL, summary
    assert not bad1 and not bad2, (summary, bad1, bad2)
    return summary, paths


def test_c3_one_step_from_rest(pkg, oracle):
    """Full C3 (1,048,576 particles), one step from the lattice: the headline configuration."""
    sim = pkg.SPHSim.from_config("C3")
    try:
        x0 = sim.positions()
        assert len(x0) == 1_048_576
        compare_one_step(pkg, oracle, sim, x0, np.zeros_like(x0), "C3 rest")
    finally:
        sim.close()


def test_c4_one_step_sloshing_forced(pkg, oracle):
    """Full C4 (4,194,304 particles, BASELINE configs[3], sloshing): 400 GPU steps so that the lateral
    forcing f_ext(t) = A·sin(2πf₁t) is well away from zero, then one step on both sides from the
    same uploaded state at the same t (sph_set_sim_time)."""
    sim = pkg.SPHSim.from_config("C4")
    try:
        assert sim.n == 4_194_304
        sim.step(400)
        t = float(np.float32(sim.ctx.stats().sim_time))
        p = sim.params
        fext = float(p.forcing_amp) * np.sin(2 * np.pi * float(p.forcing_freq) * t)
        assert abs(fext) > 0.05 * abs(float(p.forcing_amp)) > 0, (fext, p.forcing_amp, t)
        x0, v0 = sim.positions(), sim.velocities()
        assert np.isfinite(x0).all() and np.isfinite(v0).all()
        assert np.abs(v0[:, 0]).max() > 0           # the forcing has set the layer moving
        compare_one_step(pkg, oracle, sim, x0, v0, "C4 sloshing", t=t)
    finally:
        sim.close()


def test_c5_one_step_from_rest(pkg, oracle):
    """Full C5 (16,777,216 particles, BASELINE configs[4]) on ONE context, one step from the lattice:
    the 8-GPU configuration's whole domain against the oracle (the decomposed step is checked
    against the single context in test_gpu_multi.py)."""
    sim = pkg.SPHSim.from_config("C5")
    try:
        x0 = sim.positions()
        assert len(x0) == 16_777_216
        compare_one_step(pkg, oracle, sim, x0, np.zeros_like(x0), "C5 rest")
    finally:
        sim.close()


def test_c3_mid_collapse(pkg, oracle):
    """C3 after 5,000 GPU steps (0.30 s simulated, T = t·sqrt(2g/L) ≈ 1.7: the surge front runs
    along the floor), then one step on both sides from the same uploaded state."""
    sim = pkg.SPHSim.from_config("C3")
    try:
        sim.step(5000)
        x0, v0 = sim.positions(), sim.velocities()
        assert np.isfinite(x0).all() and np.isfinite(v0).all()
        front = np.percentile(x0[:, 0], 99.9) / (64 * 0.01)
        assert front > 1.5, f"the column has not collapsed yet (front {front:.2f} column widths)"
        s, _ = compare_one_step(pkg, oracle, sim, x0, v0, "C3 mid-collapse")
        assert s["wall_clamped"] > 0      # particles on the floor / walls in the compared step
    finally:
        sim.close()


def test_wall_driven_state(pkg, oracle):
    """Every wall clamps and reflects in the compared step (SPEC_SPH.md §2 walls)."""
    sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24, 20, 16, 40, 40, 40, dx=0.01, seed=5)
    sim = pkg.SPHSim(sc)
    try:
        op = oracle_sph_params(oracle, sim.params, 3)
        x0, v0 = wall_state(oracle, op, 24, 20, 16, 0.01, sim.dt)
        s, _ = compare_one_step(pkg, oracle, sim, x0, v0, "walls")
        assert s["wall_clamped"] >= len(x0) // 20
    finally:
        sim.close()


def test_splash_state_sparse_paths(pkg, oracle, monkeypatch):
    """Alternating dense / sparse x-columns: sparse workgroups see neighbour planes far beyond the
    LDS budget. The prediction (sph_states.block_paths) and the kernels' own counters agree, and
    all four sparse paths run in the compared step. The prediction assumes workgroups of 256 consecutive
    sorted targets, so the y-band schedule (schedule.hip), which cuts the targets along rows, is off here."""
    sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 32, 64, 128, 128, 128, 128, dx=0.01)
    p, dt = pkg.scenario_params(sc)
    monkeypatch.setenv("SPH_SCHED", "0")
    sim = pkg.SPHSim(sc, capacity=300_000)
    try:
        op = oracle_sph_params(oracle, sim.params, 3)
        cell = float(np.float32(2.0) * np.float32(p.h))
        x0, v0 = splash_state(int(op.grid.G[0]), 0, 0, cell, 8000, 60, tuple(p.box))
        x0 = np.minimum(x0, np.array(p.box, np.float32))
        pred = block_paths(oracle, op, x0)
        assert (pred > 0).all(), pred
        _, paths = compare_one_step(pkg, oracle, sim, x0, v0, "splash")
        assert np.array_equal(paths.astype(np.int64), pred), (paths, pred)
    finally:
        sim.close()


def test_c2_three_steps_mid_collapse(pkg, oracle):
    """C2 after 1,500 GPU steps, then 3 steps on both sides from the same state: the per-step
    differences compound through the EOS; positions agree to 1e-4·dx and densities to 1e-4."""
    sim = pkg.SPHSim.from_config("C2")
    try:
        sim.step(1500)
        x, v = sim.positions(), sim.velocities()
        sim.ctx.upload_state(x, v)
        op = oracle_sph_params(oracle, sim.params, 3)
        ids = np.arange(len(x), dtype=np.int32)
        for _ in range(3):
            x, v, ids, rho, _, _ = oracle.sph_step(op, x, v, ids, sim.dt, 0.0)
        sim.step(3)
        order = np.argsort(ids)
        np.testing.assert_allclose(sim.positions(), x[order], rtol=0, atol=1e-6)
        np.testing.assert_allclose(sim.density(), rho[order], rtol=1e-4)
    finally:
        sim.close()


def test_hit_mask_budget_fallback(pkg, oracle, monkeypatch):
    """A block of fluid compressed to 0.75 dx spacing (~2.4x the candidates per target, past the hit mask's
    256) beside fluid at rest spacing: pass 2 scans the compressed waves' planes by distance and takes the
    others from the mask (sph_read_hit_mask_counts: both kinds occur), and the step still meets the
    tolerances above."""
    sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24, 20, 16, 40, 40, 40, dx=0.01, seed=5)
    monkeypatch.setenv("SPH_SMALL", "0")           # the tiled passes (8,736 particles would take the small form)
    sim = pkg.SPHSim(sc, capacity=40_000)
    try:
        def block(x0, n, s, ny, nz):
            g = np.stack(np.meshgrid(np.arange(n), np.arange(ny), np.arange(nz), indexing="ij"), -1).reshape(-1, 3)
            return (g * s + s / 2 + np.array([x0, 0.0, 0.0])).astype(np.float32)
        a = block(0.0, 16, 0.0075, 24, 16)          # compressed: x < 0.12
        b = block(0.12, 12, 0.01, 18, 12)           # at rest spacing
        x0 = np.concatenate([a, b])
        v0 = np.zeros_like(x0)
        sim.ctx.hit_mask_counts(reset=True)        # arm the counters
        s, _ = compare_one_step(pkg, oracle, sim, x0, v0, "mask budget")
        dist_planes, waves = (int(c) for c in sim.ctx.hit_mask_counts(reset=True))
        print({"distance_wave_planes": dist_planes, "wave_planes": 3 * waves})
        assert 0 < dist_planes < 3 * waves
    finally:
        sim.close()
