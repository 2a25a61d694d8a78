"""Where pass 2's parity margin goes on the splash state (tests/test_gpu_parity_headline.py::test_splash_state_sparse_paths):
the GPU step saved by scripts/splash_dump.py against the oracle's pass 2 on the GPU's own (ρ, P/ρ²), as the test
compares them. For the particles of largest acceleration error over S (S = Σ_j m|F|r(|Pρ_i| + |Pρ_j| + |Π_ij|), the
test's scale) it lists the pairs: q, t = 2 − q, and each pair's share of S. A pair term T ∝ t² for q ≥ 1 (F·r ∝ t²), so
a q that two correct evaluations round differently by δq moves T by 2|T|δq/t: near the support edge (t → 0) the
relative error grows as 1/t. S_q = Σ_j 2|T_j|·δq/t_j (q ≥ 1; δq = 2^-21, four ulp of q in [1, 2): r² by an fma chain
against plain products, rsq against sqrt) bounds that conditioning term; the script prints err/S and err/(1e-4·S + S_q)
from its own float64 pair terms, then replays the test's own checks (test_gpu_parity_headline._check, with the
oracle's conditioning columns) on the dumped step.
    python scripts/pass2_margin.py gpurun_out/r06h/splash_gpu.npz"""
import sys
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as GE  # noqa: E402
from test_gpu_parity_headline import _check  # noqa: E402

d = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06h/splash_gpu.npz")
x0, v0, xg, vg, rg, pg, dt = d["x0"], d["v0"], d["x"], d["v"], d["rho"], d["prho"], float(d["dt"])
O = GE.load_oracle()
O.lib()
pkg = GE.load_package()
sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 32, 64, 128, 128, 128, 128, dx=0.01)
p, _ = pkg.scenario_params(sc)
op = O.sph_params(3, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box), p.wall_restitution,
                  p.forcing_amp, p.forcing_freq)
n = len(x0)
xo, vo, io, ro, _, cso, acc, mag = O.sph_step_diag(op, x0, v0, np.arange(n, dtype=np.int32), np.float32(dt), 0.0)
sk = O.grid_keys(op, x0)[io]
x2, v2, acc2, mag2 = O.force_range_diag(op, x0[io], v0[io], rg[io], pg[io], sk, cso, np.float32(dt), 0.0)
order = np.argsort(io)
x2, v2, acc2, mag2 = x2[order], v2[order], acc2[order], mag2[order]
xo, vo, ro, acc, mag = xo[order], vo[order], ro[order], acc[order], mag[order]


def ulp(a):
    a = np.abs(np.asarray(a, np.float32))
    return np.spacing(np.maximum(a, np.float32(1e-30))).astype(np.float64)


g = np.array(tuple(p.gravity), np.float64)
S = mag2[:, 0].astype(np.float64)
dv = np.abs(vg.astype(np.float64) - v2.astype(np.float64))
rnd = 2 * ulp(np.maximum(np.abs(v2), np.abs(vg))) + 2 * ulp(np.abs(acc2 + g[None, :])) * dt
err = (np.maximum(dv - rnd, 0.0) / dt).max(1)          # the test's acceleration error beyond the kick's rounding

# pair terms in float64 from the same inputs (particle order)
h, m, sig, B = float(op.h), float(op.mass), float(op.sigma), float(op.B)
eta2 = 0.01 * h * h
ac0 = float(op.alpha) * float(op.c0)
tree = cKDTree(x0.astype(np.float64))
pairs = tree.query_pairs(2 * h, output_type="ndarray")
i, j = np.concatenate([pairs[:, 0], pairs[:, 1]]), np.concatenate([pairs[:, 1], pairs[:, 0]])
dx = x0[i].astype(np.float64) - x0[j]
r = np.sqrt((dx * dx).sum(1))
q = r / h
t = 2.0 - q
F = np.where(q < 1.0, sig / h / h * (-3.0 + 2.25 * q), -sig / h * 0.75 * t * t / np.maximum(r, 1e-30))
vr = ((v0[i].astype(np.float64) - v0[j]) * dx).sum(1)
rbar = 0.5 * (rg[i].astype(np.float64) + rg[j])
pi_ij = np.where(vr < 0.0, -ac0 * (h * vr / (r * r + eta2)) / rbar, 0.0)
T = m * np.abs(F) * r * (np.abs(pg[i].astype(np.float64)) + np.abs(pg[j]) + np.abs(pi_ij))
DQ = 2.0 ** -21
Sq = np.bincount(i, weights=np.where(q >= 1.0, 2.0 * T * DQ / np.maximum(t, 1e-30), 0.0), minlength=n)
Sp = np.bincount(i, weights=T, minlength=n)
print({"n": n, "pairs": len(i), "S_pairs_over_S_oracle_median": float(np.median(Sp[S > 0] / S[S > 0]))})
ratio = err / np.maximum(S, 1e-30)
bound = 1e-4 * S + Sq
print({"err_over_S_max": float(ratio.max()), "err_over_bound_max": float((err / np.maximum(bound, 1e-30)).max()),
       "err_over_Sq_max": float((err / np.maximum(Sq, 1e-30)).max()),
       "particles_err_over_S_above_1e-5": int((ratio > 1e-5).sum())})
top = np.argsort(-ratio)[:6]
for k in top:
    sel = i == k
    tt, qq, TT = t[sel], q[sel], T[sel]
    o = np.argsort(-TT)
    print({"particle": int(k), "err_over_S": float(ratio[k]), "err_over_Sq": float(err[k] / max(Sq[k], 1e-30)),
           "neighbours": int(sel.sum()), "S": float(S[k]), "Sq": float(Sq[k]),
           "pairs (q, t, share of S)": [(round(float(qq[a]), 6), float(f"{tt[a]:.3g}"), round(float(TT[a] / Sp[k]), 3))
                                        for a in o[:6]]})
print({"Sq_python_over_oracle_max_rel_diff": float((np.abs(Sq - mag2[:, 3]) / np.maximum(Sq, 1e-30))[Sq > 1e-20].max())})
# the test's checks (tests/test_gpu_parity_headline.py compare_one_step) on the dumped step
L = np.array(tuple(p.box), np.float64)
e = float(p.wall_restitution)
rerr = np.abs(rg.astype(np.float64) - ro) / ro
S1 = np.concatenate([mag2[:, :2], np.abs(acc2 + g[None, :])], axis=1).astype(np.float64)
S2 = np.concatenate([mag[:, :2], np.abs(acc + g[None, :])], axis=1).astype(np.float64)
s1, bad1 = _check("pass2", dt, e, L, x0, xg, vg, x2, v2, S1, mag2[:, 3:5].astype(np.float64), 0.0, n)
s2, bad2 = _check("step", dt, e, L, x0, xg, vg, xo, vo, S2, mag[:, 3:5].astype(np.float64),
                  mag[:, 2:3].astype(np.float64) * rerr.max(), n)
print({"rho_rel_max": float(rerr.max()), **s1, **s2, "failures": bad1 + bad2})
# the particles that now hold the tightest margin
rb = err / np.maximum(1e-4 * S + mag2[:, 3].astype(np.float64), 1e-30)
for k in np.argsort(-rb)[:4]:
    sel = i == k
    print({"particle": int(k), "err_over_bound": float(rb[k]), "err_over_S": float(ratio[k]), "neighbours": int(sel.sum()),
           "min_t": float(t[sel].min()) if sel.any() else None, "Q_over_1e-4S": float(mag2[k, 3] / max(1e-4 * S[k], 1e-30))})
