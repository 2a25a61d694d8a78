"""Model of a pass-1 candidate cut that keeps the oracle's visit order (verdict r5 item 4): reuse a skin-widened hit
mask across steps. A target may reuse the candidate list of an earlier full evaluation only while its windows hold the
same particles in the same order: its own cell and row windows (zlo, zhi per row) unchanged and no mover's old or new
key in any cell of its windows. This counts, on the oracle's states (CPU, test infrastructure), the fraction of such
clean targets per step and prices the pass: a dirty target evaluates every candidate (17.75 VALU per candidate in the
4-candidate loop), a clean one walks its skin list by mask bits as pass 2 walks hits (~20 VALU per entry
at the walk's measured ~69% lane use). Skin s: candidates within 2h + s.
    python scripts/pass1_reuse_model.py [--config C2] [--steps 0,20,1500] [--skin 0.05]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402

VALU_CAND, VALU_WALK, WALK_USE = 17.75, 20.0, 0.69


def windows(g, pos):
    """Per target and row k (9 rows): the key range [lo, hi] of its trimmed window (SPEC_SPH.md §0, common.h
    row_window), or -1 for a row outside the grid / beyond 2h."""
    cell = np.float32(2.0) * np.float32(g["h"])
    inv_cell, inv_cz = np.float32(1.0) / cell, np.float32(g["zsub"]) / cell
    G = g["G"]
    gx = (pos[:, 0] * inv_cell)
    gy = (pos[:, 1] * inv_cell)
    cx = np.clip(np.floor(gx), 0, G[0] - 1).astype(np.int64)
    cy = np.clip(np.floor(gy), 0, G[1] - 1).astype(np.int64)
    fx = np.clip(gx - cx, 0, 1).astype(np.float32)
    fy = np.clip(gy - cy, 0, 1).astype(np.float32)
    gzf = (pos[:, 2] * inv_cz).astype(np.float32)
    lo = np.full((len(pos), 9), -1, np.int64)
    hi = np.full((len(pos), 9), -1, np.int64)
    for k in range(9):
        dx, dy = k // 3 - 1, k % 3 - 1
        gxg = fx if dx < 0 else (1 - fx if dx > 0 else np.zeros_like(fx))
        gyg = fy if dy < 0 else (1 - fy if dy > 0 else np.zeros_like(fy))
        d2 = gyg * gyg + gxg * gxg
        xx, yy = cx + dx, cy + dy
        ok = (d2 < 1) & (xx >= 0) & (xx < G[0]) & (yy >= 0) & (yy < G[1])
        hz = np.sqrt(np.maximum(1 - d2, 0)) * np.float32(g["zsub"]) + np.float32(1e-3)
        zlo = np.maximum((gzf - hz).astype(np.float32), 0).astype(np.int64)
        zhi = np.minimum(np.floor(gzf + hz), G[2] - 1).astype(np.int64)
        row = (xx * G[1] + yy) * G[2]
        lo[:, k] = np.where(ok, row + zlo, -1)
        hi[:, k] = np.where(ok, row + zhi, -1)
    return lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", default="0,20,1500")
    ap.add_argument("--skin", type=float, default=0.05, help="skin in units of h")
    args = ap.parse_args()
    pkg = GE.load_package()
    O = GE.load_oracle()
    sim = pkg.SPHSim.from_config(args.config, device=None) if False else None
    sc = pkg.config_scenario(args.config)
    prm, dt = pkg.scenario_params(sc)
    op = O.sph_params(3, prm.dx, prm.h, prm.rho0, prm.c0, prm.alpha, prm.xsph_eps, tuple(prm.gravity), tuple(prm.box),
                      prm.wall_restitution)
    g = {"h": prm.h, "zsub": 6, "G": (int(op.grid.G[0]), int(op.grid.G[1]), int(op.grid.G[2]))}
    nc = g["G"][0] * g["G"][1] * g["G"][2]
    x = O.lattice(3, sc.nx, sc.ny, sc.nz, prm.dx)
    v = np.zeros_like(x)
    ids = np.arange(len(x), dtype=np.int32)
    done = 0
    for k in [int(s) for s in args.steps.split(",")]:
        while done < k:
            x, v, ids, *_ = O.sph_step(op, x, v, ids, dt, 0.0, nthreads=8)
            done += 1
        # transition k -> k + 1
        o = np.argsort(ids)
        x0 = x[o]
        x1, v1, ids1, *_ = O.sph_step(op, x, v, ids, dt, 0.0, nthreads=8)
        x1 = x1[np.argsort(ids1)]
        k0, k1 = O.grid_keys(op, x0).astype(np.int64), O.grid_keys(op, x1).astype(np.int64)
        mv = k0 != k1
        dirty = np.zeros(nc + 1, np.int64)
        dirty[k0[mv]] = 1
        dirty[k1[mv]] = 1
        D = np.concatenate([[0], np.cumsum(dirty)])
        lo0, hi0 = windows(g, x0)
        lo1, hi1 = windows(g, x1)
        same_w = np.all((lo0 == lo1) & (hi0 == hi1), axis=1) & ~mv
        clean = same_w.copy()
        for r in range(9):
            ok = lo1[:, r] >= 0
            hit = np.where(ok, D[np.maximum(hi1[:, r], 0) + 1] - D[np.maximum(lo1[:, r], 0)], 0) > 0
            clean &= ~hit
        # candidates and skin candidates per target (a sample)
        srt = np.argsort(k1, kind="stable")
        cs = np.searchsorted(k1[srt], np.arange(nc + 1))
        samp = np.random.default_rng(0).choice(len(x1), 2000, replace=False)
        cand = skin = hits = 0
        R, Rs = 2 * prm.h, (2 + args.skin) * prm.h
        for i in samp:
            js = np.concatenate([srt[cs[lo1[i, r]]:cs[hi1[i, r] + 1]] for r in range(9) if lo1[i, r] >= 0])
            d = np.linalg.norm(x1[js] - x1[i], axis=1)
            cand += len(js)
            skin += int(np.sum(d <= Rs))
            hits += int(np.sum(d <= R))
        n = len(samp)
        disp = np.linalg.norm(x1 - x0, axis=1) / prm.h
        dmax, d999 = float(disp.max()), float(np.quantile(disp, 0.999))
        fc = float(clean.mean())
        c_full = cand / n * VALU_CAND
        c_clean = skin / n * VALU_WALK / WALK_USE
        model = (1 - fc) * c_full + fc * c_clean
        print({"config": args.config, "step": k, "movers": int(mv.sum()), "clean_frac": round(fc, 3),
               "cand": round(cand / n, 1), "skin_cand": round(skin / n, 1), "hits": round(hits / n, 1),
               "valu_per_target_now": round(c_full, 0), "valu_per_target_model": round(model, 0),
               "pass1_change": round(model / c_full - 1, 3), "disp_max_h": round(dmax, 4),
               "disp_p999_h": round(d999, 4), "skin_steps": round(args.skin / (2 * dmax), 1) if dmax > 0 else None},
              flush=True)


if __name__ == "__main__":
    main()
