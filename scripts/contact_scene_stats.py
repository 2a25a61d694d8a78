"""Per-target work of the flat contact form (contact.hip contact_accumulate_flat) on a Model R scene, from the oracle's
state after K steps: candidates per target (the 27 cells of the reference's 4.0 grid, compute:102-105), touching
candidates, chunks a round scans, and the body passes a wave runs, as the kernel schedules them now (a lane's touches
in up to three slots, the wave running max-per-lane passes; chunk by chunk when a lane has more) and with the touches
compacted over the wave's lanes (ceil(touches / 64) passes). CPU only (the oracle restatement, test infrastructure).
    python scripts/contact_scene_stats.py [--steps K] [--n 4096] [--trim]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402

CHUNKS, SLOTS = 8, 3


def sphere(pkg, n):   # scripts/small_n_timing.py, bench.py --table
    rng = np.random.default_rng(1234)
    parts = np.zeros(n, pkg.PARTICLE84)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    parts["position"] = d * (15.0 * rng.random((n, 1)) ** (1 / 3))
    parts["radius"] = rng.uniform(1.5, 2.0, n)
    parts["velocity"] = rng.normal(size=(n, 3))
    parts["mass"] = 0.1 * 4.0 / 3.0 * 3.1415926 * parts["radius"] ** 3
    parts["angularVelocity"] = rng.normal(size=(n, 3))
    parts["momentOfInertia"] = 0.4 * parts["mass"] * parts["radius"] ** 2
    parts["drag"] = rng.uniform(0.5, 1.0, n)
    parts["repulsionStrength"] = 1.0
    parts["rotation"] = (0, 0, 0, 1)
    parts["modeIndex"] = -1
    return parts


def stats(parts, spawn=15.0, trim=False):
    """trim: the rows and end z cells contact.hip's cell_reach / reach_row drop (beyond rA/2 + rmax/2)."""
    x = parts["position"].astype(np.float32)
    r = parts["radius"].astype(np.float32)
    gq = (x + np.float32(spawn)) * np.float32(0.25)
    c = np.clip(np.floor(gq).astype(np.int64), 0, 31)
    fr = gq - c.astype(np.float32)
    rmax = float(r.max())
    key = (c[:, 0] * 32 + c[:, 1]) * 32 + c[:, 2]
    order = np.argsort(key, kind="stable")
    ks = key[order]
    cs = np.searchsorted(ks, np.arange(32 ** 3 + 1))
    out = {"cand": [], "touch": [], "chunks": [], "passes_now": [], "passes_compact": []}
    for a in range(len(x)):
        cx, cy, cz = c[a]
        z0, z1 = max(cz - 1, 0), min(cz + 1, 31)
        b = ((0.5 * r[a] + 0.5 * rmax) * 1.001 + 0.001) * 0.25
        flat = []
        for k in range(9):
            xx, yy = cx + k // 3 - 1, cy + k % 3 - 1
            if not (0 <= xx < 32 and 0 <= yy < 32):
                continue
            if trim:
                lx = fr[a, 0] if k // 3 == 0 else (1 - fr[a, 0] if k // 3 == 2 else 0.0)
                ly = fr[a, 1] if k % 3 == 0 else (1 - fr[a, 1] if k % 3 == 2 else 0.0)
                l2 = lx * lx + ly * ly
                if l2 > b * b:
                    continue
                z0 = cz - 1 if cz > 0 and not (l2 + fr[a, 2] ** 2 > b * b) else cz
                z1 = cz + 1 if cz < 31 and not (l2 + (1 - fr[a, 2]) ** 2 > b * b) else cz
            row = (xx * 32 + yy) * 32
            flat.extend(order[cs[row + z0]:cs[row + z1 + 1]])
        flat = np.asarray(flat, np.int64)
        d = x[a] - x[flat]
        dist = np.sqrt((d * d).sum(1))
        t = ((r[a] * 0.5 + r[flat] * 0.5) - dist > 0.001) & (flat != a)
        f = np.nonzero(t)[0]
        total = len(flat)
        out["cand"].append(total)
        out["touch"].append(len(f))
        now = comp = chunks = 0
        for rnd in range(0, max(total, 1), 64 * CHUNKS):
            chunks += min(CHUNKS, -(-(total - rnd) // 64))
            g = f[(f >= rnd) & (f < rnd + 64 * CHUNKS)] - rnd
            per_lane = np.bincount(g % 64, minlength=64)
            if per_lane.max(initial=0) > SLOTS:
                now += len(np.unique(g // 64))
            else:
                now += int(per_lane.max(initial=0))
            comp += -(-len(g) // 64)
        out["chunks"].append(chunks)
        out["passes_now"].append(now)
        out["passes_compact"].append(comp)
    return {k: round(float(np.mean(v)), 3) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="0,20,300")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--trim", action="store_true", help="count the candidates after contact.hip's cell skipping")
    args = ap.parse_args()
    pkg = GE.load_package()
    O = GE.load_oracle()
    parts, dt = sphere(pkg, args.n), 0.01
    cp = O.contact_params(dt)
    p = parts.view(O.PARTICLE84).copy()
    done = 0
    for k in [int(s) for s in args.steps.split(",")]:
        while done < k:
            p, _ = O.contact_step(cp, p, nthreads=8)
            done += 1
        print({"scene": "sphere R=15", "n": args.n, "step": k, "trim": args.trim, **stats(p, trim=args.trim)},
              flush=True)


if __name__ == "__main__":
    main()
