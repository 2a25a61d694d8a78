#!/usr/bin/env python3
"""Pair-symmetry model of the force pass (k_force_tiled), CPU only.

The force pass evaluates every neighbour pair twice, once from each target's lane (as the reference's
contact pass does, SimulateParticles.compute:248-294). A half-shell evaluation would compute a pair whose
partner is a target of the SAME 256-target workgroup once and hand the partner its (antisymmetric) share.
This counts, on the sorted state the kernel sees (cell keys x-slowest, stable order, 256 consecutive targets
per workgroup), the hits (q <= 2, self included, as the mask walk takes them) and the share whose partner is
in the target's own workgroup, and prices the best case: every in-block pair evaluated once, the partner's
share free.

  python scripts/pair_symmetry_model.py [C3|C2] [--mid STEPS]   (--mid: advance on the oracle first)
"""
import sys
import time
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402


def model(x, keys, h, blk=256):
    order = np.argsort(keys, kind="stable")
    xs = x[order]
    n = len(xs)
    tree = cKDTree(xs.astype(np.float64))
    pairs = tree.query_pairs(2.0 * float(h), output_type="ndarray")       # unordered i < j, r <= 2h
    same = (pairs[:, 0] // blk) == (pairs[:, 1] // blk)
    ordered = 2 * len(pairs) + n                                            # both directions + self
    in_block = 2 * int(same.sum())                                          # ordered in-block pairs (no self)
    saved = in_block // 2 + n                                               # each in-block pair once, no self
    return {"particles": n, "hits_per_target": ordered / n, "in_block_share_of_hits": in_block / ordered,
            "self_share": n / ordered, "pair_evals_saved_frac": saved / ordered}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "C3"
    mid = int(sys.argv[sys.argv.index("--mid") + 1]) if "--mid" in sys.argv else 0
    O = GE.load_oracle()
    pkg = GE.load_package()
    sc = pkg.config_scenario(cfg)
    p, dt = pkg.scenario_params(sc)
    op = O.sph_params(sc.dim, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                      p.wall_restitution, p.forcing_amp, p.forcing_freq)
    x = O.lattice(sc.dim, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    v = np.zeros_like(x)
    ids = np.arange(len(x), dtype=np.int32)
    t0 = time.time()
    for s in range(mid):
        x, v, ids, _, _, _ = O.sph_step(op, x, v, ids, dt, float(np.float32(s * dt)), nthreads=8)
    res = {"config": cfg, "state": f"step {mid}" if mid else "rest", "advance_s": round(time.time() - t0, 1)}
    res.update(model(x, O.grid_keys(op, x).astype(np.int64), p.h))
    print(res, flush=True)


if __name__ == "__main__":
    main()
