"""Pass-2 lane balance, modelled (round-5 verdict item 2).

The force pass (wcsph_tiled.hip k_force_tiled) gives each lane one target, in sorted order, 64 consecutive targets per
wave, and walks one dx plane at a time (the plane is what LDS holds): a wave runs as many 4-hit trips per plane as its
busiest lane needs. This script counts, for a real particle state, every target's hits per plane (q <= 2 neighbours,
the target itself included, as the mask walk visits them) and prices the walk's lane-slots under:

  S0  the product: per wave and plane, trips = max over the 64 lanes of ceil(h_p / 4);
  S1  one walk over all three planes (all of a block's planes staged together: 3x the LDS per workgroup):
      trips = max over lanes of ceil((h_-1 + h_0 + h_+1) / 4);
  S1b the two side planes (dx = -1, +1) in one walk, the centre plane alone (2x the LDS per workgroup):
      trips = max of ceil((h_-1 + h_+1) / 4) + max of ceil(h_0 / 4);
  S2  two lanes per target, each plane's hits split at ceil(h_p / 2) (a split fixed by the target alone, so the
      result does not depend on the block partition): 32 targets per wave, trips = max over lanes of the halves;
  S3  the wave's hits dealt out as 4-hit chunks of one target each (chunk boundaries fixed by the target alone, chunk
      sums added in order by the owner): trips = ceil(chunks / 64) per wave and plane, before any cost of the
      hand-out (target state by ds_bpermute, the k-th set bit, the chunk sums through LDS);
  S4  (r6) the workgroup's 256 targets dealt to its four waves in order of their hit counts (total, centre plane, or
      4-hit trips), so a wave's lanes need similar trip counts; a target's sums stay on one lane in visit order.

busy = useful hit-slots / issued lane-slots (64 x 4 per trip). The product's measured figure (SPH_DIAG counters,
scripts/pass_util.py) is 66-71 % from rest; S0 should reproduce it.

    python scripts/lane_balance_model.py [--npz state.npz (key "x": positions, float32 [n, 3])] [--config C3]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def state(args):
    import __graft_entry__ as GE
    pkg = GE.load_package()
    sc = pkg.config_scenario(args.config)
    p, _ = pkg.scenario_params(sc)
    if args.npz:
        x = np.load(args.npz)["x"].astype(np.float32)
    else:
        O = GE.load_oracle()
        x = O.lattice(sc.dim, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    return x, float(p.h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--npz", default="")
    args = ap.parse_args()
    x, h = state(args)
    n = len(x)
    cell = 2.0 * h
    cx = np.floor(x[:, 0] / cell).astype(np.int64)
    cy = np.floor(x[:, 1] / cell).astype(np.int64)
    cz = np.floor(x[:, 2] / (cell / 6.0)).astype(np.int64)
    order = np.lexsort((np.arange(n), cz, cy, cx))   # (key, index): the stable radix sort's order
    xs, cxs = x[order], cx[order]
    pairs = cKDTree(xs.astype(np.float64)).query_pairs(2.0 * h, output_type="ndarray")
    i, j = pairs[:, 0], pairs[:, 1]
    hp = np.zeros((n, 3), np.int64)   # hits per plane dx = -1, 0, +1 (self in plane 0)
    for a, b in ((i, j), (j, i)):
        np.add.at(hp, (a, cxs[b] - cxs[a] + 1), 1)
    hp[:, 1] += 1
    nw = n // 64
    w = hp[: nw * 64].reshape(nw, 64, 3)
    useful = w.sum()
    c4 = lambda v: -(-v // 4)   # noqa: E731
    s0 = 64 * 4 * c4(w).max(axis=1).sum()
    s1 = 64 * 4 * c4(w.sum(axis=2)).max(axis=1).sum()
    s1b = 64 * 4 * (c4(w[:, :, 0] + w[:, :, 2]).max(axis=1).sum() + c4(w[:, :, 1]).max(axis=1).sum())
    halves = np.stack([-(-w // 2), w // 2], axis=2)        # [wave, 64 targets, 2 halves, 3 planes]
    h2 = halves.reshape(nw * 2, 64, 3)                     # 32 targets (64 lanes) per wave
    s2 = 64 * 4 * c4(h2).max(axis=1).sum()
    chunks = c4(w).sum(axis=1)                             # [wave, plane] 4-hit chunks
    s3 = 64 * 4 * (-(-chunks // 64)).sum()
    # S4: the block's 256 targets re-dealt to lanes by hit count (a permutation inside the workgroup; each target's sums
    # stay on one lane in visit order, so the results keep every bit): waves of 64 consecutive in the sorted order
    nb = n // 256
    blk = hp[: nb * 256].reshape(nb, 256, 3)
    def s4(key):
        o = np.argsort(key(blk), axis=1, kind="stable")
        srt = np.take_along_axis(blk, o[:, :, None], axis=1).reshape(nb * 4, 64, 3)
        return 64 * 4 * c4(srt).max(axis=1).sum(), int(srt.sum())
    s4t, u4 = s4(lambda b: b.sum(axis=2))
    s4c, _ = s4(lambda b: b[:, :, 1] * 1000 + b[:, :, 0] + b[:, :, 2])
    s4q, _ = s4(lambda b: c4(b).sum(axis=2) * 1000 + b[:, :, 1])
    s0b = 64 * 4 * c4(blk.reshape(nb * 4, 64, 3)).max(axis=1).sum()
    per_t = hp.sum(axis=1)
    out = {"config": args.config, "state": args.npz or "lattice", "particles": n, "h": h,
           "hits_per_target_mean": round(float(per_t.mean()), 2),
           "hits_per_plane_mean": [round(float(v), 2) for v in hp.mean(axis=0)],
           "busy_S0_product": round(float(useful) / s0, 4), "busy_S1_three_planes": round(float(useful) / s1, 4),
           "busy_S1b_side_planes_together": round(float(useful) / s1b, 4),
           "busy_S2_two_lanes_per_target": round(float(useful) / s2, 4), "busy_S3_chunks_before_overhead": round(float(useful) / s3, 4),
           "busy_S4_sorted_by_hits": round(u4 / s4t, 4), "busy_S4_sorted_by_centre_plane": round(u4 / s4c, 4),
           "busy_S4_sorted_by_trips": round(u4 / s4q, 4), "walk_slots_S4_vs_S0": round(float(min(s4t, s4c, s4q)) / s0b, 4),
           "walk_slots_vs_S0": {"S1": round(float(s1) / s0, 4), "S1b": round(float(s1b) / s0, 4), "S2": round(float(s2) / s0, 4), "S3": round(float(s3) / s0, 4)}}
    print(out, flush=True)


if __name__ == "__main__":
    main()
