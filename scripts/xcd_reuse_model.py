"""Force-pass staging traffic against the block -> XCD mapping, modelled (round-5 verdict item 3).

k_force_tiled stages, per workgroup of 256 sorted targets and per dx plane, the three rows' candidate intervals
(x, v, rho/P: 16 + 16 + 8 bytes per slot, three arrays). Every slot is staged by the workgroups of its own column and
of the columns on either side, and by those of the y rows around it. Whether a re-stage hits in an XCD's L2 (4 MB,
MI355X_MICROARCH.md) depends on which XCD runs those workgroups and when. This script replays the staging reads of
one launch, workgroup by workgroup in dispatch order, through one LRU cache of 128-byte lines per XCD, and counts the
lines each XCD fetches (L2 misses = what rocprofv3 FETCH_SIZE counts, Infinity-Cache hits included):

  runs16   the product: runs of 16 consecutive blocks dealt round-robin to the 8 XCDs (common.h xcd_block);
  range    one contiguous block range per XCD;
  yband    XCD k takes a band of y rows of every column: the blocks are ordered column by column within the band
           (a schedule table would map dispatch index -> target range).

The state is a dam-break lattice (SPEC_SPH.md §0 grid: cells 2h in x and y, 2h/6 in z). Workgroups are modelled as
running one after another per XCD (an XCD runs ~128 at once, so reuse distances shorter than that are optimistic).

    python scripts/xcd_reuse_model.py [--scenario nx,ny,nz] [--dx 0.01] [--l2-mb 4]
"""
import argparse
from collections import OrderedDict

import numpy as np


def lattice(nx, ny, nz, dx):
    g = np.stack(np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij"), -1).reshape(-1, 3)
    return ((g + 0.5) * dx).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="16,256,512", help="lattice nx,ny,nz (default: a C5/8 rank's columns)")
    ap.add_argument("--dx", type=float, default=0.01)
    ap.add_argument("--l2-mb", type=float, default=4.0)
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--kinds", default="runs16,range,yband")
    a = ap.parse_args()
    nx, ny, nz = (int(t) for t in a.scenario.split(","))
    x = lattice(nx, ny, nz, a.dx)
    h = 1.2 * a.dx
    cell, cz = 2 * h, 2 * h / 6
    cx = np.floor(x[:, 0] / cell).astype(np.int64)
    cy = np.floor(x[:, 1] / cell).astype(np.int64)
    czz = np.floor(x[:, 2] / cz).astype(np.int64)
    gx, gy, gz = cx.max() + 2, cy.max() + 2, czz.max() + 2
    key = (cx * gy + cy) * gz + czz
    key.sort()
    n = len(key)
    ncell = gx * gy * gz
    cs = np.searchsorted(key, np.arange(ncell + 1))
    B = (n + 255) // 256
    zwin = 7
    # per logical block: the 9 row intervals [c0, c1) of its staged planes
    kf, kl = key[np.arange(B) * 256], key[np.minimum(np.arange(B) * 256 + 255, n - 1)]
    rows = []
    for dxk in (-1, 0, 1):
        for dyk in (-1, 0, 1):
            off = (dxk * gy + dyk) * gz
            ka = np.clip(kf + off - zwin, 0, ncell - 1)
            kb = np.clip(kl + off + zwin, 0, ncell - 1)
            rows.append((cs[ka], cs[kb + 1]))
    c0 = np.stack([r[0] for r in rows], 1)
    c1 = np.stack([r[1] for r in rows], 1)
    lines_per_slot = {16: 8, 8: 16}   # slots per 128-B line for 16-B and 8-B elements

    def block_lines(b):
        out = []
        for arr, esz in ((0, 16), (1, 16), (2, 8)):
            per = lines_per_slot[esz]
            for r in range(9):
                lo, hi = c0[b, r], c1[b, r]
                if hi > lo:
                    out.extend((arr << 40) | l for l in range(lo // per, (hi - 1) // per + 1))
        return out

    # the blocks' column and y row (of their first target) for the band schedule
    bcol = kf // (gy * gz)
    brow = (kf // gz) % gy

    def order(kind):
        if kind == "runs16":
            C = 16
            seq = [[] for _ in range(8)]
            full = B // (8 * C) * (8 * C)
            for d in range(B):
                if d >= full:
                    lb = d
                else:
                    xx, k = d % 8, d // 8
                    lb = ((k // C) * 8 + xx) * C + (k % C)
                seq[d % 8].append(lb)
            return seq
        if kind == "range":
            per = -(-B // 8)
            return [list(range(k * per, min(B, (k + 1) * per))) for k in range(8)]
        if kind == "yband":   # a.bands bands (a multiple of 8): XCD k takes bands k, k + 8, ... one after another
            nb = a.bands
            edges = np.linspace(0, brow.max() + 1, nb + 1).astype(int)
            seq = [[] for _ in range(8)]
            for band in range(nb):
                sel = np.nonzero((brow >= edges[band]) & (brow < edges[band + 1]))[0]
                seq[band % 8] += list(sel[np.lexsort((sel, bcol[sel]))])
            return seq
        raise ValueError(kind)

    cap = int(a.l2_mb * 2**20 / 128)
    design = n * 40
    res = {"scenario": a.scenario, "particles": n, "blocks": int(B), "l2_mb_per_xcd": a.l2_mb,
           "design_bytes_per_particle": 40}
    for kind in a.kinds.split(","):
        miss = 0
        for seq in order(kind):
            lru = OrderedDict()
            for b in seq:
                for ln in block_lines(b):
                    if ln in lru:
                        lru.move_to_end(ln)
                    else:
                        miss += 1
                        lru[ln] = None
                        if len(lru) > cap:
                            lru.popitem(last=False)
        res[kind if kind != "yband" else f"yband{a.bands}"] = {"fetched_MB": round(miss * 128 / 1e6, 1), "bytes_per_particle": round(miss * 128 / n, 1),
                     "over_design": round(miss * 128 / design, 2)}
        print(kind, a.bands, res[kind if kind != "yband" else f"yband{a.bands}"], flush=True)
    print(res)


if __name__ == "__main__":
    main()
