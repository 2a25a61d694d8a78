#!/usr/bin/env python3
"""Candidate-volume model of the neighbour passes for other cell shapes, CPU only.

For the C3 lattice at rest it counts, per target, the candidates of the trimmed row windows (the kernels'
row_window, generalised to a cell of cx × cy in units of 2h, z sub-cells of h/3), and prices pass 1's scan
on the wave level the way the kernel runs it: per row, the wave runs max over its lanes of the 4-candidate
iterations, then max of the 1-candidate tail iterations (VALU per iteration from the ISA: ~85 for four
candidates, ~25 for one, ~25 per row of window set-up). It also counts the candidates a 256-target
block stages (x-slowest keys, consecutive sorted targets), which pass 2 pays 32 B each for.

  python scripts/cell_shape_model.py [--blocks 200]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402

V4, V1, VROW = 85.0, 25.0, 25.0


def model(x, h, box, sx, sy, zsub, nblocks, rng, lane_order="quadrant"):
    """sx, sy: cell size in x, y in units of 2h. Returns per-target means."""
    cell_x, cell_y = np.float32(2 * h * sx), np.float32(2 * h * sy)
    cz = np.float32(2 * h / zsub)
    gx = int(np.floor(box[0] / cell_x)) + 1
    gy = int(np.floor(box[1] / cell_y)) + 1
    gz = int(np.floor(box[2] / cz)) + 1
    rx, ry = int(np.ceil(1 / sx)), int(np.ceil(1 / sy))     # neighbour rows each side
    cxi = np.minimum((x[:, 0] / cell_x).astype(np.int64), gx - 1)
    cyi = np.minimum((x[:, 1] / cell_y).astype(np.int64), gy - 1)
    czi = np.minimum((x[:, 2] / cz).astype(np.int64), gz - 1)
    keys = (cxi * gy + cyi) * gz + czi
    order = np.argsort(keys, kind="stable")
    x, keys, cxi, cyi = x[order], keys[order], cxi[order], cyi[order]
    ncells = gx * gy * gz
    cs = np.searchsorted(keys, np.arange(ncells + 1))
    n = len(x)
    nblk = (n + 255) // 256
    blocks = rng.choice(nblk, size=min(nblocks, nblk), replace=False)
    zwin = zsub + 1
    cand = valu = staged = rows_nz = 0.0
    ntarg = 0
    for b in blocks:
        idx = np.arange(b * 256, min(b * 256 + 256, n))
        p = x[idx]
        cx, cy = cxi[idx], cyi[idx]
        fx = (p[:, 0] / cell_x - cx).astype(np.float32)          # in-cell fraction (cell units)
        fy = (p[:, 1] / cell_y - cy).astype(np.float32)
        gzf = (p[:, 2] / cz).astype(np.float32)
        if lane_order == "quadrant":
            lanes = np.argsort((fx >= 0.5).astype(int) + 2 * (fy >= 0.5).astype(int), kind="stable")
        else:
            lanes = np.arange(len(idx))
        kf, kl = keys[idx[0]], keys[idx[-1]]
        L = []
        for dxk in range(-rx, rx + 1):
            for dyk in range(-ry, ry + 1):
                # gap to the row's cell in units of 2h
                gxg = np.where(dxk < 0, fx + (-dxk - 1), np.where(dxk > 0, (1 - fx) + (dxk - 1), 0)) * sx
                gyg = np.where(dyk < 0, fy + (-dyk - 1), np.where(dyk > 0, (1 - fy) + (dyk - 1), 0)) * sy
                d2 = gxg * gxg + gyg * gyg
                xx, yy = cx + dxk, cy + dyk
                ok = (xx >= 0) & (xx < gx) & (yy >= 0) & (yy < gy) & (d2 < 1)
                hz = np.sqrt(np.maximum(1 - d2, 0)) * zsub + 1e-3
                zlo = np.maximum((gzf - hz).astype(np.int64), 0)
                zhi = np.clip((gzf + hz).astype(np.int64), 0, gz - 1)
                rowk = (np.clip(xx, 0, gx - 1) * gy + np.clip(yy, 0, gy - 1)) * gz
                r0 = cs[np.minimum(rowk + zlo, ncells)]
                r1 = cs[np.minimum(rowk + zhi + 1, ncells)]
                L.append(np.where(ok, r1 - r0, 0))
                # block interval of this row offset
                off = (dxk * gy + dyk) * gz
                ka, kb = max(kf + off - zwin, 0), min(kl + off + zwin, ncells - 1)
                if kb >= ka:
                    staged += cs[kb + 1] - cs[ka]
        L = np.array(L)[:, lanes]                     # rows x lanes
        cand += L.sum()
        rows_nz += (L > 0).sum()
        for w in range(0, L.shape[1], 64):
            Lw = L[:, w:w + 64]
            valu += (V4 * (Lw // 4).max(axis=1) + V1 * (Lw % 4).max(axis=1) + VROW).sum() * 64 / Lw.shape[1]
        ntarg += len(idx)
    return {"cells": f"{sx}x{sy} (2h units), zsub {zsub}", "rows": (2 * rx + 1) * (2 * ry + 1),
            "candidates": round(cand / ntarg, 1), "nonempty_rows": round(rows_nz / ntarg, 2),
            "pass1_valu_per_target": round(valu / ntarg, 0), "staged_per_target": round(staged / ntarg, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=200)
    args = ap.parse_args()
    O = GE.load_oracle()
    pkg = GE.load_package()
    sc = pkg.config_scenario("C3")
    p, _ = pkg.scenario_params(sc)
    x = O.lattice(3, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    for sx, sy in ((1, 1), (1, 0.5), (0.5, 0.5)):
        for order in ("quadrant", "sorted"):
            r = model(x, p.h, p.box, sx, sy, 6, args.blocks, np.random.default_rng(3), order)
            r["lanes"] = order
            print(r, flush=True)


if __name__ == "__main__":
    main()
