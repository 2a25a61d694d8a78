#!/usr/bin/env python3
"""LDS bank-conflict model of pass 1 (k_density_tiled) at C3 from rest, CPU only.

Rebuilds what one workgroup of the density pass reads from LDS: the C3 lattice sorted by cell key (the
oracle's grid), 256 targets per block in quadrant lane order, each plane's three block intervals
staged back to back, every lane's trimmed row windows (row_window, common.h), and the scan loop (four
candidates per iteration while any lane has four left, then the 1-candidate tail) with its exec
masks. Every ds_read_b128 is then priced with the gfx950 rule (MI355X_MICROARCH.md §LDS): four lane
groups of 16, one LDS cycle per group plus one per extra distinct address on a busy bank (a 16-B read
covers 4 consecutive banks of 64); identical addresses broadcast. The model's conflict share is
compared with the PMC counter SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (profiles/pmc_C3.json) and then
used to rank layouts: the staged slot s sits at LDS float4 index phys(s).

  python scripts/lds_bank_model.py [--blocks 300]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
B128_GROUPS = [np.array(g) for g in B128_GROUPS]


def b128_cycles(addr_slots, active, phys):
    """LDS cycles of one wave's ds_read_b128 (addr in float4 slots, active lanes mask)."""
    cyc = 0
    for g in B128_GROUPS:
        a = addr_slots[g][active[g]]
        if a.size == 0:
            cyc += 1
            continue
        u = np.unique(phys(a))
        quads = u % 16
        cyc += int(np.bincount(quads, minlength=16).max())
    return cyc


LAYOUTS = {
    "linear": lambda s: s,
    "xor4": lambda s: s ^ ((s >> 4) & 3),
    "xor16": lambda s: s ^ ((s >> 4) & 15),
    "x2_4": lambda s: s ^ (((s >> 2) ^ (s >> 4)) & 3),
    "x4_6": lambda s: s ^ (((s >> 4) ^ (s >> 6)) & 3),
    "x4_6_15": lambda s: s ^ (((s >> 4) ^ (s >> 8)) & 15),
    "x4m": lambda s: s ^ (((s >> 4) * 5) & 15),
    "x4m3": lambda s: s ^ (((s >> 4) * 3) & 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=300)
    ap.add_argument("--lane-order", choices=("quadrant", "sorted", "halfx", "halfy"), default="quadrant")
    args = ap.parse_args()
    O = GE.load_oracle()
    pkg = GE.load_package()
    sc = pkg.config_scenario("C3")
    p, _ = pkg.scenario_params(sc)
    op = O.sph_params(3, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                      p.wall_restitution, p.forcing_amp, p.forcing_freq)
    x = O.lattice(3, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    keys = O.grid_keys(op, x).astype(np.int64)
    order = np.argsort(keys, kind="stable")
    x, keys = x[order], keys[order]
    G = [int(v) for v in op.grid.G]
    gx, gy, gz = G
    ncells = gx * gy * gz
    cs = np.searchsorted(keys, np.arange(ncells + 1)).astype(np.int64)
    inv_cell = np.float32(op.grid.inv_cell)
    inv_cz = np.float32(op.grid.inv_cell_z)
    zsub, zwin = 6, int(op.grid.zwin)
    n = len(x)
    nblk = (n + 255) // 256
    rng = np.random.default_rng(7)
    blocks = np.sort(rng.choice(nblk, size=min(args.blocks, nblk), replace=False))
    tot = {k: [0, 0] for k in LAYOUTS}   # [cycles, ideal cycles]
    for b in blocks:
        i0 = b * 256
        idx = np.arange(i0, min(i0 + 256, n))
        pi = x[idx]
        cx = np.minimum(np.floor(pi[:, 0] * inv_cell).astype(np.int64), gx - 1)
        cy = np.minimum(np.floor(pi[:, 1] * inv_cell).astype(np.int64), gy - 1)
        fx = np.clip(pi[:, 0] * inv_cell - cx, 0, 1).astype(np.float32)
        fy = np.clip(pi[:, 1] * inv_cell - cy, 0, 1).astype(np.float32)
        gzf = (pi[:, 2] * inv_cz).astype(np.float32)
        if args.lane_order == "quadrant":
            q = (fx >= 0.5).astype(int) + 2 * (fy >= 0.5).astype(int)
            lanes = np.argsort(q, kind="stable")     # lane -> target (within the block)
        elif args.lane_order in ("halfx", "halfy"):
            q = ((fx if args.lane_order == "halfx" else fy) >= 0.5).astype(int)
            lanes = np.argsort(q, kind="stable")
        else:
            lanes = np.arange(len(idx))
        kf, kl = keys[i0], keys[idx[-1]]
        for pl in range(3):
            c0, ln_ = [], []
            lo_l, len_l = [], []
            for r in range(3):
                dxk, dyk = pl - 1, r - 1
                off = (dxk * gy + dyk) * gz
                ka, kb = kf + off - zwin, kl + off + zwin
                if kb < 0 or ka > ncells - 1:
                    c0.append(0); ln_.append(0)
                else:
                    ka, kb = max(ka, 0), min(kb, ncells - 1)
                    c0.append(int(cs[ka])); ln_.append(int(cs[kb + 1] - cs[ka]))
                xx, yy = cx + dxk, cy + dyk
                gxg = fx if dxk < 0 else (1 - fx if dxk > 0 else np.zeros_like(fx))
                gyg = fy if dyk < 0 else (1 - fy if dyk > 0 else np.zeros_like(fy))
                d2 = gxg * gxg + gyg * gyg
                ok = (xx >= 0) & (xx < gx) & (yy >= 0) & (yy < gy) & (d2 < 1)
                hz = np.sqrt(np.maximum(1 - d2, 0)).astype(np.float32) * np.float32(zsub) + np.float32(1e-3)
                a_, b_ = gzf - hz, gzf + hz
                zlo = np.where(a_ > 0, a_.astype(np.int64), 0)
                zhi = np.where(b_ < gz - 1, b_.astype(np.int64), gz - 1)
                zhi = np.maximum(zhi, 0)
                rowk = (np.clip(xx, 0, gx - 1) * gy + np.clip(yy, 0, gy - 1)) * gz
                r0 = np.where(ok, cs[np.minimum(rowk + zlo, ncells)], 0)
                r1 = np.where(ok, cs[np.minimum(rowk + zhi + 1, ncells)], 0)
                lo_l.append(r0 - c0[-1])
                len_l.append(r1 - r0)
            if sum(ln_) > 1350:
                continue                      # chunked planes: not modelled (~10% at C3)
            o = 0
            for r in range(3):
                lo = (o + lo_l[r])[lanes]
                ln = len_l[r][lanes]
                o += ln_[r]
                for w in range(0, len(lanes), 64):
                    wl, wn = lo[w:w + 64], ln[w:w + 64]
                    if len(wl) < 64:
                        wl = np.concatenate([wl, np.zeros(64 - len(wl), np.int64)])
                        wn = np.concatenate([wn, np.zeros(64 - len(wn), np.int64)])
                    t = 0
                    while (t + 4 <= wn).any():
                        act = t + 4 <= wn
                        for k in range(4):
                            for name, f in LAYOUTS.items():
                                tot[name][0] += b128_cycles(wl + t + k, act, f)
                                tot[name][1] += 4
                        t += 4
                    for j in range(3):   # the tail: each lane from its own t = 4*floor(ln/4)
                        tl = (wn // 4) * 4 + j
                        act = tl < wn
                        if not act.any():
                            break
                        for name, f in LAYOUTS.items():
                            tot[name][0] += b128_cycles(wl + tl, act, f)
                            tot[name][1] += 4
    for name, (cyc, ideal) in tot.items():
        print(f"{name:8s} LDS cycles {cyc:9d}  ideal {ideal:9d}  conflict share {(cyc - ideal) / cyc:.3f}")


if __name__ == "__main__":
    main()
