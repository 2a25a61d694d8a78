"""Model S input states for the GPU-vs-oracle parity tests (tests/test_gpu_parity_headline.py).

Every state is (positions, velocities) in particle-index order, uploaded to both sides through
`sph_upload_state` / the oracle's `sph_step_diag`. Besides the resting lattice and a mid-collapse
state (made on the GPU), two synthetic states drive the branches a resting dam-break never takes:

  * wall_state: a lattice with random velocities of about one z sub-cell per step, plus a shell of
    particles set exactly on the six box walls moving outward, so one step clamps and reflects
    (SPEC_SPH.md §2 walls) on every wall;
  * splash_state: x-columns of alternating dense and sparse fluid, so workgroups of sparse targets
    see neighbour planes far longer than the LDS budget (the chunked and the global-gather paths of
    wcsph_tiled.hip). `block_paths` predicts, from the sorted keys alone, how many planes / rows
    take those paths, with the kernels' budgets.
"""
from __future__ import annotations

import numpy as np

# wcsph_tiled.hip budgets: targets per workgroup, LDS candidates per plane (density, force)
TT_BLK, TT_GCAP, TF_GCAP = 256, 1350, 1270   # wcsph_tiled.hip (the plane budgets)


def wall_state(O, op, nx, ny, nz, dx, dt, seed=11):
    """A lattice (the oracle's dam-break init) with random velocities of about one z sub-cell per
    step, and ~6% of the particles moved exactly onto a wall with an outward velocity."""
    x = O.lattice(3, nx, ny, nz, dx, seed=seed)
    rng = np.random.default_rng(seed)
    sub = 2.0 * float(op.h) / 6.0
    v = (rng.uniform(-1.0, 1.0, x.shape) * (sub / dt)).astype(np.float32)
    L = np.array([op.L[0], op.L[1], op.L[2]], np.float32)
    pick = rng.choice(len(x), size=max(6, len(x) // 16), replace=False)
    for k, i in enumerate(pick):
        a, hi = (k // 2) % 3, k % 2
        x[i, a] = L[a] if hi else np.float32(0.0)
        speed = np.float32(abs(v[i, a]) + 0.5 * sub / dt)
        v[i, a] = speed if hi else -speed
    return x, v


def splash_state(nx_cols, ny, nz, cell, dense_per_col, sparse_per_col, box, seed=3):
    """Uniform random particles in x-columns of width `cell` (the grid's 2h), alternating dense and
    sparse; velocities small and random. Positions avoid exact duplicates (continuous uniform)."""
    rng = np.random.default_rng(seed)
    xs = []
    for c in range(nx_cols):
        m = dense_per_col if c % 2 == 0 else sparse_per_col
        p = rng.random((m, 3)).astype(np.float32)
        p[:, 0] = (np.float32(c) + p[:, 0]) * np.float32(cell)
        p[:, 1] *= np.float32(box[1])
        p[:, 2] *= np.float32(box[2])
        xs.append(p)
    x = np.concatenate(xs).astype(np.float32)
    x = x[rng.permutation(len(x))]
    v = (rng.normal(size=x.shape) * 0.05).astype(np.float32)
    return x, v


def grid_dims(op):
    """(sub-columns, gy, gz, zwin, xsub): keys count x sub-columns (SPEC_SPH.md §0)."""
    xs = int(op.grid.xsub)
    return int(op.grid.G[0]) * xs, int(op.grid.G[1]), int(op.grid.G[2]), int(op.grid.zwin), xs


def block_paths(O, op, x):
    """How the tiled passes will process state x: [density planes chunked, density rows global,
    force planes chunked, force rows global], summed over workgroups (the kernels' counters count
    the same events, sph_read_path_counts)."""
    gx, gy, gz, zwin, xs = grid_dims(op)
    nc = gx * gy * gz
    keys = O.grid_keys(op, x).astype(np.int64)
    sk = np.sort(keys, kind="stable")
    cs = np.searchsorted(sk, np.arange(nc + 1), side="left").astype(np.int64)
    n = len(sk)
    out = np.zeros(4, np.int64)
    for i0 in range(0, n, TT_BLK):
        kf, kl = sk[i0], sk[min(i0 + TT_BLK, n) - 1]
        for p in range(2 * xs + 1):
            lens = []
            for r in range(3):
                dxk, dyk = p - xs, r - 1
                off = (dxk * gy + dyk) * gz
                ka, kb = kf + off - zwin, kl + off + zwin
                if kb < 0 or ka > nc - 1:
                    lens.append(0)
                    continue
                ka, kb = max(ka, 0), min(kb, nc - 1)
                lens.append(int(cs[kb + 1] - cs[ka]))
            tot = sum(lens)
            for base, (gcap, ctr) in enumerate(((TT_GCAP, 0), (TF_GCAP, 2))):
                if tot > gcap:
                    out[ctr] += 1
                    out[ctr + 1] += sum(1 for ln in lens if ln > 4 * gcap)
    return out
