"""Host check of the incremental re-sort's counting formulas (sph-test_amd/csrc/resort.hip header).

The formulas place every particle by counting alone: stayers (key unchanged) and movers (key
changed, ranked among themselves). They are restated here in numpy, together with the cell-start
update, and checked against the stable argsort on random cases: 0%, 1%, 30% and 100% movers, ties,
and empty cells. The GPU kernels are compared bit for bit with the full radix sort in
tests/test_gpu_resort.py.
"""
import numpy as np
import pytest


def _comp(k, i):
    return np.asarray(k, np.int64) * (1 << 32) + np.asarray(i, np.int64)


def resort_emulation(ks, newk, nc):
    n = len(ks)
    cs_old = np.searchsorted(ks, np.arange(nc + 1), side="left")
    movers = np.nonzero(newk != ks)[0]                  # Mi: index order
    mk = newk[movers]
    cm = _comp(mk, movers)
    rank = np.array([(cm < c).sum() for c in cm], dtype=np.int64)
    ms = np.sort(cm)                                     # sorted-mover table
    dst = np.empty(n, np.int64)
    for r, x in enumerate(movers):
        k = mk[r]
        q = min(max(x, cs_old[k]), cs_old[k + 1])
        dst[x] = (q - np.searchsorted(movers, q, side="left")) + rank[r]
    a = np.concatenate([[0], np.cumsum(newk != ks)])    # A(i) = movers with index < i
    for i in np.nonzero(newk == ks)[0]:
        dst[i] = (i - a[i]) + np.searchsorted(ms, _comp(ks[i], i), side="left")
    perm = np.empty(n, np.int64)
    perm[dst] = np.arange(n)
    # cell starts: cs_old + (#movers with new key < k) - (#movers with old key < k)
    kk = np.arange(nc + 1)
    cs_new = cs_old + np.searchsorted(ms, _comp(kk, 0), side="left") \
        - np.searchsorted(ks[movers], kk, side="left")
    return perm, cs_new


@pytest.mark.parametrize("frac", [0.0, 0.01, 0.3, 1.0])
def test_resort_formulas_match_stable_sort(frac):
    rng = np.random.default_rng(int(frac * 1000))
    for _ in range(40):
        n = int(rng.integers(1, 2000))
        nc = int(rng.integers(1, 300))
        ks = np.sort(rng.integers(0, nc, n)).astype(np.int64)
        newk = ks.copy()
        mv = rng.random(n) < frac
        newk[mv] = rng.integers(0, nc, int(mv.sum()))
        perm, cs_new = resort_emulation(ks, newk, nc)
        ref = np.argsort(newk, kind="stable")
        assert np.array_equal(perm, ref)
        assert np.array_equal(cs_new, np.searchsorted(newk[ref], np.arange(nc + 1), side="left"))


def range_ranks(ks, newk, G, win=2048, blocks=False):
    """resort.hip k_mv_rank restated: workgroup b owns the old slots [x0, x1) = [b·n/G, (b+1)·n/G) and the new keys
    [ks[x0], ks[x1]) (first range from 0, last to infinity); rk counts the movers below the key range plus those in
    range with a smaller (key, slot). The slots staged are those in [xw, x1), xw = x0 − win: a source entry's rank is
    the movers below x0 plus the staged slots in [x0, x); A(q) for a dest entry likewise from x0 (minus the staged
    slots in [q, x0) when q < x0), or counted against the whole list when q < xw (a cell of more than win slots)."""
    n = len(ks)
    movers = np.nonzero(newk != ks)[0]
    mk = newk[movers]
    nc = int(max(ks.max(initial=0), newk.max(initial=0))) + 1
    cs_old = np.concatenate([np.searchsorted(ks, np.arange(nc + 1), side="left"), [n]])
    rk = np.full(len(movers), -1, np.int64)
    ri = np.full(len(movers), -1, np.int64)
    aq = np.full(len(movers), -1, np.int64)
    cs_new = np.full(nc + 1, -1, np.int64)
    bnd = []
    nbk = (n + 255) // 256 if blocks else n
    for b in range(G):
        x0, x1 = min(nbk * b // G * (256 if blocks else 1), n), min(nbk * (b + 1) // G * (256 if blocks else 1), n)
        kd0 = 0 if b == 0 else (ks[x0] if x0 < n else np.iinfo(np.int64).max)
        kd1 = np.iinfo(np.int64).max if b == G - 1 else (ks[x1] if x1 < n else np.iinfo(np.int64).max)
        xw = max(x0 - win, 0)
        ind = (mk >= kd0) & (mk < kd1)
        ins = (movers >= x0) & (movers < x1)
        staged = np.sort(movers[(movers >= xw) & (movers < x1)])
        below_k, below_x0 = int((mk < kd0).sum()), int((movers < x0).sum())
        r0 = int(np.searchsorted(staged, x0, side="left"))
        c = _comp(mk, movers)
        for e in np.nonzero(ind)[0]:
            assert rk[e] < 0, "a mover in two key ranges"
            rk[e] = below_k + int((c[ind] < c[e]).sum())
            q = min(max(int(movers[e]), int(cs_old[mk[e]])), int(cs_old[mk[e] + 1]))
            assert int(cs_old[kd0]) <= q <= x1
            if q >= xw:
                aq[e] = below_x0 + int(np.searchsorted(staged, q, side="left")) - r0
            else:
                aq[e] = int((movers < q).sum())
        for e in np.nonzero(ins)[0]:
            assert ri[e] < 0, "a mover in two slot ranges"
            ri[e] = below_x0 + int(np.searchsorted(staged, movers[e], side="left")) - r0
        # the range's cells kd0 < k < kd1 in place, its first cell kd0 through the boundary table
        if x0 < n or b == 0:
            mo = ks[movers]
            below_ko = int((mo < kd0).sum())
            dkeys = np.sort(mk[ind])
            okeys = np.sort(mo[(mo >= kd0) & (mo < kd1)])
            klo, khi = int(kd0) + 1, max(int(min(kd1, nc + 1)), int(kd0) + 1)
            for k in range(klo, khi):
                d = below_k - below_ko + int(np.searchsorted(dkeys, k)) - int(np.searchsorted(okeys, k))
                cs_new[k] = cs_old[k] + d
            # the kernel's segment form: events +1 (dest key) / −1 (old key) merged, Δ constant between them
            ev = sorted([(int(k), 0, 1) for k in dkeys] + [(int(k), 1, -1) for k in okeys])
            seg_cs = {}
            dlt = below_k - below_ko
            for j in range(len(ev) + 1):
                st = klo if j == 0 else max(ev[j - 1][0] + 1, klo)
                en = khi if j == len(ev) else min(ev[j][0] + 1, khi)
                for k in range(st, max(en, st)):
                    seg_cs[k] = cs_old[k] + dlt
                if j < len(ev):
                    dlt += ev[j][2]
            assert all(seg_cs.get(k, cs_old[k]) == cs_new[k] for k in range(klo, khi))
            bnd.append((int(kd0), int(cs_old[kd0]) + below_k - below_ko))
    for k, v in bnd:
        cs_new[k] = v
    return movers, mk, rk, ri, aq, cs_old, cs_new


@pytest.mark.parametrize("frac", [0.0, 0.01, 0.3, 1.0])
@pytest.mark.parametrize("G", [1, 3, 16, 256])
def test_range_ranks_equal_global_ranks(frac, G):
    rng = np.random.default_rng(int(frac * 1000) + G)
    for _ in range(20):
        n = int(rng.integers(1, 1500))
        nc = int(rng.integers(1, 300))
        ks = np.sort(rng.integers(0, nc, n)).astype(np.int64)
        newk = ks.copy()
        mv = rng.random(n) < frac
        newk[mv] = rng.integers(0, nc + 1, int(mv.sum()))    # nc: the sentinel key (inactive / left the window)
        win = int(rng.integers(1, 64)) if rng.random() < 0.5 else 2048   # small windows: the counted fallback
        blocks = bool(rng.random() < 0.5)   # ranges of whole 256-slot blocks (the kernel) or of n/G slots
        movers, mk, rk, ri, aq, cs_old, cs_new = range_ranks(ks, newk, min(G, max(n // 256, 1)) if G == 256 else G,
                                                             win, blocks)
        c = _comp(mk, movers)
        assert np.array_equal(rk, np.argsort(np.argsort(c, kind="stable"), kind="stable"))
        assert np.array_equal(ri, np.arange(len(movers)))
        q = np.minimum(np.maximum(movers, cs_old[mk]), cs_old[mk + 1])
        assert np.array_equal(aq, np.searchsorted(movers, q, side="left"))
        ref = np.sort(newk, kind="stable")
        assert np.array_equal(cs_new, np.searchsorted(ref, np.arange(len(cs_new)), side="left"))
