"""CPU checks of two identities the Model R contact pass relies on (sph-test_amd/csrc/contact.hip), on float32
restatements of its pair body in the kernel's operation order (numpy float32: IEEE single, no fused multiply-add,
correctly rounded sqrt and division, as the kernel compiles with fp contract off):

* reaction_equals_own: b's thread evaluates the pair body from its side, contact_pair(B, A), and scatters its torqueB
  into a (SimulateParticles.compute:291-294). The kernel takes that term from a's own evaluation instead: the hit codes
  agree and torqueB(B, A) equals torqueA(A, B) up to the sign of a zero component, so the truncated int terms agree.
* the flat form's square-root-free reject is a superset of the reference's test reff − |d| > 0.001 (:253).

Pairs are random, plus the degenerate ones: equal coordinates (zero components of delta), overlaps near the 0.001
threshold, slip speeds near the 1e-4 threshold, wide radius ranges."""
import numpy as np

f32 = np.float32
SCALE = f32(10000.0)


def cross(a, b):
    return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                     a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], 1)


def dot(a, b):
    return a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1] + a[:, 2] * b[:, 2]


def length(a):
    return np.sqrt(dot(a, a))


def saturate(x):
    return np.where(x > 0, np.where(x < 1, x, f32(1)), f32(0)).astype(f32)


def ftoi(x):
    x = x.astype(np.float64)
    out = np.zeros(x.shape, np.int64)
    ok = ~np.isnan(x)
    out[ok] = np.trunc(np.clip(x[ok], -2147483648.0, 2147483647.0)).astype(np.int64)
    return out


def contact_pair(c, pa, va, wa, ra, pb, vb, wb, rb):
    """contact.hip contact_pair (compute:248-295), vectorised: hit code (0, 1, 2) and torqueA, torqueB."""
    with np.errstate(all="ignore"):
        eRA = ra * f32(0.5)
        eRB = rb * f32(0.5)
        delta = pa - pb
        dist = length(delta)
        overlap = (eRA + eRB) - dist
        hit1 = overlap > f32(0.001)
        dirv = delta / dist[:, None]
        overlapFalloff = saturate(overlap / (eRA + eRB))
        cpA = pa - dirv * eRA[:, None]
        cpB = pb + dirv * eRB[:, None]
        sA = va + cross(wa, cpA - pa)
        sB = vb + cross(wb, cpB - pb)
        rel = sA - sB
        tangent = rel - dirv * dot(rel, dirv)[:, None]
        slip = length(tangent)
        hit2 = hit1 & (slip > f32(1e-4))
        fdir = tangent / slip[:, None]
        tin = np.abs(slip * c["torque_factor"])
        d = tin.astype(np.float64)
        fmag = (d * np.sqrt(np.sqrt(d))).astype(f32)          # pow125_r
        fmag = np.minimum(fmag, f32(10.0))
        trs = overlapFalloff * overlapFalloff
        eRTA = trs * eRA * c["roll_mult"]
        eRTB = trs * eRB * c["roll_mult"]
        tA = cross(-dirv * eRTA[:, None], -fdir * fmag[:, None])
        tB = cross(dirv * eRTB[:, None], fdir * fmag[:, None])
    code = np.where(hit2, 2, np.where(hit1, 1, 0))
    return code, tA, tB


def pairs(rng, n):
    pa = rng.normal(size=(n, 3)).astype(f32) * f32(3)
    ra = rng.uniform(1.0, 2.5, n).astype(f32)
    rb = rng.uniform(1.0, 2.5, n).astype(f32)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    # distances around the contact distance and the 0.001 threshold
    reff = (ra * f32(0.5) + rb * f32(0.5)).astype(np.float64)
    k = rng.integers(0, 3, n)
    dist = np.where(k == 0, reff * rng.uniform(0.2, 1.1, n), reff - 0.001 + rng.normal(scale=1e-6, size=n))
    pb = (pa - (u * dist[:, None])).astype(f32)
    # zero components of delta: copy coordinates
    z = rng.integers(0, 4, n)
    for ax in range(3):
        m = z == ax + 1
        pb[m, ax] = pa[m, ax]
    va = rng.normal(size=(n, 3)).astype(f32)
    vb = va + (rng.normal(size=(n, 3)) * np.where(rng.random(n) < 0.2, 1e-5, 1.0)[:, None]).astype(f32)
    wa = rng.normal(size=(n, 3)).astype(f32)
    wb = rng.normal(size=(n, 3)).astype(f32)
    still = rng.random(n) < 0.05   # identical velocities and spins: slip exactly 0
    vb[still] = va[still]
    wa[still] = 0
    wb[still] = 0
    return pa, va, wa, ra, pb, vb, wb, rb


def test_reaction_torque_equals_own_torque():
    rng = np.random.default_rng(7)
    c = {"torque_factor": f32(1.0), "roll_mult": f32(1.0)}
    dt = f32(0.01)
    pa, va, wa, ra, pb, vb, wb, rb = pairs(rng, 200_000)
    h_ab, tA, _ = contact_pair(c, pa, va, wa, ra, pb, vb, wb, rb)
    h_ba, _, tB2 = contact_pair(c, pb, vb, wb, rb, pa, va, wa, ra)
    assert np.array_equal(h_ab, h_ba)
    m = h_ab == 2
    assert m.sum() > 50_000 and (h_ab == 1).sum() > 1000 and (h_ab == 0).sum() > 10_000
    assert np.array_equal(tA[m], tB2[m])            # equal as values (+0 == -0)
    assert np.array_equal(ftoi(tA[m] * dt * SCALE), ftoi(tB2[m] * dt * SCALE))


def test_superset_reject_contains_the_reference_test():
    rng = np.random.default_rng(11)
    pa, _, _, ra, pb, _, _, rb = pairs(rng, 400_000)
    for scale in (f32(1e-3), f32(1.0), f32(1e3)):   # tiny, reference-sized and huge radii
        a, b = pa * scale, pb * scale
        r1, r2 = ra * scale, rb * scale
        d = a - b
        reff = r1 * f32(0.5) + r2 * f32(0.5)
        exact = reff - length(d) > f32(0.001)
        t = (reff - f32(0.0009)) + reff * f32(1e-5)
        superset = (t > 0) & (dot(d, d) < t * t)
        assert not np.any(exact & ~superset), scale
        assert exact.sum() > 1000 or scale < 1
