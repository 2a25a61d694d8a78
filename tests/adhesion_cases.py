"""Seeded adhesion scenes shared by the CPU and GPU adhesion tests and tests/golden/make_golden.py.

A random sphere of particles (SURVEY.md §8c recipe: positions in R=15, radii U[1.5,2],
v, ω ~ N(0,1)) with random unit rotations, bonded to near neighbours the way
CellAdhesionManager builds bonds (CellAdhesionManager.cs:524-564): genome-default spring
(restLength, springStiffness, springDamping), anchorConstraintStiffness =
orientationConstraintStrength × 10, anchors on the particle surfaces, and the relative
orientation of the pair at bond creation.
"""
from __future__ import annotations

import numpy as np


def _qmul(a, b):
    av, aw = a[..., :3], a[..., 3:]
    bv, bw = b[..., :3], b[..., 3:]
    v = aw * bv + bw * av + np.cross(av, bv)
    w = aw * bw - np.sum(av * bv, axis=-1, keepdims=True)
    return np.concatenate([v, w], axis=-1)


def _qconj(q):
    return q * np.array([-1, -1, -1, 1], q.dtype)


def bonded_sphere(PARTICLE84, ADHESION84, n, seed=1234, R=15.0, bonds_per=2, enable_frac=0.5):
    rng = np.random.default_rng(seed)
    p = np.zeros(n, PARTICLE84)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    p["position"] = d * (R * rng.random((n, 1)) ** (1 / 3))
    p["radius"] = rng.uniform(1.5, 2.0, n)
    p["velocity"] = rng.normal(size=(n, 3))
    p["mass"] = 0.1 * 4.0 / 3.0 * 3.1415926 * p["radius"] ** 3
    p["angularVelocity"] = rng.normal(size=(n, 3))
    p["momentOfInertia"] = 0.4 * p["mass"] * p["radius"] ** 2
    p["drag"] = rng.uniform(0.5, 1.0, n)
    p["repulsionStrength"] = 1.0
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    p["rotation"] = q.astype(np.float32)
    p["modeIndex"] = -1
    # bonds: each particle to its `bonds_per` nearest others (brute force; n is small)
    x = p["position"].astype(np.float64)
    pairs = set()
    for i in range(n):
        dist = np.linalg.norm(x - x[i], axis=1)
        dist[i] = np.inf
        for j in np.argsort(dist)[:bonds_per]:
            pairs.add((min(i, int(j)), max(i, int(j))))
    pairs = sorted(pairs)
    order = rng.permutation(len(pairs))            # bond list order is arbitrary (hash-set order)
    A = np.array([pairs[k][0] for k in order], np.int32)
    B = np.array([pairs[k][1] for k in order], np.int32)
    swap = rng.random(len(A)) < 0.5                # either end may be particleA
    A, B = np.where(swap, B, A), np.where(swap, A, B)
    m = len(A)
    c = np.zeros(m, ADHESION84)
    c["particleA"], c["particleB"] = A, B
    c["restLength"] = rng.uniform(2.0, 3.0, m)
    c["springStiffness"] = rng.uniform(50.0, 150.0, m)
    c["springDamping"] = rng.uniform(1.0, 8.0, m)
    c["connectionColor"] = (1, 1, 1, 1)
    qa = p["rotation"][A].astype(np.float64)
    qb = p["rotation"][B].astype(np.float64)
    rel = _qmul(_qconj(qa), qb)
    # perturb the rest orientation so the correction is non-trivial
    dq = np.concatenate([rng.normal(scale=0.2, size=(m, 3)), np.ones((m, 1))], axis=1)
    dq /= np.linalg.norm(dq, axis=1, keepdims=True)
    c["initialRelOrientation"] = _qmul(dq, rel).astype(np.float32)
    ua = rng.normal(size=(m, 3))
    ub = rng.normal(size=(m, 3))
    c["anchorLocalPosA"] = ua / np.linalg.norm(ua, axis=1, keepdims=True) * p["radius"][A, None]
    c["anchorLocalPosB"] = ub / np.linalg.norm(ub, axis=1, keepdims=True) * p["radius"][B, None]
    c["anchorConstraintStiffness"] = rng.uniform(0.0, 1.0, m) * 10.0
    c["enableAnchorConstraint"] = (rng.random(m) < enable_frac).astype(np.int32)
    return p, c
