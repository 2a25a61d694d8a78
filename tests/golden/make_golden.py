#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz from the CPU oracle (test infrastructure).

The reference ships no golden vectors, so these fixtures pin the oracle's own
outputs. They catch regressions in the restatement. They are NOT reference outputs: the
reference's HLSL cannot run here. Inputs follow SURVEY.md §8c's fixture recipe.
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import oracle as O  # noqa: E402


def sphere_particles(n, seed=1234, R=15.0):
    rng = np.random.default_rng(seed)
    p = np.zeros(n, O.PARTICLE84)
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
    p["rotation"] = (0, 0, 0, 1)
    p["modeIndex"] = -1
    return p


def contact_case(n, steps, dt=0.01):
    parts = sphere_particles(n)
    cp = O.contact_params(dt, global_drag=10.0)          # scene value (Particle Simulation.unity:155)
    cur, tq = parts, None
    for _ in range(steps):
        cur, tq = O.contact_step(cp, cur, nthreads=1)
    return parts, cur, tq


def sph_case(steps):
    dx = 0.01
    h = 1.2 * dx
    c0 = float(np.float32(10 * np.sqrt(2 * 9.81 * 64 * dx)))
    op = O.sph_params(2, dx, h, 1000.0, c0, 0.02, 0.5, (0, -9.81, 0), (256 * dx, 128 * dx, 0), 0.5)
    x = O.lattice(2, 64, 64, 1, dx, seed=1234)
    v = np.zeros_like(x)
    ids = np.arange(len(x), dtype=np.int32)
    dt = float(np.float32(0.25 * h / c0))
    x0 = x.copy()
    for s in range(steps):
        x, v, ids, rho, _, _ = O.sph_step(op, x, v, ids, dt, float(np.float32(s * dt)), nthreads=1)
    o = np.argsort(ids)
    return x0, x[o], v[o], rho[o], dt, c0


def adhesion_case(n, steps, dt=0.01):
    """A bonded sphere (tests/adhesion_cases.py) stepped with its bonds (compute:424-607)."""
    sys.path.insert(0, str(HERE.parent))
    from adhesion_cases import bonded_sphere
    parts, conns = bonded_sphere(O.PARTICLE84, O.ADHESION84, n, seed=21)
    cp = O.contact_params(dt, global_drag=10.0)
    cur, tq, terms = parts, None, None
    for _ in range(steps):
        cur, tq, terms = O.contact_step_bonds(cp, cur, conns, nthreads=1)
    return parts, conns, cur, tq, terms


def main():
    for n, steps in [(64, 1), (64, 10), (4096, 1)]:
        inp, out, tq = contact_case(n, steps)
        np.savez_compressed(HERE / f"contact_n{n}_s{steps}.npz", input=inp.view(np.uint8), output=out.view(np.uint8),
                            torque=tq)
    for n, steps in [(512, 1), (512, 5)]:
        inp, conns, out, tq, terms = adhesion_case(n, steps)
        np.savez_compressed(HERE / f"adhesion_n{n}_s{steps}.npz", input=inp.view(np.uint8),
                            conns=conns.view(np.uint8), output=out.view(np.uint8), torque=tq, terms=terms)
    for steps in [1, 10]:
        x0, x, v, rho, dt, c0 = sph_case(steps)
        np.savez_compressed(HERE / f"wcsph_c1_s{steps}.npz", x0=x0, x=x, v=v, rho=rho, dt=dt, c0=c0)


if __name__ == "__main__":
    main()
