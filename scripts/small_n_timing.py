"""Host and wall time per step at the reference's own scale (DESIGN.md §5 rate table rows): Model R at N = 4,096
(the rate table's sphere) and Model S C1 (4,096 particles, 2D). Host = time to issue `steps` steps (sph_step returns
before the GPU finishes), wall = until the stream drains.
    python scripts/small_n_timing.py [steps]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
pkg = GE.load_package()


def sphere(n):
    rng = np.random.default_rng(1234)
    parts = np.zeros(n, pkg.PARTICLE84)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    parts["position"] = d * (15.0 * rng.random((n, 1)) ** (1 / 3))
    parts["radius"] = rng.uniform(1.5, 2.0, n)
    parts["velocity"] = rng.normal(size=(n, 3))
    parts["mass"] = 0.1 * 4.0 / 3.0 * 3.1415926 * parts["radius"] ** 3
    parts["angularVelocity"] = rng.normal(size=(n, 3))
    parts["momentOfInertia"] = 0.4 * parts["mass"] * parts["radius"] ** 2
    parts["drag"] = rng.uniform(0.5, 1.0, n)
    parts["repulsionStrength"] = 1.0
    parts["rotation"] = (0, 0, 0, 1)
    parts["modeIndex"] = -1
    return parts


def timed(step, sync, n, label):
    step(20)
    sync()
    t0 = time.perf_counter()
    step(steps)
    host = time.perf_counter() - t0
    sync()
    wall = time.perf_counter() - t0
    print({"case": label, "particles": n, "steps": steps, "us_per_step": round(wall * 1e6 / steps, 2),
           "host_us_per_step": round(host * 1e6 / steps, 2), "particle_steps_per_s": round(n * steps / wall)}, flush=True)


import os  # noqa: E402
for n in (4096, 32768):
    for team in ("", "65"):   # the default lanes per target, and the flat form (contact.hip CT_FLAT)
        if team:
            os.environ["SPH_CT_TEAM"] = team
        ctl = pkg.ParticleSystemController(particleCount=n)
        ctl.Start(sphere(n))
        timed(lambda k: ctl.context.step(0.01, k), ctl.context.synchronize, n, f"R sphere N={n} team {team or 'default'}")
        ctl.OnDestroy()
        os.environ.pop("SPH_CT_TEAM", None)
for cfg in ("C1",):
    sim = pkg.SPHSim.from_config(cfg)
    timed(sim.step, sim.ctx.synchronize, sim.n, f"S {cfg}")
    sim.close()
