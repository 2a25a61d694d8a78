"""One GPU step of tests/test_gpu_parity_headline.py's splash state, saved for a CPU analysis of pass 2's margin
(scripts/pass2_margin.py): the input (x0, v0) and the GPU's x, v, ρ, P/ρ² in particle order.
    python scripts/splash_dump.py --out gpurun_out/splash_gpu.npz"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as GE  # noqa: E402
from conftest import oracle_sph_params  # noqa: E402
from sph_states import splash_state  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/splash_gpu.npz")
a = ap.parse_args()
pkg = GE.load_package()
O = GE.load_oracle()
sc = pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 32, 64, 128, 128, 128, 128, dx=0.01)
p, dt = pkg.scenario_params(sc)
sim = pkg.SPHSim(sc, capacity=300_000)
try:
    cell = float(np.float32(2.0) * np.float32(p.h))
    op = oracle_sph_params(O, sim.params, 3)   # the grid's column count, as the test takes it
    x0, v0 = splash_state(int(op.grid.G[0]), 0, 0, cell, 8000, 60, tuple(p.box))
    x0 = np.minimum(x0, np.array(p.box, np.float32))
    sim.ctx.upload_state(x0, v0)
    sim.step(1)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(a.out, x0=x0, v0=v0, x=sim.positions(), v=sim.velocities(), rho=sim.density(),
                        prho=sim.ctx.pressure_term(), dt=np.float32(sim.dt))
    print({"n": len(x0), "out": a.out})
finally:
    sim.close()
