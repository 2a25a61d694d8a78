"""Diagnostic: the in-library group (ndev) against the single context, with different host pacing."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as GE
pkg = GE.load_package()
sc = pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99)
ndev = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = 8
single = pkg.SPHSim(sc)
single.step(steps)
xs = single.positions()
p = pkg.scenario_params(sc)[0]
cell = np.float32(2) * np.float32(p.h)
import os
for mode in sys.argv[2].split(","):
    grp = pkg.SPHSim(sc, ndev=ndev, rebalance_every=0)
    if mode == "all":
        grp.step(steps)
    else:
        for s in range(steps):
            grp.step(1)
            if mode == "sync":
                grp.ctx.synchronize()
            elif mode == "decomp":
                grp.ctx.decomposition()
            else:
                grp.positions()
    xg = grp.positions()
    bad = np.abs(xs - xg).max(axis=1) > 2e-6
    col = np.floor(xs[:, 0] / cell).astype(int)
    print(mode, "bad", int(bad.sum()), "cols", np.unique(col[bad]).tolist()[:20], "max", float(np.abs(xs - xg).max()),
          "cuts", grp.ctx.decomposition().cut.cx_lo, flush=True)
    grp.close()
