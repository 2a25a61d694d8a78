"""How many steps bench.py's N > 1 check needs before the re-balancing moves a cut (local groups on one GPU)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE
import bench
pkg = GE.load_package()
for ndev in (2, 4, 8):
    sc = bench.check_scenario(pkg, ndev)
    single = pkg.SPHSim(sc)
    grp = pkg.SPHSim(sc, ndev=ndev, rebalance_every=20)
    done = 0
    for steps in (60, 300, 600, 1000):
        single.step(steps - done)
        grp.step(steps - done)
        done = steps
        dx = float(np.abs(grp.positions() - single.positions()).max())
        print({"ndev": ndev, "steps": steps, "rebalances": grp.ctx.decomposition().rebalances, "max_dx": dx}, flush=True)
    single.close()
    grp.close()
