import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as GE
pkg = GE.load_package()
sc = pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99)
sim = pkg.SPHSim(sc, ndev=int(sys.argv[1]), rebalance_every=int(sys.argv[2]), validate=True)
for k in range(int(sys.argv[3]) // 10):
    try:
        sim.step(10)
    except Exception as e:
        print("step", (k + 1) * 10, "FAILED", e, flush=True)
        break
    d = sim.ctx.decomposition()
    print("step", (k + 1) * 10, "cut", d.cut.cx_lo, d.cut.cx_hi, "owned", d.owned, "rebal", d.rebalances, flush=True)
