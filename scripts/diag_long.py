"""Locate a fault of the in-library decomposed step (SPH_FLAG_VALIDATE checkpoints name the phase).
   python scripts/diag_long.py NDEV REBALANCE_EVERY STEPS [SINGLE_FROM]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import __graft_entry__ as GE
pkg = GE.load_package()
sc = pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99)
sim = pkg.SPHSim(sc, ndev=int(sys.argv[1]), rebalance_every=int(sys.argv[2]), validate=True)
total = int(sys.argv[3])
single_from = int(sys.argv[4]) if len(sys.argv) > 4 else total
done = 0
while done < total:
    k = 10 if done + 10 <= single_from else 1
    try:
        sim.step(k)
    except Exception as e:
        print("step", done + k, "FAILED", e, flush=True)
        sys.exit(3)
    done += k
    if k == 10:
        d = sim.ctx.decomposition()
        print("step", done, "cut", d.cut.cx_lo, d.cut.cx_hi, "owned", d.owned, "rebal", d.rebalances, flush=True)
    else:
        print("step", done, "ok", flush=True)
