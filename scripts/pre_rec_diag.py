"""Diagnostic: a 2-slab group stepped one step at a time, printing each step's outcome (validation off / on)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import __graft_entry__ as GE  # noqa: E402

pkg = GE.load_package()
from test_gpu_slab import _scenario  # noqa: E402
sc = _scenario(pkg, 0)
sim = pkg.SPHSim(sc, ndev=2, rebalance_every=0, validate=bool(int(sys.argv[1])) if len(sys.argv) > 1 else False)
for k in range(8):
    try:
        sim.step(1)
        print("step", k, "ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print("step", k, "FAILED", e, flush=True)
        break
sim.close()
