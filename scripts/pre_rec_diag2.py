"""Diagnostic: a 2-slab group stepped 8 steps in one sph_step call (the host runs ahead), against one context."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import __graft_entry__ as GE  # noqa: E402

pkg = GE.load_package()
from test_gpu_slab import _scenario  # noqa: E402
sc = _scenario(pkg, 0)
sim = pkg.SPHSim(sc, ndev=2, rebalance_every=0)
try:
    sim.step(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
    print("ok", flush=True)
except Exception as e:  # noqa: BLE001
    print("FAILED", e, flush=True)
sim.close()
