"""Per-step sha1 of the positions and velocities of a single-context run (tests/test_gpu_slab.py's dam-break
scenario, or a BASELINE config), for bit-identity checks between two library builds:
  SPHHIP_LIB=build/variants/lib_a.so python scripts/step_hashes.py out_a.json [steps] [config]
With a save step, the state at that step is written next to the json as .npz."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402

pkg = GE.load_package()
out = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
cfg = sys.argv[3] if len(sys.argv) > 3 else "slab"
save = int(sys.argv[4]) if len(sys.argv) > 4 else -1
if cfg == "slab":
    sim = pkg.SPHSim(pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99))
else:
    sim = pkg.SPHSim.from_config(cfg)
hs = []
for k in range(1, steps + 1):
    sim.step(1)
    x, v = sim.positions(), sim.velocities()
    hs.append(hashlib.sha1(x.tobytes() + v.tobytes()).hexdigest()[:16])
    if k == save:
        np.savez(out.replace(".json", f"_{k}.npz"), x=x, v=v, rho=sim.densities() if hasattr(sim, "densities") else x[:, 0])
sim.close()
json.dump(hs, open(out, "w"))
print(out, len(hs), hs[-1])
