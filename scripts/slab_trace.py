"""A short run for rocprofv3 kernel traces of the slab step: C3 x N as a local group of N slabs on
one device, serialised on one stream (SPH_DEBUG_SERIAL_GROUP=1), or C3 on one context (N = 1).
    rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 scripts/slab_trace.py N [steps]"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
pkg = GE.load_package()
from sph_test_amd import slab  # noqa: E402
if n > 1:
    os.environ.setdefault("SPH_DEBUG_SERIAL_GROUP", "1")
    sim = pkg.SPHSim(slab.weak_scenario("C3", n), ndev=n, rebalance_every=0)
else:
    sim = pkg.SPHSim.from_config("C3")
sim.step(20)
sim.ctx.synchronize()
t0 = time.perf_counter()
sim.step(steps)
host = time.perf_counter() - t0
sim.ctx.synchronize()
wall = time.perf_counter() - t0
print({"n": n, "steps": steps, "ms_per_step": round(wall * 1e3 / steps, 4), "host_ms_per_step": round(host * 1e3 / steps, 4)},
      flush=True)
sim.close()
