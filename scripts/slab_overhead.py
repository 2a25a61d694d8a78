"""The decomposition's cost on one GPU: C3 x N (bench.py's weak scenario) as one context against a local group of N
slab contexts on the same device (sph_config.ndev = N; the halo copies are then device-local). Both do the same
particle work; the difference is what the slab step adds (counts, packing, the halo records' re-sort, ρ halo,
boundary force passes, bookkeeping) and the serialisation of N slabs' launches on one GPU."""
import sys
import time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE
pkg = GE.load_package()
from sph_test_amd import slab
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
for world in [int(w) for w in (sys.argv[1] if len(sys.argv) > 1 else "2").split(",")]:
    sc = slab.weak_scenario("C3", world)
    res = {"world": world, "particles": sc.nx * sc.ny * sc.nz}
    for label, kw in (("single", {}), ("group", {"ndev": world, "rebalance_every": 50})):
        sim = pkg.SPHSim(sc, **kw)
        sim.step(20)
        sim.ctx.synchronize()
        t0 = time.perf_counter()
        sim.step(steps)
        sim.ctx.synchronize()
        res[label + "_ms"] = round((time.perf_counter() - t0) * 1e3 / steps, 4)
        sim.close()
    res["overhead_ms"] = round(res["group_ms"] - res["single_ms"], 4)
    res["overhead_per_slab_ms"] = round(res["overhead_ms"] / world, 4)
    print(res, flush=True)
