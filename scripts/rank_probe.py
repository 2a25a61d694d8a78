"""Per-workgroup timing of the re-sort's rank kernel mid-collapse: needs the probe build,
`bash scripts/build_variant.sh probe -DSPH_RANK_PROBE`, loaded through SPHHIP_LIB (set here). Advances C3 to the
bench line's mid-collapse state, then steps one at a time and reads each launch's per-workgroup wall clocks
(100 MHz) and entry counts: the kernel's time is its slowest workgroup's, so this shows which ranges set it.
    python scripts/rank_probe.py [--advance 5000] [--steps 10]"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("SPHHIP_LIB", str(ROOT / "build/variants/lib_probe.so"))
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--advance", type=int, default=5000)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--slab", type=int, default=0,
                help="C3 x N as a serialised local group of N slabs; the probe holds the last re-sort launched")
a = ap.parse_args()
pkg = GE.load_package()
from importlib import import_module  # noqa: E402
abi = import_module(pkg.__name__ + "._abi")
L = abi.lib()
if a.slab > 1:
    from sph_test_amd import slab  # noqa: E402
    os.environ.setdefault("SPH_DEBUG_SERIAL_GROUP", "1")
    sim = pkg.SPHSim(slab.weak_scenario(a.config, a.slab), ndev=a.slab, rebalance_every=0)
else:
    sim = pkg.SPHSim.from_config(a.config)
done = 0
while done < a.advance:
    k = min(1000, a.advance - done)
    sim.step(k)
    sim.ctx.synchronize()
    done += k
buf = (C.c_uint64 * (256 * 8))()
for s in range(a.steps):
    sim.step(1)
    sim.ctx.synchronize()
    assert L.sph_debug_rank_probe(buf) == 0
    p = np.frombuffer(buf, np.uint64).reshape(256, 8).astype(np.int64)
    live = p[:, 3] > 0
    t0 = p[live, 0].min()
    tot = (p[live, 3] - p[live, 0]) / 100.0
    stream = (p[live, 1] - p[live, 0]) / 100.0
    sort = (p[live, 2] - p[live, 1]) / 100.0
    tail = (p[live, 3] - p[live, 2]) / 100.0
    span = (p[live, 3].max() - t0) / 100.0
    start_spread = (p[live, 0].max() - t0) / 100.0
    worst = np.argsort(-tot)[:4]
    print({"step": s, "m": int(p[live, 6][0]), "span_us": span, "start_spread_us": start_spread,
           "wg_us_median": float(np.median(tot)), "wg_us_max": float(tot.max()),
           "stream_med": float(np.median(stream)), "sort_med": float(np.median(sort)), "tail_med": float(np.median(tail)),
           "nd_max": int(p[live, 4].max()), "ns_max": int(p[live, 5].max()), "bitmap_all": bool(p[live, 7].all()),
           "worst": [{"us": float(tot[w]), "stream": float(stream[w]), "sort": float(sort[w]), "tail": float(tail[w]),
                      "nd": int(p[live, 4][w]), "ns": int(p[live, 5][w])} for w in worst]}, flush=True)
sim.close()
