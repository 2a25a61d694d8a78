"""Per-workgroup phase times of the one-launch Model R step (k_contact_fused) on the rate table's R = 15 sphere,
N = 4,096: needs the probe build, `bash scripts/build_variant.sh ctprobe -DSPH_CONTACT_PROBE`, loaded through
SPHHIP_LIB (set here). Steps one at a time and reads each launch's wall clocks (100 MHz): permutation build, the
neighbour sums (the workgroup's slowest wave), the barrier, the 16 targets' finish on wave 0, and the launch's span.
    python scripts/contact_probe.py [--steps 20] [--n 4096]"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("SPHHIP_LIB", str(ROOT / "build/variants/lib_ctprobe.so"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))
import __graft_entry__ as GE  # noqa: E402
from contact_scene_stats import sphere  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--n", type=int, default=4096)
a = ap.parse_args()
pkg = GE.load_package()
from importlib import import_module  # noqa: E402
L = import_module(pkg.__name__ + "._abi").lib()
ctl = pkg.ParticleSystemController(particleCount=a.n)
ctl.Start(sphere(pkg, a.n))
ctl.context.step(0.01, 20)
ctl.context.synchronize()
W = 32
buf = (C.c_uint64 * (256 * W))()
acc = []
L_count = []
nwg = min(256, (a.n + 15) // 16)
for s in range(a.steps):
    ctl.context.step(0.01, 1)
    ctl.context.synchronize()
    assert L.sph_debug_contact_probe(buf) == 0
    try:
        L_count.append(ctl.context.mover_count())
    except Exception:  # noqa: BLE001 (the count is informative only)
        pass
    p = np.frombuffer(buf, np.uint64).reshape(256, W)[:nwg].astype(np.int64)
    t0 = p[:, 0].min()
    wv = p[:, 8:24].max(1)
    acc.append([(p[:, 1] - p[:, 0]).mean(), (wv - p[:, 1]).mean(), (p[:, 2] - wv).mean(), (p[:, 3] - p[:, 2]).mean(),
                p[:, 3].max() - t0, (p[:, 0] - t0).max(), (p[:, 8:24] - p[:, 1:2]).mean(),
                (p[:, 4] - p[:, 0]).mean(), (p[:, 5] - p[:, 4]).mean(), (p[:, 6] - p[:, 5]).mean(), (p[:, 1] - p[:, 6]).mean(),
                (p[:, 24] - p[:, 2]).mean(), (p[:, 25] - p[:, 24]).mean(), (p[:, 3] - p[:, 25]).mean()])
m = np.mean(acc, 0) / 100.0   # 100 MHz ticks -> us
print({"n": a.n, "steps": a.steps, "build_us": round(m[0], 2), "sums_slowest_wave_us": round(m[1], 2),
       "sums_mean_wave_us": round(m[6], 2), "barrier_us": round(m[2], 2), "finish_us": round(m[3], 2),
       "span_us": round(m[4], 2), "last_start_us": round(m[5], 2), "build_loads_us": round(m[7], 2),
       "build_sort_us": round(m[8], 2), "build_prefix_dst_us": round(m[9], 2), "build_table_us": round(m[10], 2),
       "finish_math_us": round(m[11], 2), "finish_stores_us": round(m[12], 2), "finish_append_us": round(m[13], 2),
       "movers_mean": round(float(np.mean(L_count)), 1) if L_count else None}, flush=True)
ctl.OnDestroy()
