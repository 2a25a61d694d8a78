"""Workgroup timeline of the two neighbour passes at C3 (a -DSPH_BTIME library: SPHHIP_LIB=build/variants/
lib_bt.so): kernel span, the span if the summed workgroup time filled every resident slot, and the tail, from
rest and mid-collapse."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE

BT_MAX = 16384
SLOTS = {"density": 7 * 256, "force": 4 * 256}   # resident workgroups (per CU x 256 CUs)

pkg = GE.load_package()
sim = pkg.SPHSim.from_config("C3")
L = sim.ctx._L
nb = (sim.n + 255) // 256


def report(label):
    buf = np.zeros(2 * BT_MAX * 2, np.uint64)
    assert L.sph_debug_block_times(buf.ctypes.data_as(C.c_void_p), len(buf)) == 0
    t = buf.reshape(2, BT_MAX, 2)[:, :nb, :].astype(np.float64) * 10.0 / 1e3   # 100 MHz ticks -> us
    np.save(Path(__file__).resolve().parent.parent / "gpurun_out" / f"block_times_{label}.npy", t)
    for k, name in enumerate(("density", "force")):
        st, en = t[k, :, 0], t[k, :, 1]
        t0 = st.min()
        span = en.max() - t0
        dur = en - st
        ideal = dur.sum() / SLOTS[name]
        # resident workgroups over time: the tail is the time after the count first drops below 90% of slots
        # for good (after the last start)
        last_start = st.max() - t0
        order = np.argsort(dur)[::-1]
        print({"state": label, "pass": name, "span_us": round(span, 1), "filled_us": round(ideal, 1),
               "tail_us_after_last_start": round(span - last_start, 1),
               "block_us_mean": round(dur.mean(), 1), "block_us_p50": round(float(np.median(dur)), 1),
               "block_us_p99": round(float(np.percentile(dur, 99)), 1), "block_us_max": round(dur.max(), 1),
               "slowest_blocks": [int(x) for x in order[:5]]}, flush=True)


sim.step(20)
report("rest")
sim.step(5000)
report("mid-collapse")
sim.close()
