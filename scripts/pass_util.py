"""Lane utilisation of the two neighbour passes at C3, from rest and mid-collapse. Needs a -DSPH_DIAG
library (SPHHIP_LIB=build/variants/lib_diag.so): sph_debug_pass_counts reads the counters that build adds."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE

pkg = GE.load_package()
sim = pkg.SPHSim.from_config("C3")
ctx = sim.ctx


def read(reset=True):
    out = np.zeros(8, np.uint32)
    st = ctx._L.sph_debug_pass_counts(ctx._h, out.ctypes.data_as(C.c_void_p), 1 if reset else 0)
    assert st == 0, st
    return out.astype(np.float64)


sim.step(20)
read()
for label, adv in (("rest", 0), ("mid-collapse", 5000)):
    sim.step(adv)
    read()
    sim.step(10)
    c = read()
    cand, it4, it1, pairs, fit, nfl, ait, pieces = c
    waves = nfl / max(1.0, nfl) * 1.0
    print({
        "state": label,
        "pass1_candidates_per_target": cand / (10 * sim.n),
        "pass1_lane_util_group_iters": cand / (64 * (4 * it4 + it1)),
        "pass1_tail_share_of_iters": it1 / (it4 + it1),
        "pass2_pairs_per_target": pairs / (10 * sim.n),
        "pass2_flush_lane_util": pairs / (64 * fit),
        "pass2_flushes_per_wave": nfl / (10 * sim.n / 64),
        "pass2_append_iters_per_wave": ait / (10 * sim.n / 64),
        "pass2_append_iters_per_pair_lane": ait * 64 / max(1.0, pairs),
        "pass2_pieces_per_wave": pieces / (10 * sim.n / 64),
    }, flush=True)
sim.close()
