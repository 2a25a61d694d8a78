"""Child process of tests/test_gpu_path_independence.py (run once per library build, SPHHIP_LIB selects it):
steps a Model S scenario and writes, as JSON, a sha1 of the positions and velocities after every step and the
sparse-path counters summed over the run (sph_read_path_counts: density chunked, density global, force
chunked, force global), the hit-mask counters (wave-planes scanned by distance, waves) and the incremental
re-sort's counters (sph_read_resort_counts: whole-list ranges, whole-list lanes, multi-pass ranges, passes,
largest range, cell shares that re-streamed). `violent`: tests/test_gpu_resort.py's many-movers state (random velocities of up to a z
sub-cell per step), where most ranges take the re-sort's multi-pass path in the small-cap variant library.

  python tests/hash_run.py OUT.json STEPS {slab|violent|C1|C2|C3}
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402


def main() -> None:
    out, steps, cfg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    pkg = GE.load_package()
    if cfg == "slab":   # tests/test_gpu_slab.py's dam-break: a 48 x 32 x 32 lattice column in a 120 x 48 x 32 tank
        sim = pkg.SPHSim(pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99))
    elif cfg == "violent":
        sim = pkg.SPHSim(pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24, 20, 16, 40, 40, 40, dx=0.01, seed=5))
        rng = np.random.default_rng(11)
        x = sim.positions()
        sub = 2 * sim.params.h / 6                  # z sub-cell (SPEC_SPH.md §0)
        sim.ctx.upload_state(x, rng.uniform(-1.0, 1.0, x.shape).astype(np.float32) * (sub / sim.dt))
    else:
        sim = pkg.SPHSim.from_config(cfg)
    try:
        sim.ctx.path_counts(reset=True)          # arm the counters
        sim.ctx.hit_mask_counts(reset=True)
        paths = np.zeros(4, np.int64)
        hm = np.zeros(2, np.int64)
        sim.ctx.resort_counts(reset=True)
        rs = np.zeros(6, np.int64)
        hs = []
        for _ in range(steps):
            sim.step(1)
            paths += sim.ctx.path_counts(reset=True).astype(np.int64)
            hm += sim.ctx.hit_mask_counts(reset=True).astype(np.int64)
            c = sim.ctx.resort_counts(reset=True).astype(np.int64)
            rs[:4] += c[:4]
            rs[4] = max(rs[4], c[4])
            rs[5] += c[5]
            x, v = sim.positions(), sim.velocities()
            hs.append(hashlib.sha1(x.tobytes() + v.tobytes()).hexdigest()[:16])
        lib = str(pkg._abi.lib_path()) if hasattr(pkg, "_abi") else ""
    finally:
        sim.close()
    with open(out, "w") as f:
        json.dump({"hashes": hs, "paths": paths.tolist(), "hit_mask": hm.tolist(), "resort": rs.tolist(), "lib": lib}, f)
    print(out, cfg, steps, hs[-1], paths.tolist(), hm.tolist(), rs.tolist(), flush=True)


if __name__ == "__main__":
    main()
