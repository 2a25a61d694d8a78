"""A C3 run for rocprofv3 kernel traces mid-collapse: `--advance` steps from the lattice
(default 5,000, the bench line's mid-collapse state), then `--steps` traced steps; prints the mover counts of the
traced steps (sph_read_mover_count) so that the re-sort kernels' durations can be read against m.
    rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv -- python3 scripts/mid_trace.py"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--advance", type=int, default=5000)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--sample", type=int, default=10, help="read the mover count every this many traced steps")
a = ap.parse_args()
pkg = GE.load_package()
sim = pkg.SPHSim.from_config(a.config)
done = 0
while done < a.advance:
    k = min(1000, a.advance - done)
    sim.step(k)
    sim.ctx.synchronize()
    done += k
ms = []
for s in range(0, a.steps, a.sample):
    k = min(a.sample, a.steps - s)
    sim.step(k)
    ms.append(sim.ctx.mover_count())
print({"config": a.config, "advance": a.advance, "steps": a.steps, "movers_sampled": ms,
       "movers_mean": round(sum(ms) / len(ms), 1), "resort_limit": max(4096, min(sim.n // 16, 262144))}, flush=True)
sim.close()
