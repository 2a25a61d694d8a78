#!/usr/bin/env python3
"""Long dam-break run (profiling only): per-kernel µs/step in windows of --every steps, as the
column collapses and more particles change sub-cell per step.

    python scripts/long_run.py --config C3 --steps 3000 --every 250
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--every", type=int, default=250)
    args = ap.parse_args()
    pkg = GE.load_package()
    sim = pkg.SPHSim.from_config(args.config, profile=True)
    done = 0
    while done < args.steps:
        k = min(args.every, args.steps - done)
        sim.ctx.reset_kernel_stats()
        t0 = time.perf_counter()
        sim.step(k)
        sim.ctx.synchronize()
        wall = time.perf_counter() - t0
        done += k
        ks = sim.ctx.kernel_stats()
        print(json.dumps({"step": done, "sim_time_s": round(sim.ctx.stats().sim_time, 4),
                          "ms_per_step": round(wall * 1e3 / k, 4),
                          "us_per_step": {n: round(1e3 * v["total_ms"] / k, 1) for n, v in ks.items()
                                          if v["total_ms"] > 0},
                          "launches": {n: v["launches"] for n, v in ks.items() if v["launches"]}}), flush=True)
    sim.close()


if __name__ == "__main__":
    main()
