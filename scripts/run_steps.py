#!/usr/bin/env python3
"""Plain step driver for rocprofv3 runs: `python scripts/run_steps.py --config C3 --steps 20`.
SPH_NB_VARIANT in the environment selects the neighbour-pass kernels."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    pkg = GE.load_package()
    sim = pkg.SPHSim.from_config(args.config)
    sim.step(args.warmup)
    sim.step(args.steps)
    sim.ctx.synchronize()
    sim.close()


if __name__ == "__main__":
    main()
