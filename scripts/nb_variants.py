#!/usr/bin/env python3
"""A/B the neighbour-pass variants in one process (cdna_hip_programming.md §5.4 rule 24).

For each variant (SPH_NB_VARIANT, read at context creation) it runs the same config from the
same initial state, checks the first step against variant 0, and prints the per-kernel
HIP-event times for interleaved rounds.
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    pkg = GE.load_package()
    variants = [int(v) for v in args.variants.split(",")]
    sims = {}
    for v in variants:
        os.environ["SPH_NB_VARIANT"] = str(v)
        sims[v] = pkg.SPHSim.from_config(args.config, profile=True)
    # parity of one step across variants
    first = {}
    for v, s in sims.items():
        s.step(1)
        first[v] = (s.positions(), s.velocities(), s.density())
    ref = first[variants[0]]
    for v in variants[1:]:
        got = first[v]
        print(json.dumps({"variant": v, "bitwise_pos": bool(np.array_equal(got[0], ref[0])),
                          "bitwise_rho": bool(np.array_equal(got[2], ref[2])),
                          "max_dpos": float(np.abs(got[0] - ref[0]).max()),
                          "max_drho_rel": float((np.abs(got[2] - ref[2]) / ref[2]).max()),
                          "max_dvel": float(np.abs(got[1] - ref[1]).max())}), flush=True)
    for r in range(args.rounds):
        for v, s in sims.items():
            s.ctx.reset_kernel_stats()
            s.step(args.steps)
            s.ctx.synchronize()
            ks = s.ctx.kernel_stats()
            print(json.dumps({"round": r, "variant": v,
                              "us_per_step": {k: round(1e3 * x["total_ms"] / args.steps, 1) for k, x in ks.items()}}),
                  flush=True)
    for s in sims.values():
        s.close()


if __name__ == "__main__":
    main()
