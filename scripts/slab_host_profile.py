#!/usr/bin/env python3
"""Host-side time per phase of the slab step at N=1 (profiling only): where the host waits
(sync points) and how long each ABI call takes to return.

    python scripts/slab_host_profile.py --steps 200
"""
import argparse
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import __graft_entry__ as GE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--config", default="C3")
    args = ap.parse_args()
    import torch
    GE.load_package()
    from sph_test_amd import slab
    torch.cuda.set_device(0)
    runner = slab.SlabRunner(args.config, 0, 1, device=0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    runner.bind_stream(stream.cuda_stream)
    runner.step(20)
    torch.cuda.synchronize()
    acc = defaultdict(float)
    be = runner.be
    for name in ("count_sends_into", "send_capacity", "pack_send", "assemble", "density", "ranges", "pack_rho",
                 "unpack_rho", "force", "finish"):
        fn = getattr(be, name)

        def wrap(*a, _fn=fn, _n=name, **k):
            t0 = time.perf_counter()
            r = _fn(*a, **k)
            acc[_n] += time.perf_counter() - t0
            return r
        setattr(be, name, wrap)
    t0 = time.perf_counter()
    runner.step(args.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = {k: round(v * 1e6 / args.steps, 1) for k, v in acc.items()}
    out["other_python"] = round(wall * 1e6 / args.steps - sum(out.values()), 1)
    print(json.dumps({"us_per_step_host": out, "wall_us_per_step": round(wall * 1e6 / args.steps, 1)}))
    runner.close()


if __name__ == "__main__":
    main()
