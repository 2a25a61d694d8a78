#!/usr/bin/env python3
"""Plain step driver for rocprofv3 runs: `python scripts/run_steps.py --config C3 --steps 20`.
`--model-r N` steps the
reference controller instead (Model R, N particles from its InitParticles, dt = 1/144); `--sphere N` the rate table's
Model R sphere (R = 15, dt = 0.01, scripts/contact_scene_stats.py)."""
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
    ap.add_argument("--model-r", type=int, default=0)
    ap.add_argument("--sphere", type=int, default=0)
    ap.add_argument("--scenario", default="", help="kind,dim,nx,ny,nz,tx,ty,tz (dx 0.01) instead of --config, e.g. a "
                    "C5/8 rank's cross-section: 0,3,16,256,512,64,512,512")
    args = ap.parse_args()
    pkg = GE.load_package()
    if args.model_r or args.sphere:
        ctl = pkg.ParticleSystemController(particleCount=args.model_r or args.sphere)
        dt = 1 / 144
        if args.sphere:
            sys.path.insert(0, str(ROOT / "scripts"))
            from contact_scene_stats import sphere
            ctl.Start(sphere(pkg, args.sphere))
            dt = 0.01
        else:
            ctl.Start()
        ctl.context.step(dt, args.warmup)
        ctl.context.step(dt, args.steps)
        ctl.context.synchronize()
        ctl.OnDestroy()
        return
    if args.scenario:
        v = [int(t) for t in args.scenario.split(",")]
        sim = pkg.SPHSim(pkg.make_scenario(*v, dx=0.01, seed=1234))
    else:
        sim = pkg.SPHSim.from_config(args.config)
    sim.step(args.warmup)
    sim.step(args.steps)
    sim.ctx.synchronize()
    sim.close()


if __name__ == "__main__":
    main()
