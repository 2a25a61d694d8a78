import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np
import __graft_entry__ as GE
pkg = GE.load_package(); O = GE.load_oracle()
from test_gpu_parity import random_sphere
for n in (4096, 32768, 262144):
    parts = random_sphere(pkg.PARTICLE84, n)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts.copy())
    t0 = time.time(); ctl.Update(0.01); got = ctl.GetParticles(); tg = time.time() - t0
    t0 = time.time(); ref, tq = O.contact_step(O.contact_params(0.01), parts.view(O.PARTICLE84), nthreads=16); tc = time.time() - t0
    out = {"n": n, "gpu_s": round(tg, 3), "cpu_s": round(tc, 1)}
    for f in ("velocity", "angularVelocity", "position", "rotation"):
        a, b = got[f].astype(np.float64), ref[f].astype(np.float64)
        rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-3)
        out[f] = [float(np.quantile(rel, 0.5)), float(np.quantile(rel, 0.999)), float(rel.max()), float((rel > 1e-5).mean())]
    d = np.abs(ctl.context.torque_int().astype(np.int64) - tq)
    out["torque_lsb"] = [int(d.max()), float((d > 0).mean())]
    print(out, flush=True)
    ctl.OnDestroy()
