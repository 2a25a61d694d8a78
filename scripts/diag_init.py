"""Diagnostic: field-wise GPU vs oracle InitParticles differences."""
import sys
import numpy as np
sys.path.insert(0, ".")
import __graft_entry__ as GE
pkg = GE.load_package(); O = GE.load_oracle()
n = 4096
with pkg.Context(pkg.SPH_MODEL_CONTACT, 3, n) as ctx:
    ctx.init_particles(n, n, 0, 0)
    got = ctx.download_aos84()
ref = O.init_particles(n, n)
for f in ["position", "radius", "mass", "momentOfInertia", "drag", "modeIndex", "rotation"]:
    g, r = got[f], ref[f]
    d = np.abs(g.astype(np.float64) - r.astype(np.float64))
    print(f, "differ:", int((g != r).reshape(n, -1).any(axis=1).sum()), "max abs diff", d.max())
for i in range(1, 4):
    print(i, got["position"][i], ref["position"][i], got["radius"][i], ref["radius"][i])
