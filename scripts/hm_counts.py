"""Hit-mask coverage: force wave-planes scanned by distance (mask budget passed or sparse path) per
wave-plane, at C3 from rest and mid-collapse."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE
pkg = GE.load_package()
sim = pkg.SPHSim.from_config("C3")
sim.step(20)
sim.ctx.hit_mask_counts(reset=True)
for label, adv in (("rest", 0), ("mid-collapse", 5000)):
    sim.step(adv)
    sim.ctx.hit_mask_counts(reset=True)
    sim.step(20)
    d, w = (int(x) for x in sim.ctx.hit_mask_counts(reset=True))
    print({"state": label, "distance_wave_planes": d, "wave_planes": 3 * w, "fraction": d / max(1, 3 * w)}, flush=True)
sim.close()
