import sys
sys.path.insert(0, "/root/repo")
import __graft_entry__ as GE
pkg = GE.load_package()
from sph_test_amd import slab
sim = pkg.SPHSim(slab.weak_scenario("C3", 2), ndev=2, rebalance_every=0, validate=True)
sim.step(int(sys.argv[1]) if len(sys.argv) > 1 else 12)
sim.close()
