"""Sparse-path mix of the neighbour passes at C3 from rest and mid-collapse: planes processed row by row in
chunks and rows gathered from global memory (sph_read_path_counts), per block-plane."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import __graft_entry__ as GE
pkg = GE.load_package()
sim = pkg.SPHSim.from_config("C3")
sim.step(20)
sim.ctx.path_counts(reset=True)
blocks = (sim.n + 255) // 256
for label, adv in (("rest", 0), ("mid-collapse", 5000)):
    sim.step(adv)
    sim.ctx.path_counts(reset=True)
    sim.step(10)
    c = [int(x) for x in sim.ctx.path_counts(reset=True)]
    print({"state": label, "density_chunked_planes": c[0], "density_gathered_rows": c[1],
           "force_chunked_planes": c[2], "force_gathered_rows": c[3],
           "block_planes": 10 * 3 * blocks,
           "force_chunked_fraction": c[2] / (10 * 3 * blocks)}, flush=True)
sim.close()
