"""No result may depend on the block partition or the LDS plane budget.

A workgroup's targets, and the intervals its planes stage, depend on where the blocks fall (block size,
the slab decomposition's cuts, the incremental re-sort's slot order). Which path a plane takes then
depends on its intervals against the LDS budget: staged whole, chunked row by row, or gathered straight
from global memory. Every path must find the same neighbours (q ≤ 2, rounded alike) and add them in the
same order, or the single-context and decomposed runs drift apart bit by bit. The neighbour distance, the
pair body's r² and v·r and the row-window radius are explicit fmaf chains for this (wcsph_tiled.hip
dist2/pair_force, common.h row_window): left to the compiler's contraction they rounded one way in the LDS
scans and another in the global-gather path.

The product library runs against libsphhip_smallplanes.so, the same sources with 64-candidate plane budgets
(rows past 256 candidates from global memory), 128-target force workgroups and 32-entry re-sort ranges
(csrc/Makefile `variants`): the per-step sha1 of positions and velocities must be equal at every step, and
the variant's counters must show that its planes really took the chunked and global-gather paths. The
violent state (most particles change sub-cell every step) runs both libraries on the incremental re-sort
(SPH_RESORT=2) against the product's full sort (SPH_RESORT=0), so the variant's ranges take the re-sort's
multi-pass path (resort.hip: dest entries beyond LDS, staged per key sub-interval) and its cell shares the
path for keys beyond LDS (a stream per pass); C3 gives the variant's shares several passes of 1,024 cells.
All must still give the full sort's permutation and cell starts. The analogue in the reference is its
contact test `SimulateParticles.compute:249-253`, evaluated the same way for every candidate.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
SMALL = ROOT / "sph-test_amd" / "libsphhip_smallplanes.so"


def _run(tmp_path, lib, steps, cfg, tag, resort=None):
    out = tmp_path / f"{tag}_{cfg}.json"
    env = dict(os.environ)
    if resort is not None:
        env["SPH_RESORT"] = resort
    if lib is not None:
        env["SPHHIP_LIB"] = str(lib)
    else:
        env.pop("SPHHIP_LIB", None)
    subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "hash_run.py"), str(out), str(steps), cfg],
                   env=env, check=True, timeout=240)
    return json.loads(out.read_text())


@pytest.mark.parametrize("cfg,steps", [("slab", 300), ("C3", 30)])
def test_block_partition_and_plane_budget_do_not_change_results(tmp_path, cfg, steps):
    assert SMALL.exists(), f"{SMALL} not built: run __graft_entry__.build()"
    prod = _run(tmp_path, None, steps, cfg, "product")
    small = _run(tmp_path, SMALL, steps, cfg, "small")
    print({"cfg": cfg, "product_paths": prod["paths"], "small_paths": small["paths"],
           "product_hit_mask": prod["hit_mask"], "small_hit_mask": small["hit_mask"]})
    dc, dg, fc, fg = small["paths"]
    assert dc > 0 and fc > 0, small["paths"]              # planes chunked in both passes
    if cfg == "slab":
        assert dg > 0 and fg > 0, small["paths"]          # rows gathered from global memory in both passes
    first = next((k for k, (a, b) in enumerate(zip(prod["hashes"], small["hashes"])) if a != b), None)
    assert first is None, f"{cfg}: states differ from step {first + 1} on"


def test_resort_multi_pass_matches_the_full_sort(tmp_path):
    assert SMALL.exists(), f"{SMALL} not built: run __graft_entry__.build()"
    full = _run(tmp_path, None, 12, "violent", "full", resort="0")
    prod = _run(tmp_path, None, 12, "violent", "product", resort="2")
    small = _run(tmp_path, SMALL, 12, "violent", "small", resort="2")
    print({"product_resort": prod["resort"], "small_resort": small["resort"]})
    whole, whole_lanes, multi, passes, _, restream = small["resort"]
    assert multi > 0 and passes > multi, small["resort"]     # ranges ran in several passes
    assert restream > 0, small["resort"]                     # cell shares whose keys overflowed LDS
    assert whole == 0 and whole_lanes == 0, small["resort"]  # and none counted against the whole list
    assert prod["resort"][0] == 0 and prod["resort"][1] == 0, prod["resort"]
    for name, run in (("product", prod), ("small", small)):
        first = next((k for k, (a, b) in enumerate(zip(full["hashes"], run["hashes"])) if a != b), None)
        assert first is None, f"{name} incremental re-sort differs from the full sort from step {first + 1} on"
