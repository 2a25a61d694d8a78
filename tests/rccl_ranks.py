"""Ranks of the in-library RCCL step on one GPU (tests/test_gpu_rccl.py): each rank poses as its own host
(NCCL_HOSTID, as bench.py's SPH_RCCL_HOST_PER_RANK), so RCCL takes its socket transport over loopback. No torch:
rank 0 writes the RCCL unique id to ID_FILE, the other ranks read it from there.

    python tests/rccl_ranks.py MODE RANK WORLD ID_FILE

MODE overflow: every rank caps the lag-sized halo messages (SPH_DEBUG_MSG_CAP, set by the test for all ranks), so the
    receiving sides overflow from step 3 on; every rank must fail its sph_step with SPH_ERR_CAPACITY at the same step
    (the flags' OR over the ranks rides in the lag record of flag steps) instead of one rank returning alone while its
    neighbour waits in the next exchange.
MODE disagree: rank 1 alone sets SPH_NO_EARLY_SENDS; every rank's sph_init_scenario must fail alike (the switch decides
    where a rank issues its exchanges).
Each rank prints one JSON line: {"rank", "mode", "status", "msg"}."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

mode, rank, world, id_file = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), Path(sys.argv[4])
os.environ["NCCL_HOSTID"] = f"sph-test-rank-{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
os.environ.setdefault("NCCL_DEBUG", "WARN")
if mode == "disagree" and rank == 1:
    os.environ["SPH_NO_EARLY_SENDS"] = "1"

import __graft_entry__ as GE  # noqa: E402

pkg = GE.load_package()
from sph_test_amd.context import comm_unique_id  # noqa: E402

if rank == 0:
    tmp = id_file.with_suffix(".tmp")
    tmp.write_bytes(comm_unique_id())
    tmp.rename(id_file)
    uid = id_file.read_bytes()
else:
    t0 = time.time()
    while not id_file.exists():
        if time.time() - t0 > 120:
            raise SystemExit("rank %d: no unique id from rank 0" % rank)
        time.sleep(0.05)
    uid = id_file.read_bytes()
sc = pkg.make_scenario(0, 3, 24 * world, 32, 32, 60 * world, 48, 32, dx=0.01, seed=99)
p, dt = pkg.scenario_params(sc)
ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 1000, device=0)
out = {"rank": rank, "mode": mode, "status": 0, "msg": ""}
try:
    ctx.comm_init(uid, world, rank)
    ctx.set_params(p)
    ctx.set_rebalance(0)
    ctx.init_scenario(sc)
    print(f"rank {rank}: init done", file=sys.stderr, flush=True)
    for s in range(40):   # one call per step: the stderr log shows where a rank stopped
        ctx.step(dt, 1)
        print(f"rank {rank}: step {s} issued", file=sys.stderr, flush=True)
    ctx.synchronize()
except pkg.SphError as e:
    out["status"], out["msg"] = e.status, str(e)
print(json.dumps(out), flush=True)
ctx.close()
