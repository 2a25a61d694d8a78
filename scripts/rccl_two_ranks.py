"""Two RCCL ranks of the in-library step (sph_comm_init), one per GPU; needs two GPUs (RCCL refuses two
ranks on one device: "ncclCommInitRank: invalid usage", seen on the one-GPU test box). Compares the owned
particles after 60 steps with re-balancing every 20 against a single context (2e-6, as the group tests).
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 scripts/rccl_two_ranks.py"""
import os
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import torch
import torch.distributed as dist
import __graft_entry__ as GE

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = rank % max(1, torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group("gloo")
pkg = GE.load_package()
from sph_test_amd.context import comm_unique_id
uid = [comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, 0)
sc = pkg.make_scenario(0, 3, 48, 32, 32, 120, 48, 32, dx=0.01, seed=99)
p, dt = pkg.scenario_params(sc)
ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, 3, 1000, device=dev)
ctx.comm_init(uid[0], world, rank)
ctx.set_params(p)
ctx.set_rebalance(20)
ctx.init_scenario(sc)
steps = 60
ctx.step(dt, steps)
d = ctx.decomposition()
import ctypes as C
from sph_test_amd import _abi as A
rec = np.empty((ctx.stats().capacity, 8), np.float32)
n = C.c_int32()
A.check("sph_slab_read_owned", ctx._L.sph_slab_read_owned(ctx.handle, A.ptr(rec), len(rec), C.byref(n)), ctx.handle)
rec = rec[: n.value]
allrec = [None] * world
dist.all_gather_object(allrec, rec)
if rank == 0:
    rec = np.concatenate(allrec)
    order = np.argsort(rec[:, 6].view(np.int32))
    sim = pkg.SPHSim(sc)
    sim.step(steps)
    xs = sim.positions()
    x = rec[order, 0:3]
    print({"world": world, "owned_total": len(rec), "particles": len(xs), "rebalances": d.rebalances,
           "max_dx": float(np.abs(x - xs).max())}, flush=True)
    assert len(rec) == len(xs)
    assert np.abs(x - xs).max() < 2e-6
    print("rccl two ranks: OK", flush=True)
ctx.close()
dist.barrier()
dist.destroy_process_group()
