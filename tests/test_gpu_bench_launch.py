"""`python bench.py --gpus 2` started plainly (no torch.distributed.run) on the one-GPU test box: bench.py
launches the two ranks itself (launch_ranks), both ranks share device 0 over gloo (RCCL needs one GPU per
rank, so the per-phase transport over torch.distributed stands in for it here), the decomposed step passes
its check against one context before anything is timed, and rank 0's line says n_gpus 2."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def test_plain_bench_gpus2_measures_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SPH_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--transport", "python", "--steps", "5",
                        "--warmup", "2", "--no-cpu-baseline", "--mid-steps", "0", "--watchdog", "200"],
                       env=env, capture_output=True, text=True, timeout=400)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    line = lines[0]
    print({k: line.get(k) for k in ("n_gpus", "value", "ms_per_step", "slab_check_max_dx")})
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["slab_check"]["ok"] and line["slab_check"]["particles"] == line["slab_check"]["owned_total"]
    assert line["config"]["particles"] == 2 * 1_048_576     # C3 x 2, weak


def test_plain_bench_gpus2_library_rccl_on_one_gpu():
    """The in-library decomposed step over RCCL (sph_comm_init; early sends on the comm stream, the flags'
    all-reduce) with both ranks on the one GPU: each rank poses as its own host (SPH_RCCL_HOST_PER_RANK sets
    NCCL_HOSTID; RCCL refuses two ranks of one host on one device), so the exchanges take RCCL's socket transport
    over loopback. bench.py's slab check (300 steps, re-balanced every 20) must be bit-identical to one context."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SPH_DIST_BACKEND="gloo", SPH_RCCL_HOST_PER_RANK="1", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
                        "--no-cpu-baseline", "--mid-steps", "0", "--watchdog", "200"],
                       env=env, capture_output=True, text=True, timeout=400)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout[-3000:], r.stderr[-3000:])
    line = lines[0]
    print({k: line.get(k) for k in ("n_gpus", "value", "ms_per_step")}, line["slab_check"])
    assert line["n_gpus"] == 2 and line["config"]["transport"] == "library-rccl"
    assert line["slab_check"]["ok"] and line["slab_check"]["bitwise"] and line["slab_check"]["transport"] == "library"
