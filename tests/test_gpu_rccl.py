"""The in-library RCCL step's failure paths with two ranks on the one GPU (tests/rccl_ranks.py): each rank poses
as its own host, so the exchanges take RCCL's socket transport over loopback.

  * a halo-message overflow on every rank stops both ranks with SPH_ERR_CAPACITY at the same step (step 5: the first
    lag-sized step is 3, its flags are read two steps on), as a local group does: the SZ_* flags are OR-reduced over
    the ranks behind the step's exchanges (abi_multi.cpp phase_finish), no longer between the ρ halo and the boundary
    force pass;
  * ranks that disagree on a switch that decides the exchange sequence (SPH_NO_EARLY_SENDS) fail their init alike
    (read_switches) instead of hanging in mismatched send / receive sequences."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _run(mode: str, tmp_path, extra_env=None, world: int = 2):
    """The ranks as plain processes (no torch.distributed: rank 0 hands the RCCL id over through a file), each with its
    own limit: a rank stuck in a collective is killed, and the test fails instead of hanging."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    idf = tmp_path / "rccl.id"
    errs = [tmp_path / f"rank{r}.err" for r in range(world)]
    procs = [subprocess.Popen([sys.executable, str(ROOT / "tests" / "rccl_ranks.py"), mode, str(r), str(world), str(idf)],
                              env=env, stdout=subprocess.PIPE, stderr=open(errs[r], "w"), text=True) for r in range(world)]
    outs = []
    for p, ef in zip(procs, errs):
        try:
            o, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            tails = "\n".join(f"--- rank {r} stderr:\n" + errs[r].read_text()[-2500:] for r in range(world))
            raise AssertionError(f"{mode}: a rank did not finish within 150 s (a rank waiting alone in a collective)\n"
                                 + tails)
        outs.append((p.returncode, o, ef.read_text()))
    lines = []
    for rc, o, e in outs:
        got = [json.loads(l) for l in o.splitlines() if l.startswith("{")]
        assert rc == 0 and len(got) == 1, (rc, o[-2000:], e[-3000:])
        lines += got
    lines.sort(key=lambda d: d["rank"])
    print(lines)
    return lines


def test_rccl_overflow_stops_every_rank_at_the_same_step(tmp_path):
    lines = _run("overflow", tmp_path, {"SPH_DEBUG_MSG_CAP": "256"})
    for d in lines:
        assert d["status"] == -3, d
        assert "slab step 5:" in d["msg"] and "halo message overflow" in d["msg"], d


def test_rccl_switch_disagreement_fails_every_rank_at_init(tmp_path):
    lines = _run("disagree", tmp_path)
    for d in lines:
        assert d["status"] == -1 and "disagree on SPH_NO_EARLY_SENDS" in d["msg"], d
