"""bench.py's multi-rank safety logic on CPU (gloo, world 2): the phase agreement of the library-transport
setup (a rank that fails before a collective makes every rank give up together, none waits in it), and the
watchdog that turns a rank stuck in a collective into a failure line and exit status 3."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agree_worker(rank, world, port, fail_phase, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class FakeRunner:
        """Stands in for LibraryRankRunner: rank 1 fails in `fail_phase`; join and init count their calls."""
        calls = []

        def __init__(self, *a, **k):
            if rank == 1 and fail_phase == "create":
                raise RuntimeError("create failed")
            self.ctx = type("C", (), {"close": lambda self: None})()

        def join(self):
            FakeRunner.calls.append("join")
            if rank == 1 and fail_phase == "join":
                raise RuntimeError("join failed")

        def init(self):
            FakeRunner.calls.append("init")
            if rank == 1 and fail_phase == "init":
                raise RuntimeError("init failed")

    bench.LibraryRankRunner = FakeRunner
    runner, err = bench.make_library_runner(None, "C3", None, rank, world, 0, 0, 50, dist, "cpu")
    with open(os.path.join(out, f"r{rank}.json"), "w") as f:
        json.dump({"ok": runner is not None, "err": err, "calls": FakeRunner.calls}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_phase", ["none", "create", "join", "init"])
def test_library_setup_agreement(tmp_path, fail_phase):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, fail_phase, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    if fail_phase == "none":
        assert all(r["ok"] and r["err"] is None and r["calls"] == ["join", "init"] for r in res)
        return
    # every rank gives up, and no rank entered a phase after the one that failed on rank 1
    assert not any(r["ok"] for r in res) and all(r["err"] for r in res)
    stop = {"create": [], "join": ["join"], "init": ["join", "init"]}[fail_phase]
    assert res[0]["calls"] == stop and res[1]["calls"] == stop
    assert f"{fail_phase} failed" in res[1]["err"]


def test_watchdog_fires_with_a_failure_line():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "w = bench.Watchdog(0, 2, 1.0); w.arm('a stuck collective', 1.0); time.sleep(30)") % str(ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and "a stuck collective" in line["watchdog"] and line["n_gpus"] == 2


def test_device_code_hash_identifies_the_code_objects(pkg):
    """The counter files are stamped with this hash and bench.py refuses counters of other code: it is the
    sha256 of libsphhip.so's .hip_fatbin section, stable across loads, and differs for other bytes."""
    import hashlib
    A = pkg._abi
    h = A.device_code_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert A.device_code_hash() == h
    data = A.lib_path().read_bytes()
    assert hashlib.sha256(data).hexdigest()[:16] != h        # the section, not the whole file


def test_load_pmc_refuses_other_code(tmp_path, monkeypatch):
    """A counter file stamped with another hash yields no traffic and a note saying why."""
    sys.path.insert(0, str(ROOT))
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_C3.json").write_text(json.dumps({"config": "C3", "device_code_hash": "0000000000000000",
                                                  "kernel_bytes": {"force_integrate": 123.0}, "kernels": {}}))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    out = bench.load_pmc("C3", "1111111111111111")
    assert "traffic" not in out and "1111111111111111" in out["note"]
    out = bench.load_pmc("C3", "0000000000000000")
    assert out["traffic"] == 123.0


def test_step_bytes_follow_survey_8d():
    """B = 152 + 20·P + 8·C/N (P = ceil(key bits / 8) sort passes)."""
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.step_bytes_per_particle(22, 0, 1) == 152 + 20 * 3
    assert abs(bench.step_bytes_per_particle(22, 3663680, 1048576) - (212 + 8 * 3663680 / 1048576)) < 1e-9
    assert bench.FORCE_BYTES_PER_PARTICLE == 56.0


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def test_plain_start_launches_the_ranks():
    """`python bench.py --gpus 2` without torch.distributed.run starts the two ranks itself: they form one
    process group (gloo here; no GPU call in the launcher) and rank 0's line says n_gpus 2."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launch-check"],
                       env=_bench_env(SPH_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["launch_check"]["backend"] == "gloo"
    assert sorted(x["rank"] for x in line["launch_check"]["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in line["launch_check"]["ranks"]) == [0, 1]
    assert len({x["pid"] for x in line["launch_check"]["ranks"]}) == 2


def test_world_size_mismatch_fails():
    """Launched as one rank of a 2-rank job while asked for 3 GPUs: a failure line and exit status 2,
    before any process group or GPU call."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3"],
                       env=_bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and line["n_gpus"] == 3 and "WORLD_SIZE 2" in line["world_size_mismatch"]


def test_launcher_reports_a_failed_rank(tmp_path):
    """A rank that fails before rank 0 prints: the launcher exits with the worst status and prints a
    failure line naming the ranks' statuses."""
    script = tmp_path / "child.py"
    script.write_text("import os, sys\nr = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '2' and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "sys.exit(5 if r == 1 else 0)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, [], script=%r, grace_s=5))") % (str(ROOT), str(script))
    r = subprocess.run([sys.executable, "-c", code], env=_bench_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 5, (r.stdout, r.stderr)
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] is None and line["n_gpus"] == 2 and [1, 5] in line["failed_ranks"]


def test_kernel_sum_check_flags_a_step_the_samples_miss():
    """verdict r5 item 2: the sampled kernels' sum against the GPU events; within 5% no note, beyond it a note that
    names the gap (the r5 C5 line read 4.37 ms of kernels against 7.75 ms of events)."""
    sys.path.insert(0, str(ROOT))
    import bench
    ok = bench.kernel_sum_check({"density": 0.115, "force_integrate": 0.165, "resort": 0.030}, 0.3125, 16)
    assert ok["kernels_sum_ms_per_step"] == pytest.approx(0.31) and "kernels_note" not in ok
    assert ok["kernels_sum_over_gpu_event"] == pytest.approx(0.31 / 0.3125, abs=1e-4)
    bad = bench.kernel_sum_check({"density": 1.55, "force_integrate": 2.27, "resort": 0.55}, 7.75, 16)
    assert bad["kernels_sum_over_gpu_event"] == pytest.approx(4.37 / 7.75, abs=1e-4)
    assert "+43.6%" in bad["kernels_note"] and "one step in 16" in bad["kernels_note"]
    assert bench.kernel_sum_check({"a": 1.0}, 0.0, 16)["kernels_sum_over_gpu_event"] is None


def test_resort_counts_dict_names_the_library_words():
    """sph_read_resort_counts' eight words (include/sphhip.h) into the bench line's names, in the ABI's order."""
    sys.path.insert(0, str(ROOT))
    import bench
    d = bench.resort_counts_dict([3, 5, 7, 11, 13, 17, 0, 0])
    assert d == {"whole_list_ranges": 3, "whole_list_lanes": 5, "multi_pass_ranges": 7, "passes": 11,
                 "max_range_entries": 13, "share_restreams": 17}
    hdr = (ROOT / "include" / "sphhip.h").read_text()
    assert "sph_read_resort_counts" in hdr
