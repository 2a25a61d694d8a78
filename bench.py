#!/usr/bin/env python3
"""Headline benchmark: particle-steps/s (+ ms/step) of the SPH step on MI355X.

BASELINE.json metric: "particle-steps/sec + ms/step at 1M particles; 1/2/4/8 MI355X
scaling". At N=1 the workload is configs[2] = C3: 1,048,576 particles, 3D dam-break,
fp32, h = 1.2·dx (SPEC_SPH.md §2), synthetic lattice init (seed 1234). One step = hash →
radix sort → reorder → cell-start → density → force+integrate, over all particles, with
the state already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--no-cpu-baseline]

`python bench.py --gpus N` measures N GPUs however it is started: under torch.distributed.run (WORLD_SIZE
set) it is one rank; started plainly with N > 1 it launches the N rank processes itself (launch_ranks:
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, before any GPU call in the parent),
relays rank 0's JSON line and exits with the worst rank status. A world size other than --gpus is a failure
line and exit status 2. Every rank owns an x-slab of the global tank and exchanges one-cell halos with its
neighbours over RCCL (SPEC_SPH.md §3), so per-GPU work is fixed as N grows ("weak" scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as GE  # noqa: E402

PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
# SURVEY.md §8d, algorithmic bytes per particle-step of the force+visc+XSPH+KDK pass: read x,v,ρ,P 32 B
# + write x,v 24 B (SoA fp32, neighbour reads counted once). roofline.frac prices the kernel on these.
FORCE_BYTES_PER_PARTICLE = 56.0
# this design's own traffic on top: pass 2 reads pass 1's hit mask, 8 words = 32 B per
# target (pass 1 writes the same 32 B). Reported apart, as roofline.frac_design, never as frac.
HIT_MASK_BYTES_PER_PARTICLE = 32.0


def step_bytes_per_particle(key_bits: int, ncells: int, n: int) -> float:
    """algorithmic bytes of one whole step per particle, B = 152 + 20·P + 8·C/N (hash 20,
    sort 20 per 8-bit pass, reorder 52, cell start 4 + 8·C/N, density 20, force 56)."""
    passes = (int(key_bits) + 7) // 8
    return 152.0 + 20.0 * passes + 8.0 * float(ncells) / max(1, int(n))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event pass")
    ap.add_argument("--profile-every", type=int, default=0,
                    help="time the kernels of one step in this many (events in the dispatch packets cost the step "
                         "they ride on; C3: every 4th step +1.0%%, every 16th +0.4%%, profiles/r03_profile_cost_ab.log). "
                         "0 (default): 16, or 4 when fewer than 160 steps are timed")
    ap.add_argument("--slab", action="store_true", help="run the multi-GPU slab step even at N=1 (rehearsal)")
    ap.add_argument("--rebalance", type=int, default=50, help="slab cut re-balancing interval in steps (0: off)")
    ap.add_argument("--transport", choices=("library", "python"), default="library",
                    help="N>1: the decomposed step inside libsphhip.so over RCCL (sph_comm_init), or the per-phase "
                         "slab ABI driven from Python over torch.distributed")
    ap.add_argument("--strong", action="store_true",
                    help="decompose --config itself over the N ranks (strong scaling: C4 on 4 GPUs, C5 on 8) "
                         "instead of stretching it xN")
    ap.add_argument("--mid-steps", type=int, default=200,
                    help="N=1: also time this many steps from a mid-collapse state (0: skip)")
    ap.add_argument("--mid-at", type=int, default=5000,
                    help="step count (from the lattice) at which the mid-collapse timing starts")
    ap.add_argument("--no-check", action="store_true",
                    help="N > 1: skip the decomposed step's correctness check against one context")
    ap.add_argument("--no-strong-extra", action="store_true",
                    help="N = 4 / 8: skip the extra strong-scaling line of BASELINE's C4 / C5")
    ap.add_argument("--watchdog", type=float, default=900.0,
                    help="seconds after which a rank stuck in a phase (a peer failed inside a collective) "
                         "prints the failure and exits 3")
    ap.add_argument("--launch-check", action="store_true",
                    help="N > 1: only form the process group (SPH_DIST_BACKEND) and print which ranks joined "
                         "(tests the launcher without a GPU)")
    ap.add_argument("--table", action="store_true",
                    help="print the GPU / 1-thread / all-thread CPU rate table (SURVEY §8d) instead of the bench line")
    return ap.parse_args()


# VALU issue peak, MEASURED on MI355X (scripts/valu_peak.hip, profiles/r02_valu_peak_long.log): independent
# f32 FMA chains at 8 waves per SIMD in ~3.7 ms dispatches issue 1,153.8 G wave64-instructions/s chip-wide
# (148 TFLOP/s) at an in-kernel clock of 2.39 GHz, 94% of the spec issue rate at that clock (256 CUs x 4
# SIMDs x 1/2 wave-instruction per cycle). Round 1's 891.9 G came from 0.3 ms dispatches, whose ramp and
# tail hid a quarter of the rate. Packed f32 (v_pk_fma_f32) issues ~584 G/s: no faster per flop.
PEAK_VALU_WAVE_INSTR_PER_S = 1153.8e9


def force_kernel_name() -> str:
    return "k_force_tiled"


def load_clock(code_hash: str):
    """Effective shader clocks and the measured VALU issue peak from ONE committed clock file
    (profiles/clock_*.json, scripts/gpu_clock.sh): the force pass on its longest dispatches (C5), the VALU
    microbenchmark's GRBM clock and its issue rate, all taken in the same run on the same box. Only a file
    stamped with the code objects that are running is used (the newest such file)."""
    out = {}
    for f in sorted((ROOT / "profiles").glob("clock_*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if d.get("device_code_hash") != code_hash:
            continue
        cur = {"file": f.name}
        fk = d.get("C5", {}).get("k_force_tiled", {})
        if "clock_ghz_median" in fk:
            cur["force_ghz"] = fk["clock_ghz_median"]
            cur["force_src"] = f"{f.name}: C5 k_force_tiled, {fk['mean_us']:.0f} us dispatches"
        mk = d.get("valu", {}).get("k_fma", {})
        if "clock_ghz_median" in mk:
            cur["micro_ghz"] = mk["clock_ghz_median"]
        vp = d.get("valu_peak", {})
        if "G_wave_instr_per_s" in vp:
            cur["peak"] = vp["G_wave_instr_per_s"] * 1e9
            cur["peak_src"] = f"{f.name}: scripts/valu_peak.hip, 8 waves/SIMD, {vp.get('us', 0):.0f} us dispatches"
        out = cur
    return out


def load_pmc(config: str, code_hash: str):
    """Per-launch counters of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/pmc_*.json): HBM bytes = FETCH_SIZE×2 + WRITE_SIZE (MI355X_MICROARCH.md §HBM) and
    SQ_INSTS_VALU (wave-level VALU instructions). Only a file stamped with the device-code hash of the
    library that is running counts (scripts/pmc_summary.py writes it): counters of other kernels are
    refused, and `note` says why the line then carries no traffic."""
    out = {"note": f"no profiles/pmc_*.json for {config} stamped with device_code_hash {code_hash} "
                   f"(re-take them with scripts/gpu_pmc.sh + scripts/pmc_summary.py)"}
    for f in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if d.get("config") != config:
            continue
        if d.get("device_code_hash") != code_hash:
            continue
        out = {"file": f.name}
        if d.get("kernel_bytes", {}).get("force_integrate"):
            out["traffic"] = d["kernel_bytes"]["force_integrate"]
        for ks in d.get("kernels", {}).values():
            k = ks.get(force_kernel_name(), {})
            if "SQ_INSTS_VALU" in k:
                out["valu_instr"] = k["SQ_INSTS_VALU"]
    return out


def cpu_baseline(config: str, budget_s: float):
    """The C oracle (oracle/, port of SPEC_SPH.md §2) on the host cores, rank 0 only,
    over a bounded sample of the same workload: the C3 initial state, as many whole
    steps as fit in ~budget_s seconds."""
    import numpy as np
    O = GE.load_oracle()
    pkg = GE.load_package()
    sc = pkg.config_scenario(config)
    p, dt = pkg.scenario_params(sc)
    op = O.sph_params(sc.dim, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                      p.wall_restitution, p.forcing_amp, p.forcing_freq)
    x = O.lattice(sc.dim, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    v = np.zeros_like(x)
    ids = np.arange(len(x), dtype=np.int32)
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    threads = max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads) or threads)))
    t0 = time.perf_counter()
    x, v, ids, _, _, _ = O.sph_step(op, x, v, ids, dt, 0.0, nthreads=threads)
    one = time.perf_counter() - t0
    steps = max(1, int(budget_s / max(one, 1e-6)) - 1)
    t0 = time.perf_counter()
    for s in range(steps):
        x, v, ids, _, _, _ = O.sph_step(op, x, v, ids, dt, float(np.float32((s + 1) * dt)), nthreads=threads)
    el = time.perf_counter() - t0
    return {"value": len(x) * steps / el, "unit": "particle-steps/s", "cores": threads, "kind": "port",
            "sample": f"{config} initial state ({len(x)} particles), {steps} oracle steps after 1 warm-up "
                      f"step, {el:.1f} s, OpenMP {threads} threads"}


def _timed_cpu(step, budget_s):
    """Whole steps of `step()` for about budget_s seconds after one warm-up step: (steps, seconds)."""
    t0 = time.perf_counter()
    step()
    one = time.perf_counter() - t0
    steps = max(1, min(1000, int(budget_s / max(one, 1e-6))))
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return steps, time.perf_counter() - t0


def rate_table(budget_s: float, gpu_steps: int = 500):
    """SURVEY.md §8d CPU-baseline table: GPU, 1-thread and all-thread oracle rates (particle-steps/s) at
    C1, C2, C3 (Model S) and Model R at N = 4,096 / 32,768 (positions in the R = 15 sphere, the
    test_gpu_parity recipe). Rank 0, N = 1; the oracle runs only here, as the timed CPU reference."""
    import numpy as np
    import torch
    O = GE.load_oracle()
    pkg = GE.load_package()
    try:
        allc = len(os.sched_getaffinity(0))
    except AttributeError:
        allc = os.cpu_count() or 1
    allc = max(1, min(allc, int(os.environ.get("OMP_NUM_THREADS", allc) or allc)))
    rows = []

    def gpu_rate(step, n):
        step(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step(gpu_steps)
        torch.cuda.synchronize()
        return n * gpu_steps / (time.perf_counter() - t0)

    for cfg in ("C1", "C2", "C3"):
        sim = pkg.SPHSim.from_config(cfg, device=0)
        n = sim.n
        g = gpu_rate(sim.step, n)
        sim.close()
        sc = pkg.config_scenario(cfg)
        p, dt = pkg.scenario_params(sc)
        op = O.sph_params(sc.dim, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                          p.wall_restitution, p.forcing_amp, p.forcing_freq)
        row = {"model": "S", "config": cfg, "particles": n, "gpu": g}
        for th in (1, allc):
            st = {"x": O.lattice(sc.dim, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)}
            st["v"] = np.zeros_like(st["x"])
            st["i"] = np.arange(n, dtype=np.int32)

            def one(st=st, th=th):
                st["x"], st["v"], st["i"], _, _, _ = O.sph_step(op, st["x"], st["v"], st["i"], dt, 0.0, nthreads=th)
            k, el = _timed_cpu(one, budget_s)
            row[f"cpu_{th}t"] = n * k / el
            row[f"cpu_{th}t_steps"] = k
        rows.append(row)
        print(json.dumps(row), flush=True)

    for n in (4096, 32768):
        rng = np.random.default_rng(1234)
        parts = np.zeros(n, pkg.PARTICLE84)
        d = rng.normal(size=(n, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        parts["position"] = d * (15.0 * rng.random((n, 1)) ** (1 / 3))
        parts["radius"] = rng.uniform(1.5, 2.0, n)
        parts["velocity"] = rng.normal(size=(n, 3))
        parts["mass"] = 0.1 * 4.0 / 3.0 * 3.1415926 * parts["radius"] ** 3
        parts["angularVelocity"] = rng.normal(size=(n, 3))
        parts["momentOfInertia"] = 0.4 * parts["mass"] * parts["radius"] ** 2
        parts["drag"] = rng.uniform(0.5, 1.0, n)
        parts["repulsionStrength"] = 1.0
        parts["rotation"] = (0, 0, 0, 1)
        parts["modeIndex"] = -1
        dt = 0.01
        ctl = pkg.ParticleSystemController(particleCount=n)
        ctl.Start(parts.copy())
        g = gpu_rate(lambda k: ctl.context.step(dt, k), n)
        ctl.OnDestroy()
        row = {"model": "R", "config": f"sphere R=15, N={n}", "particles": n, "gpu": g}
        cp = O.contact_params(dt)
        for th in (1, allc):
            st = {"p": parts.view(O.PARTICLE84).copy()}

            def one(st=st, th=th):
                st["p"], _ = O.contact_step(cp, st["p"], nthreads=th)
            k, el = _timed_cpu(one, budget_s)
            row[f"cpu_{th}t"] = n * k / el
            row[f"cpu_{th}t_steps"] = k
        rows.append(row)
        print(json.dumps(row), flush=True)
    # the controller's own scene (InitParticles, ParticleSystemController.cs:12's 4,096 particles) at its 1/144 s frame
    n, dt = 4096, 1.0 / 144.0
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start()
    parts = ctl.GetParticles().copy()
    g = gpu_rate(lambda k: ctl.context.step(dt, k), n)
    ctl.OnDestroy()
    row = {"model": "R", "config": f"controller InitParticles, N={n}, dt=1/144", "particles": n, "gpu": g}
    cp = O.contact_params(dt)
    for th in (1, allc):
        st = {"p": parts.view(O.PARTICLE84).copy()}

        def one(st=st, th=th):
            st["p"], _ = O.contact_step(cp, st["p"], nthreads=th)
        k, el = _timed_cpu(one, budget_s)
        row[f"cpu_{th}t"] = n * k / el
        row[f"cpu_{th}t_steps"] = k
    rows.append(row)
    print(json.dumps(row), flush=True)
    return {"unit": "particle-steps/s", "threads_all": allc, "budget_s_per_cpu_cell": budget_s,
            "gpu_steps": gpu_steps, "rows": rows}


def per_step_ms(kstats: dict, steps: int) -> dict:
    """Mean time per step of each timed scope: mean duration of the sampled launches × launches per step."""
    return {k: round(v["total_ms"] / v["timed"] * v["launches"] / max(1, steps), 4)
            for k, v in kstats.items() if v.get("timed", 0) > 0 and v["total_ms"] > 0}


def resort_counts_dict(c) -> dict:
    """sph_read_resort_counts over the timed steps: whole-list ranges and lanes must be 0 (resort.hip)."""
    return {"whole_list_ranges": int(c[0]), "whole_list_lanes": int(c[1]), "multi_pass_ranges": int(c[2]),
            "passes": int(c[3]), "max_range_entries": int(c[4]), "share_restreams": int(c[5])}


def kernel_sum_check(ks_ms: dict, gpu_event_ms: float, every: int) -> dict:
    """The sampled kernel scopes' sum per step against the GPU-event time of the same steps: a step whose time
    the sampled launches do not name (a kernel slow on other steps than the sampled ones, or gaps between
    launches) shows as a ratio away from 1 and gets a note (verdict r5: the C5 line hid a re-sort cliff)."""
    tot = sum(ks_ms.values())
    out = {"kernels_sum_ms_per_step": round(tot, 4),
           "kernels_sum_over_gpu_event": round(tot / gpu_event_ms, 4) if gpu_event_ms > 0 else None}
    if gpu_event_ms > 0 and abs(tot / gpu_event_ms - 1.0) > 0.05:
        out["kernels_note"] = (f"the timed kernel scopes (one step in {every} sampled) sum to {tot:.4f} ms per step "
                               f"against {gpu_event_ms:.4f} ms of GPU events: {100 * (1 - tot / gpu_event_ms):+.1f}% of "
                               "the step is not in the sampled launches (unsampled slow steps, gaps or overlap)")
    return out


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, script=None, grace_s: float = 60.0) -> int:
    """Start n rank processes of this script (RANK = LOCAL_RANK = r, WORLD_SIZE = n, MASTER_ADDR 127.0.0.1,
    MASTER_PORT from the environment or a free port), as torch.distributed.run would on one node. The parent
    makes no GPU call: it only relays rank 0's stdout and waits. When a rank fails, the others get grace_s to
    finish (their own watchdogs end a collective a failed peer never joins), then are terminated. Returns the
    worst exit status (a signal counts as 128 + signal); if rank 0 printed no JSON line with "metric", a
    failure line is printed for it."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", str(script or Path(__file__).resolve()), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    printed = []

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()
            try:
                if "metric" in json.loads(line):
                    printed.append(True)
            except ValueError:
                pass
    t = threading.Thread(target=relay, daemon=True)
    t.start()
    first_fail = None
    while any(p.poll() is None for p in procs):
        codes = [p.poll() for p in procs]
        if first_fail is None and any(c not in (None, 0) for c in codes):
            first_fail = time.monotonic()
        if first_fail is not None and time.monotonic() - first_fail > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
    t.join(timeout=10)
    codes = [p.returncode for p in procs]
    worst = max((c if c >= 0 else 128 - c) for c in codes)
    if not printed:
        bad = [(r, c) for r, c in enumerate(codes) if c != 0]
        print(json.dumps({"metric": METRIC, "value": None, "unit": "particle-steps/s", "n_gpus": n,
                          "launch_failed": f"rank 0 printed no result line; exit status per rank {codes}",
                          "failed_ranks": bad}), flush=True)
        worst = worst or 1
    return worst


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1 and not args.table:
        # started plainly: this process becomes the launcher of the N ranks (no GPU call here)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if world != args.gpus:
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "particle-steps/s", "n_gpus": args.gpus,
                              "world_size_mismatch": f"--gpus {args.gpus} but WORLD_SIZE {world}"}), flush=True)
        sys.exit(2)
    every = args.profile_every if args.profile_every > 0 else (16 if args.steps >= 160 else 4)
    prof = 0 if args.no_profile else max(1, every)
    import torch
    if args.table:
        torch.cuda.set_device(0)
        print(json.dumps({"rate_table": rate_table(args.cpu_seconds)}), flush=True)
        return
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL over xGMI between GPUs; SPH_DIST_BACKEND=gloo rehearses N ranks on one GPU
    backend = os.environ.get("SPH_DIST_BACKEND", "nccl")
    if args.launch_check:
        launch_check(world, rank, local, backend, dist)
        return
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if os.environ.get("SPH_RCCL_HOST_PER_RANK"):
            # rehearsal of the in-library RCCL step with every rank on one GPU: RCCL refuses two ranks of one host
            # on one device, so each rank poses as a host of its own and the exchanges take RCCL's socket transport
            os.environ["NCCL_HOSTID"] = f"sph-rank-{rank}"
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    pkg = GE.load_package()

    dev_kind = "cuda" if backend == "nccl" else "cpu"
    multi = world > 1 or args.slab or args.strong
    watchdog = Watchdog(rank, world, args.watchdog)

    def fail_line(key: str, err: str, extra=None):
        """A multi-rank failure: one JSON line (rank 0) with the failure instead of a number, exit 3."""
        if rank == 0:
            line = {"metric": METRIC, "value": None, "unit": "particle-steps/s", "n_gpus": world, key: err}
            line.update(extra or {})
            print(json.dumps(line), flush=True)
        print(json.dumps({"rank": rank, key: err}), file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)

    check = None
    if multi and world > 1 and not args.no_check:
        # correctness of the decomposed step through the SAME transport before anything is timed
        watchdog.arm("slab_check", 300)
        check = slab_check(pkg, args.transport, rank, world, local, dist, dev_kind)
        watchdog.disarm()
        if not check["ok"]:
            fail_line("slab_check_failed", check.get("error", "mismatch"), {"slab_check": check})

    if multi and args.transport == "library":
        # the decomposed step inside libsphhip.so: one RCCL communicator, no host read per step. No
        # fallback: a failure on any rank ends the run with the failure in the line.
        watchdog.arm("library transport setup", 300)
        scenario = pkg.config_scenario(args.config) if args.strong else None
        runner, err = make_library_runner(pkg, args.config, scenario, rank, world, local, prof, args.rebalance,
                                          dist, dev_kind)
        if err:
            fail_line("library_transport_failed", err)
        watchdog.disarm()
    elif multi:
        from sph_test_amd import slab
        runner = slab.SlabRunner(args.config, rank, world, device=local, profile=bool(prof),
                                 rebalance_every=args.rebalance,
                                 scenario=pkg.config_scenario(args.config) if args.strong else None)
    else:
        runner = SingleRunner(pkg, args.config, local, profile=prof)

    # one explicit HIP stream shared by torch (events, RCCL ordering) and libsphhip
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    runner.bind_stream(stream.cuda_stream)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(r, warmup, steps):
        """W untimed steps, then K steps between barrier + synchronize pairs; max wall over ranks."""
        watchdog.arm("timed steps", args.watchdog)
        try:
            r.step(warmup)
            barrier()
            r.reset_stats()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            barrier()
            t = time.perf_counter()
            e0.record(stream)
            r.step(steps)
            e1.record(stream)
            barrier()
            w = time.perf_counter() - t
        except Exception as e:   # noqa: BLE001 - reported; the other ranks end by the watchdog
            fail_line("step_failed", f"rank {rank}: {e}")
        watchdog.disarm()
        el = torch.tensor([w], dtype=torch.float64, device=dev_kind)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()), e0.elapsed_time(e1)

    wall, gpu_ms = timed(runner, args.warmup, args.steps)
    n_total = runner.total_particles()
    value = n_total * args.steps / wall
    kstats = runner.kernel_stats()
    rcounts = runner.resort_counts() if hasattr(runner, "resort_counts") else None

    roofline = None
    fi = kstats.get("force_integrate")
    code_hash = pkg._abi.device_code_hash()
    if fi and fi.get("timed", 0) > 0 and fi["total_ms"] > 0:
        avg_s = fi["total_ms"] / fi["timed"] / 1e3
        n_local = runner.local_particles()
        # the force pass may run as several x-plane chunks per step (host_step.cpp, SPH_CHUNKS): a launch
        # then covers its share of the particles
        per_step = max(1.0, fi["launches"] / max(1, args.steps))
        n_launch = n_local / per_step
        bytes_per_launch = FORCE_BYTES_PER_PARTICLE * n_launch
        achieved = bytes_per_launch / avg_s / 1e9
        design = (FORCE_BYTES_PER_PARTICLE + HIT_MASK_BYTES_PER_PARTICLE) * n_launch / avg_s / 1e9
        if world == 1:
            pmc = load_pmc(args.config, code_hash)
        else:
            pmc = {"note": "PMC counters are taken on one GPU (profiles/pmc_*.json); none at N > 1"}
        traffic = pmc.get("traffic")
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic,
                    "kernel": force_kernel_name(), "kernel_avg_us": round(avg_s * 1e6, 2),
                    "bytes_per_launch": bytes_per_launch, "launches_per_step": per_step,
                    "algorithmic_bytes_per_particle": FORCE_BYTES_PER_PARTICLE,
                    "bytes_source": "SURVEY.md §8d: force+visc+XSPH+KDK reads x,v,rho,P 32 B, writes x,v 24 B",
                    "frac_design": round(design / PEAK_HBM_GBS, 5),
                    "design_bytes_per_particle": FORCE_BYTES_PER_PARTICLE + HIT_MASK_BYTES_PER_PARTICLE,
                    "design_bytes_note": "+32 B hit-mask read (pass 1 writes it; DESIGN.md §4)",
                    "device_code_hash": code_hash}
        if traffic:
            roofline["traffic_over_algorithmic"] = round(traffic / bytes_per_launch, 3)
            roofline["traffic_source"] = pmc.get("file")
        else:
            roofline["traffic_note"] = pmc.get("note")
        try:
            st = runner.grid_stats()
            b = step_bytes_per_particle(st["key_bits"], st["ncells"], n_local)
            ms = wall * 1e3 / args.steps
            roofline["step"] = {"bytes_per_particle": round(b, 2), "achieved": round(b * n_local / (ms * 1e-3) / 1e9, 2),
                                "frac": round(b * n_local / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5),
                                "ms_per_step": round(ms, 4),
                                "source": "SURVEY.md §8d: B = 152 + 20*P + 8*C/N over the whole step, against "
                                          f"ms_per_step (P = {(st['key_bits'] + 7) // 8} 8-bit sort passes, "
                                          f"C = {st['ncells']} cells, N = {n_local})"}
        except Exception as e:   # noqa: BLE001 - reported in the line
            roofline["step"] = {"error": str(e)}
        if "valu_instr" in pmc:
            # what bounds the neighbour pass in practice: VALU issue, from the same
            # kernel's committed PMC pass and this run's kernel time, priced two ways: against the
            # microbenchmark's issue rate and against the spec issue rate (256 CUs × 4 SIMDs × ½
            # wave64-instruction per cycle) at the clock the chip held during the force pass. The peak, both
            # clocks and the counters come from files stamped with this library's device-code hash; the peak
            # and its clock were measured in one run on one box (scripts/gpu_clock.sh).
            va = pmc["valu_instr"] / avg_s
            clk = load_clock(code_hash)
            peak = clk.get("peak", PEAK_VALU_WAVE_INSTR_PER_S)
            roofline["valu"] = {"achieved": round(va / 1e9, 2), "peak": round(peak / 1e9, 1),
                                "unit": "G wave-instr/s", "frac": round(va / peak, 4),
                                "source": "rocprofv3 SQ_INSTS_VALU per launch (" + str(pmc.get("file")) + "); peak: " +
                                          clk.get("peak_src", "scripts/valu_peak.hip (profiles/r02_valu_peak_long.log)")}
            if "force_ghz" in clk:
                spec = 256 * 4 * 0.5 * clk["force_ghz"] * 1e9
                roofline["valu"].update({
                    "force_clock_ghz": round(clk["force_ghz"], 3),
                    "spec_peak_at_force_clock": round(spec / 1e9, 1),
                    "frac_of_spec_at_clock": round(va / spec, 4),
                    "clock_source": clk["force_src"]})
            if "micro_ghz" in clk and "peak" in clk:
                mf = clk["peak"] / (256 * 4 * 0.5 * clk["micro_ghz"] * 1e9)
                if mf <= 1.0:
                    roofline["valu"]["microbench_clock_ghz"] = round(clk["micro_ghz"], 3)
                    roofline["valu"]["microbench_frac_of_spec_at_its_clock"] = round(mf, 4)
                else:   # a rate above the spec at its clock: the clock reading is wrong, report neither
                    roofline["valu"]["microbench_clock_note"] = (
                        f"refused: measured peak over spec at the GRBM clock {clk['micro_ghz']:.3f} GHz ({mf:.3f} > 1)")
            for k in ("frac", "frac_of_spec_at_clock"):
                if roofline["valu"].get(k, 0) > 1.0:
                    roofline["valu"][k + "_note"] = "above 1: inconsistent denominators, not a measurement"
                    roofline["valu"].pop(k)

    mid = None
    if isinstance(runner, SingleRunner) and args.mid_steps > 0:
        # a representative state beside the driver's line: the timed region above starts a few steps
        # after the lattice, before the column moves; this one starts mid-collapse (untimed advance)
        done = args.warmup + args.steps
        if done < args.mid_at:
            runner.step(args.mid_at - done)
        barrier()
        runner.reset_stats()
        barrier()
        t0 = time.perf_counter()
        runner.step(args.mid_steps)
        barrier()
        mwall = time.perf_counter() - t0
        mks = runner.kernel_stats()
        mid = {"ms_per_step_mid_collapse": round(mwall * 1e3 / args.mid_steps, 4),
               "value_mid_collapse": round(runner.total_particles() * args.mid_steps / mwall, 1),
               "mid_collapse_state": runner.mid_state(max(done, args.mid_at), args.mid_steps),
               "kernels_ms_per_step_mid_collapse": per_step_ms(mks, args.mid_steps),
               "resort_counts_mid_collapse": runner.resort_counts()}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_seconds)

    workload = runner.workload("strong" if args.strong else "weak")
    local_n = runner.local_particles()
    transport = getattr(runner, "transport", "single" if world == 1 else "python")
    runner.close()

    strong = None
    if world in STRONG_CONFIGS and not args.strong and args.transport == "library" and not args.no_strong_extra:
        # BASELINE.json's own multi-GPU configurations in the same invocation: C4 (sloshing) decomposed
        # over 4 GPUs, C5 over 8 (strong scaling), beside the C3xN weak line above
        cfg = STRONG_CONFIGS[world]
        watchdog.arm(f"strong {cfg} setup", 300)
        r2, err = make_library_runner(pkg, cfg, pkg.config_scenario(cfg), rank, world, local, 0, args.rebalance,
                                      dist, dev_kind)
        if err:
            fail_line("library_transport_failed", f"strong {cfg}: {err}")
        watchdog.disarm()
        r2.bind_stream(stream.cuda_stream)
        w2, g2 = timed(r2, args.warmup, args.steps)
        strong = {"config": cfg, "workload": r2.workload("strong"), "particles": r2.total_particles(),
                  "value": round(r2.total_particles() * args.steps / w2, 1), "unit": "particle-steps/s",
                  "ms_per_step": round(w2 * 1e3 / args.steps, 4), "gpu_event_ms_per_step": round(g2 / args.steps, 4),
                  "scaling": "strong", "steps": args.steps, "warmup": args.warmup}
        r2.close()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "particle-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (dam-break lattice, seed 1234)",
            "config": {"workload": workload, "particles": n_total,
                       "particles_per_gpu": local_n, "h_over_dx": 1.2,
                       "parallelism": f"slab{world}" if world > 1 else "single",
                       "transport": transport},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "kernels_ms_per_step": per_step_ms(kstats, args.steps),
            "resort_counts": rcounts,
        }
        if prof:
            line.update(kernel_sum_check(line["kernels_ms_per_step"], gpu_ms / args.steps, prof))
        if mid:
            line.update(mid)
        if check is not None:
            line["slab_check"] = check
            line["slab_check_max_dx"] = check.get("max_dx")
        if strong is not None:
            line["strong_baseline_config"] = strong
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


METRIC = "particle-steps/sec + ms/step at 1M particles; 1/2/4/8 MI355X scaling"
# BASELINE.json configs[3] / configs[4]: the strong lines a 4- and an 8-GPU run add to the weak C3xN line
STRONG_CONFIGS = {4: "C4", 8: "C5"}


class Watchdog:
    """Ends a rank whose phase does not finish in time (a collective whose peer failed never returns):
    prints the failure (rank 0: as the JSON line) and exits 3, instead of hanging until an outer limit."""

    def __init__(self, rank, world, default_s):
        self.rank, self.world, self.default = rank, world, default_s
        self.t = None

    def arm(self, what, seconds=None):
        import threading
        self.disarm()
        secs = seconds or self.default

        def fire():
            err = f"rank {self.rank}: '{what}' did not finish in {secs} s (a rank failed or hung)"
            if self.rank == 0:
                print(json.dumps({"metric": METRIC, "value": None, "unit": "particle-steps/s", "n_gpus": self.world,
                                  "watchdog": err}), flush=True)
            print(json.dumps({"rank": self.rank, "watchdog": err}), file=sys.stderr, flush=True)
            os._exit(3)
        self.t = threading.Timer(secs, fire)
        self.t.daemon = True
        self.t.start()

    def disarm(self):
        if self.t is not None:
            self.t.cancel()
            self.t = None


def launch_check(world, rank, local, backend, dist):
    """--launch-check: form the process group and report the ranks that joined (no GPU with gloo)."""
    import torch
    if world > 1:
        if backend == "nccl":
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % max(1, torch.cuda.device_count())))
        else:
            dist.init_process_group(backend)
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "local_rank": local, "pid": os.getpid()})
        size = dist.get_world_size()
    else:
        got, size = [{"rank": 0, "local_rank": 0, "pid": os.getpid()}], 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "particle-steps/s", "n_gpus": size,
                          "launch_check": {"backend": backend if world > 1 else None, "ranks": got}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def agree(ok: bool, dist, dev_kind) -> bool:
    """True on every rank iff every rank's ok is True (an all-reduce MIN)."""
    import torch
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev_kind)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return int(flag.item()) == 1


def make_library_runner(pkg, config, scenario, rank, world, device, profile, rebalance_every, dist, dev_kind):
    """LibraryRankRunner in phases, each followed by an agreement over all ranks, so a rank that fails
    before a collective (ncclCommInitRank, the first step's exchanges) never leaves the others waiting
    in it: (runner, None) on every rank, or (None, error) on every rank."""
    runner, err = None, None
    try:
        runner = LibraryRankRunner(pkg, config, scenario, rank, world, device, profile, rebalance_every, dist, dev_kind)
    except Exception as e:   # noqa: BLE001 - agreed on below
        err = f"rank {rank} create: {e}"
    for phase in ("join", "init"):
        if world > 1 and not agree(err is None, dist, dev_kind):
            if runner is not None:
                runner.ctx.close()
            return None, err or f"another rank failed before '{phase}'"
        try:
            getattr(runner, phase)()
        except Exception as e:   # noqa: BLE001 - agreed on below
            err = f"rank {rank} {phase}: {e}"
    if world > 1 and not agree(err is None, dist, dev_kind):
        if runner is not None:
            runner.ctx.close()
        return None, err or "another rank failed in init"
    if err:
        return None, err
    return runner, None


def check_scenario(pkg, world):
    """The multi-rank check's workload: a dam-break whose fluid column and tank grow with the ranks
    (24 lattice columns and 60 dx of tank per rank: ~10 grid columns per slab at h = 1.2 dx)."""
    return pkg.make_scenario(pkg.SPH_SCENARIO_DAMBREAK, 3, 24 * world, 32, 32, 60 * world, 48, 32, dx=0.01, seed=99)


CHECK_STEPS, CHECK_REBALANCE = 300, 20
# owned positions against one context on rank 0 after CHECK_STEPS (300: the dam-break has moved the cuts
# 2-6 times by then). Every slab keeps the single domain's slot order, so the decomposed run is expected
# bit-identical (measured: local groups of 2, 4 and 8 slabs through 1,000 steps and 22 re-cuts,
# tests/test_gpu_multi.py); the limit leaves room only for fp32 rounding, and `bitwise` reports which.
CHECK_MAX_DX = 2e-5


def slab_check(pkg, transport, rank, world, device, dist, dev_kind):
    """Before timing N > 1: run the decomposed step through the same transport on a small dam-break for
    CHECK_STEPS steps with re-balancing every CHECK_REBALANCE, gather every rank's owned particles on
    rank 0 and compare them with a single context there. Returns a dict (the same on every rank)."""
    sc = check_scenario(pkg, world)
    out = {"ok": True, "steps": CHECK_STEPS, "rebalance_every": CHECK_REBALANCE, "transport": transport,
           "scenario": f"dam-break column {sc.nx}x{sc.ny}x{sc.nz}, tank {sc.tx}x{sc.ty}x{sc.tz} dx"}
    if transport == "library":
        r, err = make_library_runner(pkg, "check", sc, rank, world, device, 0, CHECK_REBALANCE, dist, dev_kind)
        if err:
            return {**out, "ok": False, "error": f"library transport: {err}"}
    else:
        from sph_test_amd import slab
        r = slab.SlabRunner("check", rank, world, device=device, scenario=sc, rebalance_every=CHECK_REBALANCE)
    err = None
    try:
        r.step(CHECK_STEPS)
        rec = r.owned()
    except Exception as e:   # noqa: BLE001 - agreed on below
        err, rec = f"rank {rank}: {e}", np.zeros((0, 8), np.float32)
    r.close()
    if not agree(err is None, dist, dev_kind):
        return {**out, "ok": False, "error": err or "another rank's step failed"}
    allrec = [None] * world
    dist.all_gather_object(allrec, rec)
    res = None
    if rank == 0:
        rec = np.concatenate(allrec)
        ids = rec[:, 6].view(np.int32)
        sim = pkg.SPHSim(sc, device=device)
        sim.step(CHECK_STEPS)
        xs, vs = sim.positions(), sim.velocities()
        sim.close()
        res = {"particles": len(xs), "owned_total": int(len(rec))}
        if len(rec) != len(xs) or not np.array_equal(np.sort(ids), np.arange(len(xs))):
            res.update(ok=False, error="the ranks do not own every particle exactly once")
        else:
            order = np.argsort(ids)
            dx = float(np.abs(rec[order, 0:3] - xs).max())
            dv = float(np.abs(rec[order, 3:6] - vs).max())
            res.update(max_dx=dx, max_dv=dv, max_dx_limit=CHECK_MAX_DX, bitwise=bool(dx == 0.0 and dv == 0.0))
            if not np.isfinite(rec[:, :6]).all() or not dx <= CHECK_MAX_DX:
                res.update(ok=False, error=f"max |dx| {dx:.3g} > {CHECK_MAX_DX:g} against one context")
    box = [res]
    dist.broadcast_object_list(box, 0)
    out.update(box[0])
    return out


class LibraryRankRunner:
    """One rank of the in-library decomposed step (sphhip.h sph_comm_init): rank 0 makes the RCCL
    unique id, torch.distributed hands its 128 bytes to every rank, and from then on sph_step runs the
    whole decomposed step (halos, re-sort, density, ρ halo overlapped with the interior force pass,
    re-balancing) with no host read per step. Built in three phases (make_library_runner agrees on
    each one's outcome over all ranks before the next, collective one starts)."""
    transport = "library-rccl"

    def __init__(self, pkg, config, scenario, rank, world, device, profile, rebalance_every, dist, dev_kind):
        import torch
        from sph_test_amd import slab
        from sph_test_amd.context import comm_unique_id
        self.pkg, self.config, self.world, self.rank = pkg, config, world, rank
        self.scenario = scenario if scenario is not None else slab.weak_scenario(config, world)
        self.params, self.dt = pkg.scenario_params(self.scenario)
        self.rebalance_every, self.profile = rebalance_every, profile
        buf = torch.zeros(128, dtype=torch.uint8, device=torch.device(dev_kind, device) if dev_kind == "cuda" else "cpu")
        if rank == 0:
            buf.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
        if world > 1:
            dist.broadcast(buf, 0)
        self.uid = bytes(buf.cpu().numpy().tobytes())
        self.ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, self.scenario.dim, 1024, device=device, profile=bool(profile))
        if profile:
            self.ctx.set_profile_every(profile)

    def join(self):
        """ncclCommInitRank: collective over all ranks."""
        self.ctx.comm_init(self.uid, self.world, self.rank)

    def init(self):
        self.ctx.set_params(self.params)
        self.ctx.set_rebalance(self.rebalance_every)
        self.ctx.init_scenario(self.scenario)
        d = self.ctx.decomposition()
        self.n_total, self.cut = d.total, (d.cut.cx_lo, d.cut.cx_hi)

    def grid_stats(self):
        st = self.ctx.stats()
        return {"key_bits": st.key_bits, "ncells": st.grid[0] * st.grid[1] * st.grid[2]}

    def owned(self):
        """This rank's owned particles as 8-float records (x, y, z, u, v, w, id-bits, ρ)."""
        import ctypes as C
        A = self.pkg._abi
        rec = np.empty((max(self.ctx.stats().capacity, 1), 8), np.float32)
        n = C.c_int32()
        A.check("sph_slab_read_owned", self.ctx._L.sph_slab_read_owned(self.ctx.handle, A.ptr(rec), len(rec), C.byref(n)),
                self.ctx.handle)
        return rec[: n.value]

    def bind_stream(self, handle):
        self.ctx.set_stream(handle)

    def step(self, k):
        self.ctx.step(self.dt, k)

    def reset_stats(self):
        self.ctx.reset_kernel_stats()
        self.ctx.resort_counts(reset=True)

    def kernel_stats(self):
        return self.ctx.kernel_stats()

    def resort_counts(self):
        return resort_counts_dict(self.ctx.resort_counts(reset=False))

    def total_particles(self):
        return self.n_total

    def local_particles(self):
        return int(self.ctx.decomposition().owned)

    def workload(self, scaling: str = "weak"):
        sc = self.scenario
        kind = "sloshing" if sc.kind == self.pkg.SPH_SCENARIO_SLOSHING else "dam-break"
        name = f"{self.config}x{self.world} weak" if scaling == "weak" else f"{self.config} on {self.world} GPUs"
        return (f"{name}: {self.n_total} particles, {sc.dim}D {kind}, column {sc.nx}x{sc.ny}x{sc.nz}, "
                f"tank {sc.tx}x{sc.ty}x{sc.tz} dx, x-slabs (rank 0 {self.cut})")

    def close(self):
        self.ctx.close()


class SingleRunner:
    def __init__(self, pkg, config, device, profile):
        self.pkg = pkg
        self.config = config
        self.sim = pkg.SPHSim.from_config(config, device=device, profile=bool(profile))
        if profile:
            self.sim.ctx.set_profile_every(profile)

    def bind_stream(self, handle):
        self.sim.ctx.set_stream(handle)

    def step(self, k):
        self.sim.step(k)

    def reset_stats(self):
        self.sim.ctx.reset_kernel_stats()
        self.sim.ctx.resort_counts(reset=True)

    def kernel_stats(self):
        return self.sim.ctx.kernel_stats()

    def resort_counts(self):
        return resort_counts_dict(self.sim.ctx.resort_counts(reset=False))

    def total_particles(self):
        return self.sim.n

    def local_particles(self):
        return self.sim.n

    def mid_state(self, start: int, steps: int) -> str:
        sc = self.sim.scenario
        L = sc.nx * sc.dx
        T = start * self.sim.dt * (2 * 9.81 / L) ** 0.5
        return (f"{self.config} steps {start}-{start + steps} from the lattice: t = {start * self.sim.dt:.3f} s, "
                f"T = t*sqrt(2g/L) = {T:.2f} (surge front running along the floor)")

    def grid_stats(self):
        st = self.sim.ctx.stats()
        return {"key_bits": st.key_bits, "ncells": st.grid[0] * st.grid[1] * st.grid[2]}

    def workload(self, scaling: str = "weak"):
        sc = self.sim.scenario
        kind = "sloshing" if sc.kind == self.pkg.SPH_SCENARIO_SLOSHING else "dam-break"
        return (f"{self.config}: {self.sim.n} particles, {sc.dim}D {kind}, column {sc.nx}x{sc.ny}x{sc.nz}, "
                f"tank {sc.tx}x{sc.ty}x{sc.tz} dx")

    def close(self):
        self.sim.close()


if __name__ == "__main__":
    main()
