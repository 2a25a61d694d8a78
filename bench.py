#!/usr/bin/env python3
"""Headline benchmark: particle-steps/s (+ ms/step) of the SPH step on MI355X.

BASELINE.json metric: "particle-steps/sec + ms/step at 1M particles; 1/2/4/8 MI355X
scaling". At N=1 the workload is configs[2] = C3: 1,048,576 particles, 3D dam-break,
fp32, h = 1.2·dx (SPEC_SPH.md §2), synthetic lattice init (seed 1234). One step = hash →
radix sort → reorder → cell-start → density → force+integrate, over all particles, with
the state already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--no-cpu-baseline]

For N > 1 it is launched by torch.distributed.run. Every rank owns an x-slab of the
global tank and exchanges one-cell halos with its neighbours over RCCL (SPEC_SPH.md §3),
so per-GPU work is fixed as N grows ("weak" scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as GE  # noqa: E402

PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
# SURVEY.md §8d, algorithmic bytes per particle-step of the force+visc+XSPH+KDK pass: read x,v,ρ,P 32 B
# + write x,v 24 B (SoA fp32, neighbour reads counted once) + this design's hit mask, 8 words read 32 B
# (pass 1 writes it)
FORCE_BYTES_PER_PARTICLE = 88.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel HIP-event pass")
    ap.add_argument("--profile-every", type=int, default=4,
                    help="time the kernels of one step in this many (events in the dispatch packets still cost a "
                         "C3 step ~15 us, so the timed region samples them)")
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


def load_clock():
    """Effective shader clocks from the committed rocprofv3 GRBM passes (profiles/clock_*.json,
    scripts/gpu_clock.sh): the force pass on its longest dispatches (C5) and the VALU microbenchmark."""
    out = {}
    for f in sorted((ROOT / "profiles").glob("clock_*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if "k_force_tiled" in d.get("C5", {}):
            out["force_ghz"] = d["C5"]["k_force_tiled"]["clock_ghz_median"]
            out["force_src"] = f"{f.name}: C5 k_force_tiled, {d['C5']['k_force_tiled']['mean_us']:.0f} us dispatches"
        if "k_fma" in d.get("valu", {}):
            out["micro_ghz"] = d["valu"]["k_fma"]["clock_ghz_median"]
        out["file"] = f.name
    return out


def load_pmc(config: str):
    """Per-launch counters of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/pmc_*.json): HBM bytes = FETCH_SIZE×2 + WRITE_SIZE (MI355X_MICROARCH.md §HBM) and
    SQ_INSTS_VALU (wave-level VALU instructions)."""
    out = {}
    for f in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        if d.get("config") != config:
            continue
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


def rate_table(budget_s: float, gpu_steps: int = 50):
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
    return {"unit": "particle-steps/s", "threads_all": allc, "budget_s_per_cpu_cell": budget_s,
            "gpu_steps": gpu_steps, "rows": rows}


def per_step_ms(kstats: dict, steps: int) -> dict:
    """Mean time per step of each timed scope: mean duration of the sampled launches × launches per step."""
    return {k: round(v["total_ms"] / v["timed"] * v["launches"] / max(1, steps), 4)
            for k, v in kstats.items() if v.get("timed", 0) > 0 and v["total_ms"] > 0}


def main():
    args = parse()
    prof = 0 if args.no_profile else max(1, args.profile_every)
    import torch
    if args.table:
        torch.cuda.set_device(0)
        print(json.dumps({"rate_table": rate_table(args.cpu_seconds)}), flush=True)
        return
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL over xGMI between GPUs; SPH_DIST_BACKEND=gloo rehearses N ranks on one GPU
    backend = os.environ.get("SPH_DIST_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    pkg = GE.load_package()

    runner = None
    if (world > 1 or args.slab or args.strong) and args.transport == "library":
        # the decomposed step inside libsphhip.so: one RCCL communicator, no host read per step
        try:
            runner = LibraryRankRunner(pkg, args.config, rank, world, local, profile=prof,
                                       rebalance_every=args.rebalance, strong=args.strong)
        except Exception as e:   # noqa: BLE001 - reported, then the torch.distributed slab path (also RCCL)
            print(json.dumps({"rank": rank, "library_transport_failed": str(e)}), file=sys.stderr, flush=True)
            runner = None
    if runner is not None and world > 1:
        # every rank checks one step of the in-library path; if any rank failed, all take the
        # torch.distributed slab path instead (the same kernels, RCCL through torch)
        ok = 1
        try:
            runner.step(1)
            torch.cuda.synchronize()
        except Exception as e:   # noqa: BLE001 - reported
            ok = 0
            print(json.dumps({"rank": rank, "library_step_failed": str(e)}), file=sys.stderr, flush=True)
        flag = torch.tensor([ok], dtype=torch.int32, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            runner.close()
            runner = None
    if runner is None and (world > 1 or args.slab or args.strong):
        from sph_test_amd import slab
        runner = slab.SlabRunner(args.config, rank, world, device=local, profile=bool(prof),
                                 rebalance_every=args.rebalance,
                                 scenario=pkg.config_scenario(args.config) if args.strong else None)
    elif runner is None:
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

    runner.step(args.warmup)
    barrier()
    runner.reset_stats()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    runner.step(args.steps)
    ev1.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    el = torch.tensor([wall], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    wall = float(el.item())
    n_total = runner.total_particles()
    value = n_total * args.steps / wall
    kstats = runner.kernel_stats()

    roofline = None
    fi = kstats.get("force_integrate")
    if fi and fi.get("timed", 0) > 0 and fi["total_ms"] > 0:
        avg_s = fi["total_ms"] / fi["timed"] / 1e3
        bytes_per_launch = FORCE_BYTES_PER_PARTICLE * runner.local_particles()
        achieved = bytes_per_launch / avg_s / 1e9
        pmc = load_pmc(args.config) if world == 1 else {}
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": pmc.get("traffic"),
                    "kernel": force_kernel_name(), "kernel_avg_us": round(avg_s * 1e6, 2),
                    "bytes_per_launch": bytes_per_launch}
        if "valu_instr" in pmc:
            # what bounds the neighbour pass in practice: VALU issue, from the same
            # kernel's committed PMC pass and this run's kernel time, priced two ways: against the
            # microbenchmark's measured issue rate, and against the spec issue rate (256 CUs × 4 SIMDs
            # × ½ wave64-instruction per cycle) at the clock the chip held during the force pass
            va = pmc["valu_instr"] / avg_s
            roofline["valu"] = {"achieved": round(va / 1e9, 2), "peak": round(PEAK_VALU_WAVE_INSTR_PER_S / 1e9, 1),
                                "unit": "G wave-instr/s", "frac": round(va / PEAK_VALU_WAVE_INSTR_PER_S, 4),
                                "source": "rocprofv3 SQ_INSTS_VALU per launch (profiles/pmc_C3.json); peak measured by "
                                          "scripts/valu_peak.hip, long dispatches (profiles/r02_valu_peak_long.log)"}
            clk = load_clock()
            if "force_ghz" in clk:
                spec = 256 * 4 * 0.5 * clk["force_ghz"] * 1e9
                roofline["valu"].update({
                    "force_clock_ghz": round(clk["force_ghz"], 3),
                    "spec_peak_at_force_clock": round(spec / 1e9, 1),
                    "frac_of_spec_at_clock": round(va / spec, 4),
                    "clock_source": clk["force_src"]})
            if "micro_ghz" in clk:
                roofline["valu"]["microbench_clock_ghz"] = round(clk["micro_ghz"], 3)
                roofline["valu"]["microbench_frac_of_spec_at_its_clock"] = round(
                    PEAK_VALU_WAVE_INSTR_PER_S / (256 * 4 * 0.5 * clk["micro_ghz"] * 1e9), 4)

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
               "kernels_ms_per_step_mid_collapse": per_step_ms(mks, args.mid_steps)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "particle-steps/sec + ms/step at 1M particles; 1/2/4/8 MI355X scaling",
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
            "config": {"workload": runner.workload("strong" if args.strong else "weak"), "particles": n_total,
                       "particles_per_gpu": runner.local_particles(), "h_over_dx": 1.2,
                       "parallelism": f"slab{world}" if world > 1 else "single",
                       "transport": getattr(runner, "transport", "single" if world == 1 else "python")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
            "kernels_ms_per_step": per_step_ms(kstats, args.steps),
        }
        if mid:
            line.update(mid)
        print(json.dumps(line), flush=True)
    runner.close()
    if world > 1:
        dist.destroy_process_group()


class LibraryRankRunner:
    """One rank of the in-library decomposed step (sphhip.h sph_comm_init): rank 0 makes the RCCL
    unique id, torch.distributed hands its 128 bytes to every rank, and from then on sph_step runs the
    whole decomposed step (halos, re-sort, density, ρ halo overlapped with the interior force pass,
    re-balancing) with no host read per step."""
    transport = "library-rccl"

    def __init__(self, pkg, config, rank, world, device, profile, rebalance_every, strong):
        import torch
        import torch.distributed as dist
        from sph_test_amd import slab
        from sph_test_amd.context import comm_unique_id
        self.pkg, self.config, self.world = pkg, config, world
        self.scenario = pkg.config_scenario(config) if strong else slab.weak_scenario(config, world)
        self.params, self.dt = pkg.scenario_params(self.scenario)
        buf = torch.zeros(128, dtype=torch.uint8, device=torch.device("cuda", device))
        if rank == 0:
            buf.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
        if world > 1:
            dist.broadcast(buf, 0)
        torch.cuda.synchronize()
        self.ctx = pkg.Context(pkg.SPH_MODEL_WCSPH, self.scenario.dim, 1024, device=device, profile=bool(profile))
        if profile:
            self.ctx.set_profile_every(profile)
        self.ctx.comm_init(bytes(buf.cpu().numpy().tobytes()), world, rank)
        self.ctx.set_params(self.params)
        self.ctx.set_rebalance(rebalance_every)
        self.ctx.init_scenario(self.scenario)
        d = self.ctx.decomposition()
        self.n_total, self.cut = d.total, (d.cut.cx_lo, d.cut.cx_hi)

    def bind_stream(self, handle):
        self.ctx.set_stream(handle)

    def step(self, k):
        self.ctx.step(self.dt, k)

    def reset_stats(self):
        self.ctx.reset_kernel_stats()

    def kernel_stats(self):
        return self.ctx.kernel_stats()

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

    def kernel_stats(self):
        return self.sim.ctx.kernel_stats()

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

    def workload(self, scaling: str = "weak"):
        sc = self.sim.scenario
        kind = "sloshing" if sc.kind == self.pkg.SPH_SCENARIO_SLOSHING else "dam-break"
        return (f"{self.config}: {self.sim.n} particles, {sc.dim}D {kind}, column {sc.nx}x{sc.ny}x{sc.nz}, "
                f"tank {sc.tx}x{sc.ty}x{sc.tz} dx")

    def close(self):
        self.sim.close()


if __name__ == "__main__":
    main()
