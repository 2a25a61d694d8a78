"""Slab decomposition (SPEC_SPH.md §3) on CPU: SlabRunner over gloo, world sizes 2 and 3,
with the oracle-backed CPU backend, against the single-domain oracle step."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
STEPS = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scenario(pkg):
    return pkg.make_scenario(0, 3, 24, 16, 8, 60, 24, 8, dx=0.01, seed=4321)


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    import torch.distributed as dist
    import __graft_entry__ as GE
    from slab_cpu_backend import CpuSlabBackend
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = GE.load_package()
    O = GE.load_oracle()
    from sph_test_amd import slab
    sc = _scenario(pkg)
    p, _ = pkg.scenario_params(sc)
    op = O.sph_params(3, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                      p.wall_restitution, p.forcing_amp, p.forcing_freq)
    runner = slab.SlabRunner("C3", rank, world, scenario=sc,
                             backend=lambda cut: CpuSlabBackend(O, op, sc, cut, jitter_frac=sc.jitter))
    runner.step(STEPS)
    np.save(os.path.join(outdir, f"rank{rank}.npy"), runner.owned())
    np.save(os.path.join(outdir, f"cuts{rank}.npy"), np.array(runner.cuts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_decomposition_matches_single_domain(pkg, oracle, tmp_path, world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=300)
        assert pr.exitcode == 0, f"rank exited with {pr.exitcode}"
    parts = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    cuts = np.load(tmp_path / "cuts0.npy")
    assert len(cuts) == world and all(c[0] < c[1] for c in cuts)
    rec = np.concatenate(parts)
    ids = rec[:, 6].view(np.int32)
    sc = _scenario(pkg)
    n = sc.nx * sc.ny * sc.nz
    # every particle owned by exactly one rank
    assert np.array_equal(np.sort(ids), np.arange(n))
    assert all(len(p) > 0 for p in parts)
    # single-domain reference
    p, dt = pkg.scenario_params(sc)
    op = oracle.sph_params(3, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                           p.wall_restitution, p.forcing_amp, p.forcing_freq)
    x = oracle.lattice(3, sc.nx, sc.ny, sc.nz, sc.dx, seed=sc.seed, jitter_frac=sc.jitter)
    v = np.zeros_like(x)
    oid = np.arange(n, dtype=np.int32)
    t = 0.0
    for _ in range(STEPS):
        x, v, oid, rho, _, _ = oracle.sph_step(op, x, v, oid, dt, np.float32(t))
        t += dt
    ref_x = x[np.argsort(oid)]
    ref_v = v[np.argsort(oid)]
    order = np.argsort(ids)
    got_x, got_v = rec[order, 0:3], rec[order, 3:6]
    # identical physics; only the summation order of key ties differs
    np.testing.assert_allclose(got_x, ref_x, rtol=0, atol=2e-6)
    np.testing.assert_allclose(got_v, ref_v, rtol=1e-3, atol=2e-3)
