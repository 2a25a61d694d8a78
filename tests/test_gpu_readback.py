"""Asynchronous readback and render interop through the C ABI.

AsyncGPUReadback (ParticleSystemController.cs:1115-1159) returns the buffer as it was when the
request was made, later. Every check here is bit-exact against a synchronous read of the same
state (data movement only).
"""
import numpy as np
import pytest

from adhesion_cases import bonded_sphere

pytestmark = pytest.mark.gpu


def test_async_readback_is_the_requested_state(pkg):
    from sph_test_amd import _abi as A
    parts, _ = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 20000, seed=3)
    with pkg.Context(pkg.SPH_MODEL_CONTACT, 3, len(parts)) as ctx:
        ctx.upload_aos84(parts)
        with pytest.raises(A.SphError):
            ctx.readback_ready()                       # nothing requested yet
        ctx.step(0.01, 2)
        want_pos, want_rot, want_all = ctx.positions(), ctx.rotations(), ctx.download_aos84()
        ctx.request_readback(A.SPH_READBACK_POSITIONS | A.SPH_READBACK_ROTATIONS | A.SPH_READBACK_PARTICLES)
        ctx.step(0.01, 5)                              # keeps stepping while the copy is in flight
        pos = ctx.readback_get(A.SPH_READBACK_POSITIONS)
        assert ctx.readback_ready()
        assert pos.tobytes() == want_pos.tobytes()
        assert ctx.readback_get(A.SPH_READBACK_ROTATIONS).tobytes() == want_rot.tobytes()
        assert ctx.readback_get(A.SPH_READBACK_PARTICLES).tobytes() == want_all.tobytes()
        assert ctx.positions().tobytes() != want_pos.tobytes()
        # a new request replaces the old one
        ctx.request_readback(A.SPH_READBACK_POSITIONS)
        assert ctx.readback_get(A.SPH_READBACK_POSITIONS).tobytes() == ctx.positions().tobytes()
        with pytest.raises(A.SphError):
            ctx.readback_get(A.SPH_READBACK_ROTATIONS)  # not part of this request


def test_async_readback_model_s(pkg):
    from sph_test_amd import _abi as A
    sim = pkg.SPHSim.from_config("C2")
    sim.step(3)
    want = sim.positions()
    sim.ctx.request_readback(A.SPH_READBACK_POSITIONS)
    sim.step(2)
    assert sim.ctx.readback_get(A.SPH_READBACK_POSITIONS).tobytes() == want.tobytes()
    with pytest.raises(A.SphError):
        sim.ctx.request_readback(A.SPH_READBACK_ROTATIONS)
    sim.close()


def test_export_aos84_device_and_draw_args(pkg):
    import torch
    parts, _ = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 5000, seed=4)
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    ctl.Start(parts)
    ctl.activeParticleCount = 4000
    ctl.Update(0.01)
    ctx = ctl.context
    buf = torch.zeros(len(parts) * 84, dtype=torch.uint8, device="cuda")
    args = torch.tensor([36, 0, 0, 0, 0], dtype=torch.int32, device="cuda")
    ctx.export_aos84_device(buf.data_ptr(), len(parts))
    ctx.write_draw_args(args.data_ptr())
    ctx.synchronize()
    assert buf.cpu().numpy().tobytes() == ctl.GetParticles().tobytes()
    assert args.cpu().tolist() == [36, 4000, 0, 0, 0]
    ctl.OnDestroy()


def test_controller_async_readback(pkg):
    """immediateReadback = False: the CPU arrays lag one request behind and match that state."""
    parts, _ = bonded_sphere(pkg.PARTICLE84, pkg.ADHESION84, 3000, seed=5)
    ctl = pkg.ParticleSystemController(particleCount=len(parts))
    ctl.Start(parts)
    ctl.immediateReadback = False
    ctl.Update(0.01)
    after1 = ctl.context.positions()
    ctl.Update(0.01)                                   # delivers the request made after frame 1
    assert ctl.CpuParticlePositions[: len(parts)].tobytes() == after1.tobytes()
    ctl.OnDestroy()


def test_readback_and_export_match_the_oracle(pkg, oracle):
    """The delivery paths against the CPU oracle, not against another GPU read: after one Model R step
    (SimulateParticles.compute:211-408, bit-exact, test_gpu_parity.py), the asynchronous readback
    (ParticleSystemController.cs:1115-1159: particles, positions, rotations) and the device AoS-84 export
    (the renderer's particleBuffer, InstancedParticles.shader:27-44) hold the oracle's step output byte
    for byte, with drag and inactive particles (export covers the whole buffer, as the reference's)."""
    import torch
    from sph_test_amd import _abi as A
    from test_gpu_parity import random_sphere
    n, act = 6000, 5000
    parts = random_sphere(pkg.PARTICLE84, n, seed=17)
    ctl = pkg.ParticleSystemController(particleCount=n)
    ctl.Start(parts)
    ctl.activeParticleCount = act
    ctl.drag.selectedID, ctl.drag.targetPosition, ctl.drag.strength = 9, (1.0, 2.0, -3.0), 80.0
    ctl.Update(0.01)
    cp = oracle.contact_params(0.01, drag_id=9, drag_target=(1.0, 2.0, -3.0), drag_strength=80.0)
    ref_act, _ = oracle.contact_step(cp, parts[:act].view(oracle.PARTICLE84))
    ref = parts.copy()
    ref[:act] = ref_act.view(pkg.PARTICLE84)
    ctx = ctl.context
    ctx.request_readback(A.SPH_READBACK_PARTICLES | A.SPH_READBACK_POSITIONS | A.SPH_READBACK_ROTATIONS)
    got = ctx.readback_get(A.SPH_READBACK_PARTICLES)
    assert got.tobytes() == ref.tobytes()
    assert ctx.readback_get(A.SPH_READBACK_POSITIONS).tobytes() == np.ascontiguousarray(ref["position"]).tobytes()
    assert ctx.readback_get(A.SPH_READBACK_ROTATIONS).tobytes() == np.ascontiguousarray(ref["rotation"]).tobytes()
    buf = torch.zeros(n * 84, dtype=torch.uint8, device="cuda")
    ctx.export_aos84_device(buf.data_ptr(), n)
    ctx.synchronize()
    assert buf.cpu().numpy().tobytes() == ref.tobytes()
    ctl.OnDestroy()
