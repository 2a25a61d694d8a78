"""The tiled passes' y-band workgroup schedule (schedule.hip) against their plain mapping (256 consecutive sorted
targets per workgroup, runs dealt to the XCDs): the schedule cuts the targets along y rows into other workgroups,
and no result may depend on the block partition, so whole runs must agree BIT FOR BIT. SPH_SCHED
(read at context creation): 0 plain, 1 (default) the schedule, rebuilt every 8 steps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_schedule_bit_identical(pkg, monkeypatch, cfg):
    sims = []
    for flag in ("0", "1"):
        monkeypatch.setenv("SPH_SCHED", flag)
        sims.append(pkg.SPHSim.from_config(cfg, profile=True))
    monkeypatch.delenv("SPH_SCHED")
    plain, band = sims
    try:
        for k in (1, 7, 12, 30):
            plain.step(k)
            band.step(k)
            for f in ("positions", "velocities", "density"):
                assert np.array_equal(getattr(plain, f)(), getattr(band, f)()), f"{cfg} {f} after {k} more steps"
        assert "schedule" in band.ctx.kernel_stats() and "schedule" not in plain.ctx.kernel_stats()
    finally:
        plain.close()
        band.close()
