"""SURVEY.md §8f-4 with §8f-1: the reference's shipped scene WITH the bonds its genome creates, on the GPU,
against a replay of the same controller + CellAdhesionManager host logic on the C oracle
(tests/oracle_backend.py). Model R is bit-exact per step, so the two runs take identical host decisions
(division timing, bond creation, zones, anchors, filtering) and every frame's read-back positions and
rotations, every frame's exported bond records and the final 84-byte particles must be equal bit for bit."""
import numpy as np
import pytest

from oracle_backend import oracle_backend
from test_adhesion_manager_cpu import _shipped_run

pytestmark = pytest.mark.gpu


def test_shipped_scene_with_bonds_matches_oracle_replay(pkg, oracle):
    gpu_ctl, gpu = _shipped_run(pkg, None)
    ref_ctl, ref = _shipped_run(pkg, oracle_backend(oracle))
    try:
        assert len(gpu) == len(ref) == 960
        for f, (g, r) in enumerate(zip(gpu, ref)):
            assert g[0] == r[0], f"frame {f + 1}: active {g[0]} vs {r[0]}"
            assert g[1] == r[1], f"frame {f + 1}: exported bonds differ"
            assert g[2] == r[2], f"frame {f + 1}: positions differ"
            assert g[3] == r[3], f"frame {f + 1}: rotations differ"
        assert gpu_ctl.GetParticles().tobytes() == ref_ctl.GetParticles().tobytes()
        assert len(gpu_ctl.adhesionManager.bonds) == 4
        assert gpu_ctl.context.stats().steps == 960
    finally:
        gpu_ctl.OnDestroy()
