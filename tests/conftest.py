import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as GE  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def pkg():
    return GE.load_package()


@pytest.fixture(scope="session")
def oracle():
    O = GE.load_oracle()
    O.lib()
    return O


def oracle_sph_params(O, p, dim):
    """The CPU oracle's Model S params from the library's sph_params (same floats)."""
    return O.sph_params(dim, p.dx, p.h, p.rho0, p.c0, p.alpha, p.xsph_eps, tuple(p.gravity), tuple(p.box),
                        p.wall_restitution, p.forcing_amp, p.forcing_freq)
