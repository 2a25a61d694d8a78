"""The oracle against its committed fixtures (tests/golden/, made by make_golden.py).
Bit-exact: same C source, -ffp-contract=off, one thread, same glibc image."""
from pathlib import Path

import numpy as np
import pytest

G = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("name", ["contact_n64_s1", "contact_n64_s10", "contact_n4096_s1"])
def test_contact_golden(oracle, name):
    import sys
    sys.path.insert(0, str(G))
    from make_golden import contact_case
    d = np.load(G / f"{name}.npz")
    n, steps = (int(x[1:]) for x in name.split("_")[1:])
    inp, out, tq = contact_case(n, steps)
    assert inp.view(np.uint8).tobytes() == d["input"].tobytes()
    assert out.view(np.uint8).tobytes() == d["output"].tobytes()
    assert np.array_equal(tq, d["torque"])


@pytest.mark.parametrize("steps", [1, 10])
def test_wcsph_golden(oracle, steps):
    import sys
    sys.path.insert(0, str(G))
    from make_golden import sph_case
    d = np.load(G / f"wcsph_c1_s{steps}.npz")
    x0, x, v, rho, dt, c0 = sph_case(steps)
    assert np.array_equal(x0, d["x0"])
    assert np.array_equal(x, d["x"]) and np.array_equal(v, d["v"]) and np.array_equal(rho, d["rho"])


@pytest.mark.parametrize("name", ["adhesion_n512_s1", "adhesion_n512_s5"])
def test_adhesion_golden(oracle, name):
    import sys
    sys.path.insert(0, str(G))
    from make_golden import adhesion_case
    d = np.load(G / f"{name}.npz")
    n, steps = (int(x[1:]) for x in name.split("_")[1:])
    inp, conns, out, tq, terms = adhesion_case(n, steps)
    assert inp.view(np.uint8).tobytes() == d["input"].tobytes()
    assert conns.view(np.uint8).tobytes() == d["conns"].tobytes()
    assert out.view(np.uint8).tobytes() == d["output"].tobytes()
    assert np.array_equal(tq, d["torque"]) and np.array_equal(terms, d["terms"])
