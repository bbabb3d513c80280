"""The oracle reproduces the committed golden fixtures (tests/golden/make_golden.py) —
guards the restatement against drift; GPU tests compare the HIP path to the same data."""
import os

import numpy as np
import pytest

from oracle import Oracle
from tests.golden.make_golden import CASES

HERE = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_fixture(name):
    d = np.load(os.path.join(HERE, name + ".npz"))
    system, force, pos, box = CASES[name]()
    assert np.array_equal(pos, d["pos"])
    r = Oracle(force, box).execute(pos, box)
    assert r["energy"] == pytest.approx(float(d["energy"]), rel=1e-12)
    assert np.abs(r["forces"] - d["forces"]).max() < 1e-9
    assert np.abs(r["charges"] - d["charges"]).max() < 1e-14
    assert np.allclose(r["terms"], d["terms"], rtol=1e-12, atol=1e-9)
