"""Generates the golden fixtures in this directory from the oracle (oracle/cf_oracle.c,
the CPU restatement of ReferenceCoulKernels.cpp).  Inputs are the seeded synthetic
systems of openmmcoul.testsystems.  PARITY UNPINNED: the reference itself cannot be run
here (needs OpenMM), so these vectors are oracle outputs, pinned by the KATs of
tests/test_oracle.py.  Run:  python tests/golden/make_golden.py   (c3.npz: add --c3, ~6-10 min;
c3_codata2018.npz, the same at OpenMM 8.x's Coulomb constant: --c3-codata2018)"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd"), os.path.join(ROOT, "oracle")]

import hashlib  # noqa: E402
import time  # noqa: E402

from oracle import Oracle  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

C3_SUBSET = 2000      # atoms whose forces / dE/dq / charges are stored for C3
C3_SUBSET_SEED = 7


def c3_subset(n):
    """Seeded, sorted subset of atom indices stored in c3.npz (same call in the tests)."""
    return np.sort(np.random.default_rng(C3_SUBSET_SEED).choice(n, C3_SUBSET, replace=False))


ONE_4PI_EPS0_CODATA2018 = 138.93545764438198   # OpenMM 8.x (include/chargeflux.h)


def make_c3(one_4pi_eps0=0.0, name="c3.npz"):
    """Full-size C3 (96 000 atoms, kmax 31) through the oracle: ~6-10 min on one core.
    Positions are not stored (2.3 MB); testsystems.make("C3") regenerates them and the
    fixture keeps their SHA-256 so a test can assert it got the same input.  one_4pi_eps0:
    the Coulomb constant (0 = 138.935456, OpenMM 7.x; --c3-codata2018 writes c3_codata2018.npz)."""
    system, force, pos, box = ts.make("C3")
    t0 = time.time()
    r = Oracle(force, box, one_4pi_eps0=one_4pi_eps0).execute(pos, box)
    dt = time.time() - t0
    sub = c3_subset(len(pos))
    np.savez_compressed(os.path.join(HERE, name), pos_sha256=hashlib.sha256(pos.tobytes()).hexdigest(),
                        box=box, subset=sub, energy=r["energy"], terms=r["terms"], forces=r["forces"][sub],
                        charges=r["charges"][sub], dedq=r["dedq"][sub], charge_sum=r["charges"].sum(),
                        force_sum=r["forces"].sum(0), force_sq=(r["forces"] ** 2).sum(), oracle_s=dt,
                        one_4pi_eps0=one_4pi_eps0)
    print(name, len(pos), r["energy"], "%.1f s" % dt)

CASES = {
    "c1": lambda: ts.cluster_c1(),
    "box100": lambda: ts.water_box(100, cutoff=0.6, ewald_tol=1e-5, every_bond_angle=3),
    "c2": lambda: ts.make("C2"),
}

if __name__ == "__main__":
    if "--c3" in sys.argv:
        make_c3()
        sys.exit(0)
    if "--c3-codata2018" in sys.argv:
        make_c3(ONE_4PI_EPS0_CODATA2018, "c3_codata2018.npz")
        sys.exit(0)
    for name, make in CASES.items():
        system, force, pos, box = make()
        r = Oracle(force, box).execute(pos, box)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), pos=pos, box=np.zeros((3, 3)) if box is None else box,
                            energy=r["energy"], forces=r["forces"], charges=r["charges"], dedq=r["dedq"],
                            terms=r["terms"])
        print(name, len(pos), r["energy"])
