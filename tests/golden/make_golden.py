"""Generates the golden fixtures in this directory from the oracle (oracle/cf_oracle.c,
the CPU restatement of ReferenceCoulKernels.cpp).  Inputs are the seeded synthetic
systems of openmmcoul.testsystems.  PARITY UNPINNED: the reference itself cannot be run
here (needs OpenMM), so these vectors are oracle outputs, pinned by the KATs of
tests/test_oracle.py.  Run:  python tests/golden/make_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd"), os.path.join(ROOT, "oracle")]

from oracle import Oracle  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

CASES = {
    "c1": lambda: ts.cluster_c1(),
    "box100": lambda: ts.water_box(100, cutoff=0.6, ewald_tol=1e-5, every_bond_angle=3),
    "c2": lambda: ts.make("C2"),
}

if __name__ == "__main__":
    for name, make in CASES.items():
        system, force, pos, box = make()
        r = Oracle(force, box).execute(pos, box)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), pos=pos, box=np.zeros((3, 3)) if box is None else box,
                            energy=r["energy"], forces=r["forces"], charges=r["charges"], dedq=r["dedq"],
                            terms=r["terms"])
        print(name, len(pos), r["energy"])
