"""Bitwise A/B of two builds of libchargeflux_hip.so on fixed inputs (one process per build,
so the two libraries' exported symbols never interpose).

  python tools/ab_bits.py run LIB OUT.npz     evaluate the cases with LIB, store every output
  python tools/ab_bits.py cmp A.npz B.npz     report, per case, whether energy / forces / dE/dq
                                              are bit-identical (exit 1 if any differs)

Cases: C1 (no PBC), C2 on the exact and grid k-space paths, a 4000-water box in fp64 and
mixed precision with a neighbour skin over three moved steps (half list, kept lists).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd"), ROOT]


def cases():
    from openmmcoul import testsystems as ts
    yield "c1_exact", ts.cluster_c1(), dict(kspace_algo=0), 0.0, 1
    yield "c2_exact", ts.make("C2"), dict(kspace_algo=0), 0.0, 1
    yield "c2_grid", ts.make("C2"), dict(kspace_algo=2), 0.0, 1
    box4k = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    yield "w4k_grid_skin", box4k, dict(kspace_algo=2), 0.1, 3
    yield "w4k_mixed_skin", box4k, dict(kspace_algo=2, precision="mixed"), 0.1, 3


def run(lib, out):
    from openmmcoul import HipCalcCoulForceKernel, _cabi
    _cabi._lib = _cabi.load_library(lib)
    res = {}
    for name, (system, force, pos, box), kw, skin, steps in cases():
        k = HipCalcCoulForceKernel(**kw).initialize(system, force)
        if skin:
            k.set_neighbor_skin(skin)
        rng = np.random.default_rng(1)
        x = pos.copy()
        for s in range(steps):
            e, f = k.execute_host(x, box)
            res[f"{name}/{s}/e"] = np.array([e])
            res[f"{name}/{s}/f"] = f
            res[f"{name}/{s}/dq"] = k.dedq()
            x = x + rng.normal(scale=0.002, size=x.shape)
        k.destroy()
        print(name, "done", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for key in sorted(A.files):
        same = key in B.files and np.array_equal(A[key], B[key])
        bad += not same
        d = 0.0 if same or key not in B.files else np.abs(A[key] - B[key]).max()
        print(f"{key:28s} {'identical' if same else 'DIFFERS max|d|=%.3g' % d}")
    print("ALL BIT-IDENTICAL" if not bad else f"{bad} arrays differ")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
