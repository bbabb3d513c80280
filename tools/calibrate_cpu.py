"""Calibrate the CPU baseline (the oracle, oracle/cf_oracle.c, a serial restatement of
ReferenceCoulKernels.cpp) against the compiled reference kernel's timings of BASELINE.md §2
(g++ 11 -O2, one core of this image's build host, Intel Xeon; the reference's neighbour list
there was a brute-force O(N^2) stand-in whose share is listed separately).

For each BASELINE.md row: the oracle's execute(forces + energy) time on the same kind of box
(33.43 waters/nm^3, FluxWater on every molecule, rc 1.0 nm), median of R runs, against the
reference's total and against the reference's total minus its O(N^2) neighbour-list share
(OpenMM's own voxel hash is O(N), like the oracle's cell list).  Writes
profiles/cpu_calibration.json, which bench.py quotes in cpu_baseline.sample.

usage: python tools/calibrate_cpu.py   (in this container; ~1 min)
"""
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd"), os.path.join(ROOT, "oracle")]
from oracle import Oracle  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

# (atoms, tol, kmax, reference s/eval (range lo, hi), stub O(N^2) list share s)
ROWS = [(3000, 5e-3, 5, (0.258, 0.258), 0.106),
        (3000, 1e-3, 7, (0.36, 0.47), 0.11),
        (3000, 1e-4, 9, (0.632, 0.632), 0.120),
        (6000, 1e-4, 13, (3.26, 3.26), 0.42),
        (12000, 1e-4, 15, (10.6, 10.6), 1.60)]


def host():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    rows = []
    for n, tol, kmax, (rlo, rhi), nl in ROWS:
        system, force, pos, box = ts.water_box(n // 3, cutoff=1.0, ewald_tol=tol, every_bond_angle=0)
        o = Oracle(force, box)
        assert o.ewald()[1] == (kmax,) * 3, (n, tol, o.ewald())
        reps = 5 if n <= 3000 else 3
        ts_ = []
        for _ in range(reps):
            t0 = time.perf_counter()
            o.execute(pos, box)
            ts_.append(time.perf_counter() - t0)
        t = float(np.median(ts_))
        ref = 0.5 * (rlo + rhi)
        rows.append({"atoms": n, "tol": tol, "kmax": kmax, "oracle_s": round(t, 4), "reference_s": [rlo, rhi],
                     "reference_stub_nlist_s": nl, "ratio_vs_reference": round(t / ref, 3),
                     "ratio_vs_reference_without_stub_nlist": round(t / (ref - nl), 3)})
        print(rows[-1], flush=True)
    r1 = [r["ratio_vs_reference_without_stub_nlist"] for r in rows]
    r0 = [r["ratio_vs_reference"] for r in rows]
    summ = (f"{min(r1):.2f}-{max(r1):.2f} against the reference without its O(N^2) stand-in neighbour list "
            f"({min(r0):.2f}-{max(r0):.2f} against its total)")
    out = {"host": host(), "cores_used": 1, "rows": rows, "ratio_summary": summ,
           "method": "tools/calibrate_cpu.py: median oracle execute() vs BASELINE.md §2 compiled-reference timings"}
    json.dump(out, open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w"), indent=1)
    print(summ)


if __name__ == "__main__":
    main()
