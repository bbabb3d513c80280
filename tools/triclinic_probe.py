"""Neighbour-list build and pair-kernel time of a C3-sized (96 000-atom) box, orthorhombic vs
reduced triclinic (same volume and density), list rebuilt on every evaluation (skin 0), fp64,
grid k-space: the per-phase HIP-event times of the library (cf_set_timing), averaged over
--evals evaluations after --warmup.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd")]

import torch  # noqa: E402

from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402


def run(system, force, pos, box, warmup, evals):
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2).initialize(system, force)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    f = torch.zeros_like(pt)
    e = torch.zeros(1, dtype=torch.float64, device="cuda")
    for _ in range(warmup):
        k.execute_device(pt, box, True, True, f, e)
    torch.cuda.synchronize()
    k.set_timing(True)
    for _ in range(evals):
        k.execute_device(pt, box, True, True, f, e)
    torch.cuda.synchronize()
    t = {p: v[0] / max(v[1], 1) for p, v in k.timing().items() if v[1]}
    fb = k.fallback_stats()
    k.destroy()
    out = {p: round(t.get(p, 0.0), 4) for p in ("cell_sort", "neighbor_list", "direct_pairs", "direct_excl")}
    out["fallbacks_half_evals_rows_reasons"] = list(fb)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waters", type=int, default=32000)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--evals", type=int, default=10)
    a = ap.parse_args()
    out = {"atoms": 3 * a.waters}
    s = ts.water_box(a.waters, cutoff=1.0, ewald_tol=1e-4)
    out["orthorhombic_ms"] = run(*s, a.warmup, a.evals)
    for shear in ((0.3, -0.25, 0.2), (0.5, -0.5, 0.5)):
        s = ts.triclinic_water_box(a.waters, cutoff=1.0, ewald_tol=1e-4, shear=shear)
        out[f"triclinic_{shear}_ms"] = run(*s, a.warmup, a.evals)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
