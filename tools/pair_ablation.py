#!/usr/bin/env python3
"""Kernel-time probe for direct-space A/B and ablation builds: C3 (or another config), fixed
positions, the neighbour list built once and kept (skin), N force evaluations on one stream
(CF_OVERLAP=0 recommended) -- run under rocprofv3 --kernel-trace --stats.  Ablation builds give
wrong numbers by construction; this script only times them (no MD, so nothing blows up).

usage: python tools/pair_ablation.py [--config C3] [--evals 20] [--skin 0.15] [--precision double]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "openmm-chargeflux_amd")]

import torch  # noqa: E402

from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--evals", type=int, default=20)
    ap.add_argument("--skin", type=float, default=0.15)
    ap.add_argument("--precision", default="double")
    args = ap.parse_args()
    system, force, pos, box = ts.make(args.config)
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=2, precision=args.precision).initialize(system, force)
    k.set_neighbor_skin(args.skin)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    f = torch.zeros_like(pt)
    e = torch.zeros(1, dtype=torch.float64, device="cuda")
    for _ in range(args.evals):
        k.execute_device(pt, box, True, True, f, e)
    torch.cuda.synchronize()
    print("done", args.evals, "evaluations, builds/evals", k.neighbor_stats())


if __name__ == "__main__":
    main()
