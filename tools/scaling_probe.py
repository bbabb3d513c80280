#!/usr/bin/env python3
"""Strong-scaling probe on ONE GPU: rank 0 of a W-way atom decomposition of C3, without the
collectives (the S(k) buffer is not reduced, so energies are not meaningful here).  Reports
per-step wall time, the library's per-phase GPU time and the host time to enqueue a step,
i.e. what each rank does at N = W minus RCCL.  Analysis tool, not the benchmark.

usage: python tools/scaling_probe.py [--worlds 1 2 4 8] [--steps 40] [--config C5 --precision mixed]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "openmm-chargeflux_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402
from openmmcoul.distributed import ShardedCoulKernel  # noqa: E402


def probe(system, force, pos_np, box, world, steps, skin, algo=2, timing=True, graph=False, precision="double",
          pair_list="auto"):
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    k = HipCalcCoulForceKernel(device=0, stream=stream, rank=0, world_size=world, kspace_algo=algo,
                               precision=precision, pair_list=pair_list).initialize(system, force)
    if skin > 0:
        k.set_neighbor_skin(skin)
    if graph:
        k.set_graph(True)   # begin / direct / end replayed as hipGraphs (cf_set_graph)
    kern = ShardedCoulKernel(system, force, dev, kernel=k)
    lo, hi = kern.lo, kern.hi
    n = len(pos_np)
    n_waters = force.getNumFluxWaters() + force.getNumFluxAngles()
    pos = torch.tensor(pos_np, dtype=torch.float64, device=dev)
    masses = torch.tensor([system._masses[i] for i in range(n)], dtype=torch.float64, device=dev).view(-1, 1)
    rng = np.random.default_rng(ts.SEED + 1)
    vel = torch.tensor(rng.normal(size=(n, 3)) * np.sqrt(bench.KB * 300.0 / masses.cpu().numpy()),
                       dtype=torch.float64, device=dev)
    frc = torch.zeros_like(pos)
    dt = 0.001
    md = bench.MDHarness(n_waters, lo, hi, dt, (1.0 / masses).contiguous(), stream)
    kern.execute(pos, box, frc, include_energy=True)
    first = [True]

    def step():   # the bench's step: one fused harness launch, then the force evaluation
        md.restrain_kick_drift(pos, vel, frc, first[0])
        first[0] = False
        kern.replicate_positions(pos)
        kern.execute(pos, box, frc, include_energy=True)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    k.set_timing(timing)
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    tm = k.timing()
    k.set_timing(False)
    gpu = {p: v[0] / steps for p, v in tm.items()}
    return {"world": world, "owned": hi - lo, "graph": graph, "pair_list": k.pair_list(), "ms_per_step": round(wall, 4),
            "host_enqueue_ms_per_step": round(host / steps * 1e3, 4),
            "lib_gpu_ms_per_step": round(sum(gpu.values()), 4),
            "phases": {p: round(v, 4) for p, v in gpu.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--neighbor-skin", type=float, default=0.1)
    ap.add_argument("--kspace-algo", type=int, default=2)
    ap.add_argument("--precision", default="double", help="double | mixed (C5)")
    ap.add_argument("--no-timing", action="store_true", help="no per-phase events (clean wall time)")
    ap.add_argument("--graph", action="store_true", help="replay the launches as hipGraphs (implies --no-timing)")
    ap.add_argument("--pair-list", default="auto", help="auto | cluster | atom_half | full (cf_options.pair_list)")
    args = ap.parse_args()
    system, force, pos_np, box = ts.make(args.config)
    for w in args.worlds:
        print(json.dumps(probe(system, force, pos_np, box, w, args.steps, args.neighbor_skin, args.kspace_algo,
                               not (args.no_timing or args.graph), args.graph, args.precision,
                               args.pair_list)), flush=True)


if __name__ == "__main__":
    main()
