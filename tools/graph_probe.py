"""Graph-replay time per step over many steps (C3, one rank): does replay slow down as it goes?
python tools/graph_probe.py [--handover event|memory] [--steps N] [--config C3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "openmm-chargeflux_amd")]
import torch  # noqa: E402

from openmmcoul import testsystems as ts  # noqa: E402
from openmmcoul.distributed import ShardedCoulKernel  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--handover", default="event")
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--config", default="C3")
ap.add_argument("--graph", type=int, default=1)
a = ap.parse_args()
system, force, pos_np, box = ts.make(a.config)
dev = torch.device("cuda", 0)
k = ShardedCoulKernel(system, force, 0, kspace_algo=2, neighbor_skin=0.15, handover=a.handover)
pos = torch.tensor(pos_np, dtype=torch.float64, device=dev)
frc = torch.zeros_like(pos)
for _ in range(5):
    k.execute(pos, box, frc, include_energy=True)
torch.cuda.synchronize()
if a.graph:
    k.kernel.set_graph(True)
t = time.perf_counter()
for s in range(1, a.steps + 1):
    frc.zero_()
    k.execute(pos, box, frc, include_energy=True)
    if s % 20 == 0:
        torch.cuda.synchronize()
        now = time.perf_counter()
        print(f"{a.handover} graph={a.graph} steps {s - 19}-{s}: {(now - t) / 20 * 1e3:.4f} ms/step "
              f"stats {k.kernel.graph_stats()}", flush=True)
        t = now
