"""C5 accuracy probe: max / RMS-relative force difference of mixed precision and of a narrower
grid against the fp64 W=14 grid path, to separate the fp32 pair error from the grid error."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd")]
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
# further arguments: prec:W combinations (default: the round-5 set)
combos = [(a.split(":")[0], int(a.split(":")[1])) for a in sys.argv[2:]] or \
    [("mixed", 14), ("mixed", 8), ("double", 8), ("double", 12)]
system, force, pos, box = ts.make(cfg)
pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream


def run(prec, w, algo=2):
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=algo, precision=prec, grid_width=w).initialize(system, force)
    k.set_neighbor_skin(0.2)
    f = torch.zeros_like(pt)
    e = torch.zeros(1, dtype=torch.float64, device="cuda")
    k.execute_device(pt, box, True, True, f, e)
    torch.cuda.synchronize()
    r = (e.item(), f.cpu().numpy(), k.energy_terms())
    # time: 10 evaluations on the kept list (same positions), one event pair around them
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.zeros_like(pt)
    a.record()
    for _ in range(10):
        k.execute_device(pt, box, True, True, g, e)
    b.record()
    torch.cuda.synchronize()
    k.destroy()
    return r + (a.elapsed_time(b) / 10,)


ref = run("double", 14)
for prec, w in combos:
    e, f, t, ms = run(prec, w)
    df = f - ref[1]
    i = np.unravel_index(np.abs(df).argmax(), df.shape)
    rms = np.sqrt((df ** 2).sum(1).mean() / (ref[1] ** 2).sum(1).mean())
    print(f"{cfg} {prec:6s} W={w:2d}: max|dF| {np.abs(df).max():.3e} at atom {i[0]} (|F| {np.abs(ref[1][i[0]]).max():.1f})"
          f"  rms_rel {rms:.2e}  dE {e - ref[0]:.3e}  dterms {np.array(t) - np.array(ref[2])}  {ms:.3f} ms/eval",
          flush=True)
