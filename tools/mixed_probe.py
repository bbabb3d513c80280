"""Per-term error of the mixed-precision path and the narrow grid kernel at a given config
(energy terms and RMS relative force error against the fp64 exact k-sum)."""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "openmm-chargeflux_amd")]

import numpy as np  # noqa: E402

from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
system, force, pos, box = ts.make(cfg)
runs = [("fp64 exact", dict(kspace_algo=0)), ("fp64 grid W14", dict(kspace_algo=2)),
        ("fp64 grid W8", dict(kspace_algo=2, grid_width=8)), ("mixed exact", dict(kspace_algo=0, precision="mixed")),
        ("mixed grid W8", dict(kspace_algo=2, precision="mixed"))]
ref = None
for name, kw in runs:
    k = HipCalcCoulForceKernel(**kw).initialize(system, force)
    e, f = k.execute_host(pos, box)
    t = k.energy_terms()
    if ref is None:
        ref = (e, f, t)
        print(f"{name:16s} E {e:.6f} terms {t}")
    else:
        d = f - ref[1]
        rms = np.sqrt(np.mean(np.sum(d * d, 1)) / np.mean(np.sum(ref[1] ** 2, 1)))
        print(f"{name:16s} dE {e - ref[0]:+.4e} dterms {t - ref[2]} rms_rel {rms:.2e} max|dF| {np.abs(d).max():.2e}")
    k.destroy()
