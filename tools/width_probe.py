"""Grid-width accuracy probe: the grid k-sum (kspace_algo 2) at several ES kernel widths against
the exact fp64-MFMA k-sum (kspace_algo 0) on the same positions, at a BASELINE configuration's
initial positions (the ones the GPU tests use).  Prints one JSON line per width: max |dF|, RMS
|dF|, the atom of the largest deviation, dE, and max |d(dE/dq)|.

  python tools/width_probe.py [--config C3] [--widths 12,13,14]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "openmm-chargeflux_amd"))
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--widths", default="12,13,14")
    args = ap.parse_args()
    system, force, pos, box = ts.make(args.config)
    ka = HipCalcCoulForceKernel(kspace_algo=0).initialize(system, force)
    ea, fa = ka.execute_host(pos, box)
    da = ka.dedq()
    ka.destroy()
    for w in (int(x) for x in args.widths.split(",")):
        kg = HipCalcCoulForceKernel(kspace_algo=2, grid_width=w).initialize(system, force)
        eg, fg = kg.execute_host(pos, box)
        dg = kg.dedq()
        kg.destroy()
        df = np.abs(fg - fa)
        i = int(np.argmax(df.max(axis=1)))
        print(json.dumps({"config": args.config, "width": w, "max_abs_dF": float(df.max()),
                          "rms_dF": float(np.sqrt((df ** 2).mean())), "argmax_atom": i,
                          "F_at_argmax": [float(v) for v in fa[i]],
                          "dE": float(eg - ea), "max_abs_d_dedq": float(np.abs(dg - da).max())}), flush=True)


if __name__ == "__main__":
    main()
