#!/usr/bin/env python3
"""Per-step start offsets of a rocprofv3 kernel trace of bench.py: for every CoulForce step (from
one k_flux_terms to the next k_assemble_energy end) its duration, whether the cluster list was
rebuilt (k_cl_build > 5 us), the grid bin sort's duration and when the pair kernel and the spread
started.  Steps first..last (1-based) only; bench.py's passes run warmup, breakdown, timed, ...

usage: python tools/step_stats.py TRACE_DIR [first last]
"""
import csv, glob, sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
lo, hi = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1, 10 ** 9)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in csv.DictReader(open(f)))
ends = [i for i, e in enumerate(ev) if "k_assemble_energy" in e[2]]
rows = []
for n, (a, b) in enumerate(zip(ends[:-1], ends[1:]), start=2):
    if not lo <= n <= hi:
        continue
    seg = ev[a + 1:b + 1]
    first = lambda k: next((e for e in seg if k in e[2]), None)
    fl, p, sp, cb, gb = first("k_flux_terms"), first("k_pairs"), first("spread"), first("k_cl_build"), first("k_g_bin")
    if not (fl and p and sp):
        continue
    s0 = fl[0]
    rows.append(((seg[-1][1] - s0) / 1e3, bool(cb and cb[1] - cb[0] > 5000), (gb[1] - gb[0]) / 1e3 if gb else 0,
                 (p[0] - s0) / 1e3, (sp[0] - s0) / 1e3))
for n, r in enumerate(rows):
    print(f"step {n:3d} {r[0]:7.1f} us  rebuild {'Y' if r[1] else 'n'}  g_bin {r[2]:6.1f}  pairs@{r[3]:6.1f}  spread@{r[4]:6.1f}")
for tag, sel in (("rebuild", [r for r in rows if r[1]]), ("kept list", [r for r in rows if not r[1]])):
    if sel:
        print(f"{tag}: {len(sel)} steps, mean {sum(r[0] for r in sel) / len(sel):.1f} us, pairs before spread in "
              f"{sum(r[3] < r[4] for r in sel)}")
