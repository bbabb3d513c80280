#!/usr/bin/env python3
"""One CoulForce step of a rocprofv3 kernel trace, kernel by kernel: start (us from the previous
step's k_assemble_energy end), duration, queue, and the gap to the latest end so far (positive =
the device idle).  Used to find the fork / join latencies of the two-stream step.

usage: python tools/step_timeline.py TRACE_DIR [EVAL]
EVAL: index of the evaluation (k_assemble_energy launch) to show, default -2 (the graph pass of the
bench command); with `bench.py --steps 5 --warmup 2` evaluations 8..12 are the timed region
(1 initial + 2 warm-up + 5 breakdown before it).
"""
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ","")[-28:], r["Queue_Id"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "k_assemble_energy" in e[2]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -2
k = k if k >= 0 else len(ends) + k
lo, hi = ends[k - 1] + 1, ends[k] + 1
t0 = ev[ends[k - 1]][1]
cur_e = t0
for s, e, n, q in ev[lo:hi]:
    gap = s - cur_e
    print(f"{(s - t0)/1e3:7.1f} {(e - s)/1e3:6.1f} q{q} {n:30s} gap {gap/1e3:6.1f}" )
    cur_e = max(cur_e, e)
