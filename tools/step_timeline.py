#!/usr/bin/env python3
"""One CoulForce step of a rocprofv3 kernel trace, kernel by kernel: start (us from the previous
step's k_assemble_energy end), duration, queue, and the gap to the latest end so far (positive =
the device idle).  Used to find the fork / join latencies of the two-stream step.

usage: python tools/step_timeline.py TRACE_DIR
"""
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ","")[-28:], r["Queue_Id"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "k_assemble_energy" in e[2]]
lo, hi = ends[-3] + 1, ends[-2] + 1
t0 = ev[ends[-3]][1]
cur_e = t0
last = ev[ends[-3]][2]
for s, e, n, q in ev[lo:hi]:
    gap = s - cur_e
    print(f"{(s - t0)/1e3:7.1f} {(e - s)/1e3:6.1f} q{q} {n:30s} gap {gap/1e3:6.1f}" )
    cur_e = max(cur_e, e)
