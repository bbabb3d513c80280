#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 kernel trace (run_kernel_trace.csv): for the dispatches of
the last N CoulForce steps (a step = one k_assemble_energy), the wall span per step, the busy time
(union of kernel intervals over all queues), the sum of kernel durations (> busy when two streams
overlap), and the idle gaps.  Used to compare eager launches with hipGraph replay.

usage: python tools/trace_gaps.py TRACE_CSV [--steps N]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    ends = [i for i, e in enumerate(ev) if "k_assemble_energy" in e[2]]
    if len(ends) < args.steps + 1:
        raise SystemExit("not enough steps in the trace")
    lo = ends[-args.steps - 1] + 1
    hi = ends[-1] + 1
    sel = ev[lo:hi]
    t0, t1 = ev[ends[-args.steps - 1]][1], ev[ends[-1]][1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ksum = sum(e - s for s, e, _, _ in sel)
    queues = sorted({q for _, _, _, q in sel})
    n = args.steps
    print(f"steps {n}: span {((t1 - t0) / n) / 1e3:.1f} us/step, busy {busy / n / 1e3:.1f}, "
          f"kernel sum {ksum / n / 1e3:.1f}, idle {((t1 - t0) - busy) / n / 1e3:.1f}, "
          f"dispatches/step {len(sel) / n:.1f}, queues {queues}")


if __name__ == "__main__":
    main()
