#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into per-kernel averages (profiles/*.json).

usage: pmc_summary.py OUT.json KERNEL_TRACE.csv [COUNTER_COLLECTION.csv ...]

Per kernel: launches, average duration (kernel trace) and, for every PMC counter,
the average value per launch.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide streaming
read, so hbm_read_bytes = 2 * 1024 * FETCH_SIZE (upper estimate; the exact factor depends
on access width), hbm_write_bytes = 1024 * WRITE_SIZE.
"""
import collections
import csv
import json
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    out, trace, *pmcs = sys.argv[1:]
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in pmcs:
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(p)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            ctr[names[d]][c].append(v)
    res = {}
    for k, v in dur.items():
        if not k.startswith("cf::"):
            continue
        e = {"launches": len(v), "avg_us": sum(v) / len(v) / 1e3}
        for c, vals in ctr.get(k, {}).items():
            e[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes_est"] = 2 * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = 1024 * e["WRITE_SIZE"]
        res[k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda x: -x[1]["avg_us"]):
        print(f"{k:32s} {e['avg_us']:10.1f} us  " + "  ".join(f"{c}={v:.4g}" for c, v in e.items()
                                                              if c not in ("launches", "avg_us")))


if __name__ == "__main__":
    main()
