#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into per-kernel averages (profiles/*.json).

usage: pmc_summary.py OUT.json KERNEL_TRACE.csv [COUNTER_COLLECTION.csv ...]

Per kernel: launches, average duration (kernel trace) and, for every PMC counter,
the average value per launch.  HBM bytes: FETCH_SIZE and WRITE_SIZE are in KiB.  FETCH_SIZE
counts 64-B memory requests; on gfx950 it reports half the bytes of a 16-B/lane coalesced
streaming read (MI355X_MICROARCH.md §HBM) and exactly the bytes of 64-B pieces, wave-uniform
64-B scalar loads and scattered gathers (whose 64-B granules are the real traffic), per the
calibration kernels of tools/fetch_calib.hip (profiles/r03_fetch_calibration.json).  So
hbm_read_bytes_est = fetch_factor * 1024 * FETCH_SIZE with the factor of the kernel's dominant
read pattern (FETCH_FACTOR below; 2, the upper estimate, for kernels not listed), and
hbm_write_bytes = 1024 * WRITE_SIZE (calibrated exact for 16-B and 64-B stores).
"""

# kernel-name prefix -> FETCH_SIZE factor of its dominant read pattern (tools/fetch_calib.hip)
FETCH_FACTOR = {
    "cf::k_pairs_half": 2.0,       # the neighbour list: 16-B chunks, consecutive rows per lane (streaming)
    "cf::k_pairs<": 2.0,
    "cf::k_pairs_cq": 2.0,         # the cluster-pair list: 16 consecutive 8-B entries per wave (streaming; upper estimate)
    "cf::k_g_spread_tile": 1.0,    # 64-B window pieces + wave-uniform 64-B x windows (c_seg64, c_scalar64)
    "cf::k_g_spread_mfma": 1.0,    # 64-B window pieces read as 16-B lanes (c_seg64)
    "cf::k_excl": 1.0,             # 32-B window-sum gathers (c_gather32: 64-B granules = real traffic)
    "cf::k_g_interp": 1.17,        # 168-B halo row runs (c_rows168: FETCH = 0.853 of the bytes)
}
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
            e["fetch_factor"] = next((f for p, f in FETCH_FACTOR.items() if k.startswith(p)), 2.0)
            e["hbm_read_bytes_est"] = e["fetch_factor"] * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = 1024 * e["WRITE_SIZE"]
        res[k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda x: -x[1]["avg_us"]):
        print(f"{k:32s} {e['avg_us']:10.1f} us  " + "  ".join(f"{c}={v:.4g}" for c, v in e.items()
                                                              if c not in ("launches", "avg_us")))


if __name__ == "__main__":
    main()
