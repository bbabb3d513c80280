#!/usr/bin/env python3
"""Join the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/fetch_calib with the
bytes each calibration kernel moves (every byte once, 256 MiB per kernel):

  python tools/fetch_calib.py FETCH_counter_collection.csv WRITE_counter_collection.csv

prints, per access pattern, FETCH_SIZE and WRITE_SIZE in bytes (the counters are in KiB) and
their ratio to the bytes moved: the factor by which a kernel's counter must be scaled for that
pattern (MI355X_MICROARCH.md: 1/2 for 16-B/lane coalesced streaming reads)."""
import csv
import json
import sys

MOVED = 1 << 28
MOVED_BY = {"c_rows168": (1 << 21) * 168}


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        out[name] = out.get(name, 0.0) + float(r["Counter_Value"])
    return out


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, 0.0) * 1024.0
        w = write.get(name, 0.0) * 1024.0
        moved = MOVED_BY.get(name, MOVED)
        res[name] = {"bytes_moved": moved, "fetch_bytes": f, "write_bytes": w,
                     "fetch_ratio": round(f / moved, 4), "write_ratio": round(w / moved, 4)}
        print(f"{name:14s} FETCH {f / 2**20:9.1f} MiB ({f / moved:6.3f} of moved)   "
              f"WRITE {w / 2**20:9.1f} MiB ({w / moved:6.3f})")
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
