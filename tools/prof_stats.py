#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as 'avg us  calls  name' (top N)."""
import csv
import glob
import sys

f = sys.argv[1]
if not f.endswith(".csv"):
    f = glob.glob(f + "/**/*kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in list(csv.DictReader(open(f)))[:n]:
    print(f"{float(r['AverageNs']) / 1e3:9.1f} us x{r['Calls']:>4} {float(r['TotalDurationNs']) / 1e3:10.1f} us  {r['Name'][:80]}")
