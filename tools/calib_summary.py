#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration summary (tools/calib/fetch_calib.hip):
per kernel, counter bytes per launch / the 1 GiB of distinct bytes each launch
touches.  usage: calib_summary.py <dir with p1/ (FETCH_SIZE) p2/ (WRITE_SIZE)> [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
GiB = float(1 << 30)
res = {}
for (k, c), v in sorted(agg.items()):
    kib = sum(v) / len(v)                      # FETCH_SIZE / WRITE_SIZE are in KiB
    res.setdefault(k, {})[c + "_over_distinct"] = round(kib * 1024 / GiB, 4)
out = {"distinct_bytes_per_launch": int(GiB), "ratio_counter_bytes_to_distinct_bytes": res,
       "note": "gfx950, rocprofv3 --pmc per counter in its own pass; 1 GiB buffer (4x the Infinity Cache)"}
s = json.dumps(out, indent=1)
print(s)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(s + "\n")
