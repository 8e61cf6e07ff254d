#!/usr/bin/env python3
"""Average each PMC counter per kernel name over the dispatches in a
rocprofv3 --pmc counter_collection.csv (usage: pmc_summary.py DIR)."""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
if not f:
    sys.exit("no counter_collection.csv under " + sys.argv[1])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} n={len(v):4d} avg={sum(v) / len(v):14.1f}")
