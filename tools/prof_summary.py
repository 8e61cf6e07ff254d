#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (csv ``*_kernel_stats.csv`` /
``*_kernel_trace.csv`` or the rocpd ``*_results.db``) into a per-kernel
table: calls, total/avg/min/max duration (ns) and share of GPU time.

    python tools/prof_summary.py gpurun_out/r1a/prof [--steps N] > profiles/r01_kernel_stats.csv
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    for name, s, e in c.execute("select name, start, end from kernels"):
        yield name, e - s


def rows_from_trace(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=float, default=0.0, help="divide totals by this many step-equivalents")
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        cand = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True) or \
            glob.glob(os.path.join(p, "**", "*results.db"), recursive=True)
        if not cand:
            sys.exit("no kernel trace under " + p)
        p = cand[0]
    it = rows_from_db(p) if p.endswith(".db") else rows_from_trace(p)
    agg = collections.defaultdict(list)
    for n, d in it:
        agg[n].append(d)
    tot = sum(sum(v) for v in agg.values())
    w = csv.writer(sys.stdout)
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"]
    if a.steps:
        hdr.append("UsPerStep")
    w.writerow(hdr)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        row = [n, len(v), sum(v), round(sum(v) / len(v), 1), min(v), max(v), round(100.0 * sum(v) / tot, 3)]
        if a.steps:
            row.append(round(sum(v) / a.steps / 1e3, 1))
        w.writerow(row)


if __name__ == "__main__":
    main()
