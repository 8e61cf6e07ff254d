#!/usr/bin/env python3
"""Per-launch HBM traffic of the conv-forward kernels from two rocprofv3
--pmc passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch). gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per 128-B request
of wide streaming reads -> x2. WRITE_SIZE is exact for 16-B/lane stores.

    python tools/pmc_traffic.py gpurun_out/pmc1 [--match REGEX]
"""
import argparse
import os
import csv
import json
import re


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default=r"k_conv_fwd_ps|k_conv_fwd_pp|k_conv_fwd_sq|k_conv_fwd_wide|k_conv_fwd_buf|k_conv_stem|k_conv_igemm<unsigned short, false")
    ap.add_argument("--json", default="")
    ap.add_argument("--latest", default="", help="also point profiles/pmc_latest.json's KEY at --json "
                    "(bench.py reads the pointer: 'traffic' for the conv forward, 'traffic_wgrad', ...)")
    ap.add_argument("--count", default="", help="launches = dispatches matching this regex (default: every "
                    "matched dispatch); e.g. the weight-gradient kernel of a wgrad + split-reduce pair")
    a = ap.parse_args()
    fe = load(f"{a.dir}/FETCH_SIZE/run_counter_collection.csv")
    wr = load(f"{a.dir}/WRITE_SIZE/run_counter_collection.csv")
    rx = re.compile(a.match)
    f_k = [v for _, n, v in fe if rx.search(n)]
    w_k = [v for _, n, v in wr if rx.search(n)]
    if len(f_k) != len(w_k):
        raise SystemExit(f"the two passes matched {len(f_k)} / {len(w_k)} dispatches")
    n = len([1 for _, nm, _ in fe if rx.search(nm) and re.search(a.count, nm)]) if a.count else len(f_k)
    fetch = 2.0 * sum(f_k) * 1024 / n
    write = sum(w_k) * 1024 / n
    print(f"launches {n}: fetch {fetch / 1e6:.2f} MB (x2 corrected), write {write / 1e6:.2f} MB, "
          f"traffic {(fetch + write) / 1e6:.2f} MB per launch")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"kernels": a.match, "launches": n, "fetch_mb_per_launch": round(fetch / 1e6, 2),
                       "write_mb_per_launch": round(write / 1e6, 2),
                       "traffic_mb_per_launch": round((fetch + write) / 1e6, 2),
                       "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as is"}, f, indent=1)
        if a.latest:
            set_latest(a.latest, a.json)


def set_latest(key, path):
    """Point profiles/pmc_latest.json's key at a summary (path relative to the repo root)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ptr = os.path.join(root, "profiles", "pmc_latest.json")
    try:
        with open(ptr) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    d[key] = os.path.relpath(os.path.abspath(path), root)
    with open(ptr, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
