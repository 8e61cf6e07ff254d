#!/usr/bin/env python3
"""Critical-path view of a rocprofv3 kernel trace (tools/trace_session.sh).

Windows are cut at the marker kernel (default k_input_prep8: two launches per
fusion forward, DWI and DCE). Per window: wall time, summed kernel time, the
union of busy intervals (so idle = wall - union), the busy time per queue, and
the kernels sorted by time. ``--split NAME`` reports the part of each window
after the last launch of NAME separately (e.g. the last encoder kernel).

    python tools/timeline.py gpurun_out/r03f/step/.../step_kernel_trace.csv [--last 3] [--top 25]
"""
import argparse
import collections
import csv
import gzip
import re


def load(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in rows:
        out.append(dict(name=r["Kernel_Name"], s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]),
                        q=r.get("Queue_Id", r.get("Stream_Id", "?")), grid=r.get("Grid_Size_X", r.get("Grid_Size", "?"))))
    out.sort(key=lambda k: k["s"])
    return out


def short(n):
    n = n.replace("void ", "")
    n = re.sub(r"\(.*$", "", n)
    return n[:90]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def report(ks, title, top):
    if not ks:
        return
    t0, t1 = min(k["s"] for k in ks), max(k["e"] for k in ks)
    wall = (t1 - t0) / 1e3
    summ = sum(k["e"] - k["s"] for k in ks) / 1e3
    uni = union([(k["s"], k["e"]) for k in ks]) / 1e3
    print(f"== {title}: {len(ks)} kernels, wall {wall:.1f} us, kernel sum {summ:.1f} us, busy union {uni:.1f} us, "
          f"idle {wall - uni:.1f} us")
    byq = collections.defaultdict(list)
    for k in ks:
        byq[k["q"]].append((k["s"], k["e"]))
    for q, iv in sorted(byq.items()):
        print(f"   queue {q}: {len(iv)} kernels, busy {union(iv) / 1e3:.1f} us")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for k in ks:
        a = agg[short(k["name"])]
        a[0] += 1
        a[1] += (k["e"] - k["s"]) / 1e3
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"   {t:8.1f} us {c:4d}x {t / c:7.1f} us  {n}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_input_prep8")
    ap.add_argument("--per", type=int, default=2, help="marker launches per window")
    ap.add_argument("--last", type=int, default=2)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--split", default=None)
    ap.add_argument("--seq", action="store_true", help="print the window's kernels in start order")
    a = ap.parse_args()
    ks = load(a.trace)
    marks = [i for i, k in enumerate(ks) if a.marker in k["name"]]
    starts = [ks[marks[j]]["s"] for j in range(0, len(marks), a.per)]
    wins = []
    for j, s in enumerate(starts):
        e = starts[j + 1] if j + 1 < len(starts) else None
        wins.append([k for k in ks if k["s"] >= s - 2000 and (e is None or k["s"] < e - 2000)])
    print(f"{len(ks)} kernels, {len(wins)} windows")
    for w in wins[-a.last - 1:-1] if len(wins) > a.last else wins:
        if a.split:
            idx = [i for i, k in enumerate(w) if a.split in k["name"]]
            if idx:
                cut = max(w[i]["e"] for i in idx)
                report([k for k in w if k["e"] <= cut], "until split", a.top)
                report([k for k in w if k["e"] > cut], "after split", a.top)
                if a.seq:
                    t0 = w[0]["s"]
                    for k in w:
                        if k["e"] > cut:
                            print(f"   {(k['s'] - t0) / 1e3:8.1f} +{(k['e'] - k['s']) / 1e3:6.1f} q{k['q']} {short(k['name'])}")
                continue
        report(w, "window", a.top)
        if a.seq:
            t0 = w[0]["s"]
            for k in w:
                print(f"   {(k['s'] - t0) / 1e3:8.1f} +{(k['e'] - k['s']) / 1e3:6.1f} q{k['q']} {short(k['name'])}")


if __name__ == "__main__":
    main()
