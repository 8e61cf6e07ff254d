#!/usr/bin/env python3
"""Do the DWI and DCE encoder streams overlap in the captured mode-A step?
 rocprofv3's kernel trace serialises a hipGraph's
branches, so the answer comes from the kernels themselves: every forward-conv
launch of the capture gets a stamp slot (dmf_stamp_arm, StampScope in
csrc/conv_core.h) into which its waves write [earliest start, latest end] in
s_memrealtime ticks (100 MHz, one clock for the whole chip) when the graph is
replayed -- no profiler attached.

Measured per captured graph (the full mode-A training step of FusionTrainer,
the production graph; and the encoder forward alone, two streams vs serial):
per-stream union of the conv-forward intervals, their intersection (time the
two encoders' convolutions run at the same moment), the replay's conv window,
and the average launch duration in the replay (vs the bench probe, which
replays the launches one stream at a time).

    python tools/stream_stamps.py [--json out.json]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import bench  # noqa: E402
import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402
import parameters as PR  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz
FORMS = {0: "igemm", 1: "buf", 2: "buf_ina", 3: "wide", 4: "sq", 5: "ps", 6: "pp", 7: "stem"}


def _union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _length(u):
    return sum(e - s for s, e in u)


def _intersect(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


MAXB, WAVES = 4096, 8  # csrc/conv_core.h STAMP_MAX_BLOCKS, waves per block region


class Stamps:
    def __init__(self, dev, cap):
        self.cap = cap
        self.buf = torch.zeros(cap * MAXB * WAVES * 2, dtype=torch.int64, device=dev)

    def reset(self):
        self.buf.zero_()

    def arm(self):
        self.reset()
        N.call("dmf_stamp_arm", self.buf.data_ptr(), self.cap)

    @staticmethod
    def disarm():
        n = N.load().dmf_stamp_count()
        recs = []
        st, fm, m, n_, k = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        for i in range(n):
            N.call("dmf_stamp_info", i, ctypes.byref(st), ctypes.byref(fm), ctypes.byref(m), ctypes.byref(n_),
                   ctypes.byref(k))
            recs.append((st.value or 0, fm.value, m.value, n_.value, k.value))
        N.call("dmf_stamp_arm", None, 0)
        return recs

    def read(self, recs):
        v = self.buf.view(self.cap, MAXB * WAVES, 2)[:len(recs)]
        started = v[:, :, 0] != 0
        big = torch.iinfo(torch.int64).max
        s = torch.where(started, v[:, :, 0], torch.full_like(v[:, :, 0], big)).min(1).values.cpu().tolist()
        e = v[:, :, 1].max(1).values.cpu().tolist()
        out = []
        for (st, fm, m, n, k), s_, e_ in zip(recs, s, e):
            if s_ == big or e_ == 0:  # a region this replay did not run (eager warm-up launches)
                continue
            out.append({"stream": st, "form": FORMS.get(fm, fm), "m": m, "n": n, "k": k, "start": s_, "end": e_})
        return out


def _replay_ms(replay, n=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 3)


def analyse(launches, side_handle, label, replay_ms=None):
    by = {"dwi/main": [], "dce/side": []}
    for r in launches:
        by["dce/side" if r["stream"] == side_handle else "dwi/main"].append((r["start"], r["end"]))
    t0 = min(r["start"] for r in launches)
    t1 = max(r["end"] for r in launches)
    u = {k: _union(v) for k, v in by.items()}
    inter = _intersect(u["dwi/main"], u["dce/side"])
    durs = [r["end"] - r["start"] for r in launches]
    flops = sum(2.0 * r["m"] * r["n"] * r["k"] for r in launches)
    res = {"what": label, "launches": len(launches), "replay_ms_with_stamps": replay_ms,
           "launches_per_stream": {k: len(v) for k, v in by.items()},
           "conv_window_us": round((t1 - t0) * TICK_US, 1),
           "busy_union_us": {k: round(_length(v) * TICK_US, 1) for k, v in u.items()},
           "overlap_us": round(inter * TICK_US, 1),
           "overlap_of_side_busy": round(inter / max(1, _length(u["dce/side"])), 3),
           "conv_sum_us": round(sum(durs) * TICK_US, 1),
           "avg_launch_us_in_replay": round(sum(durs) / len(durs) * TICK_US, 2),
           "conv_tflops_in_window": round(flops / ((t1 - t0) * TICK_US * 1e-6) / 1e12, 1)}
    print(json.dumps(res))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from dmf_dp import FusionTrainer

    stamps = Stamps(dev, 640)
    out = []
    lm = bench.build(PR.default_parameters(), dev, torch.bfloat16, "A", seed=0)
    batch = bench.synthetic_batch(32, 256, dev, 2)

    # (1) the production graph: the whole captured mode-A training step
    tr = FusionTrainer(lm, world=1, use_graph=True)
    tr.capture(batch)  # (warm; captured again below with the stamps armed)
    stamps.arm()
    tr.capture(batch)
    recs = Stamps.disarm()
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    ms = _replay_ms(tr.graphs[0].replay)
    stamps.reset()
    tr.graphs[0].replay()
    torch.cuda.synchronize()
    side = lm.__dict__["_side_stream"].cuda_stream
    out.append(analyse(stamps.read(recs), side, "captured mode-A training step (FusionTrainer graph 1)", ms))

    # (2) the encoder forward alone, two streams and serial (the north-star workload)
    dwi, dce = batch[0], batch[1]
    for par in (1, 0):
        O.set_knobs(parallel_encoders=par)

        def fwd():
            with torch.no_grad():
                return lm._encode(dwi, dce)

        fwd()
        fwd()
        torch.cuda.synchronize()
        stamps.arm()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fwd()
        recs = Stamps.disarm()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        ms = _replay_ms(g.replay)
        stamps.reset()
        g.replay()
        torch.cuda.synchronize()
        out.append(analyse(stamps.read(recs), side, f"encoder forward, parallel_encoders={par}", ms))
        del g
    O.set_knobs(parallel_encoders=1)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
