#!/usr/bin/env python3
"""Weight-gradient microbench on the hot path's conv shapes (bf16, B=32): the
split-K slab kernel (dmf_conv2d_wgrad) per shape, HIP events over a hipGraph
of R launches, for each engine variant (dmf_conv_wgrad_tune key 0: LDS-DMA
staging on / off; key 1: its 128x256 tile on / off), interleaved; the reduced
gradients of the variants are compared (every variant sums each weight's
pixels in the same order, so they must agree bit for bit).

    python tools/wgrad_bench.py [--from profiles/r02o_conv_launches.jsonl] [--reps 10] [--rounds 3]
"""
import argparse
import collections
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402


def setup(shape):
    n, h, w, ci, co, k, st, dl = shape
    pad = (k // 2) * dl
    ho, wo = (h + 2 * pad - dl * (k - 1) - 1) // st + 1, (w + 2 * pad - dl * (k - 1) - 1) // st + 1
    x = torch.randn(n, ci, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, co, ho, wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    m = n * ho * wo
    splits = N.load().dmf_conv2d_wgrad_splits(N.BF16, co, ci, k, k, m)
    ws = torch.empty(splits * co * k * k * ci, dtype=torch.float32, device="cuda")
    dw = torch.empty(co, ci, k, k, dtype=torch.float32, device="cuda")

    def launch():
        N.call("dmf_conv2d_wgrad", N.BF16, x.data_ptr(), n, h, w, ci, ci, None, 0, 0, dy.data_ptr(), ho, wo, co, co, k,
               k, st, pad, dl, splits, ws.data_ptr(), O._stream())

    def reduce():
        N.call("dmf_conv2d_wgrad_reduce", ws.data_ptr(), splits, co, ci, ci, k, k, dw.data_ptr(), 0, O._stream())
        return dw.clone()

    flops = 2.0 * m * co * ci * k * k
    return launch, reduce, flops


def timed(launch, reps):
    launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            launch()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--from", dest="src", default=os.path.join(ROOT, "profiles", "r02o_conv_launches.jsonl"))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--sq", action="store_true", help="A/B the 256x256 form against the default")
    ap.add_argument("--reduce", action="store_true",
                    help="time dmf_conv2d_wgrad_reduce alone, split-lane reducers off / on (key 4)")
    a = ap.parse_args()
    if a.reduce:
        return reduce_ab(a)
    cnt = collections.Counter(tuple(json.loads(l)["shape"]) for l in open(a.src))
    shapes = [s for s in sorted(cnt, key=lambda s: -cnt[s] * s[0] * s[1] * s[2] * s[3] * s[4] * s[5] ** 2 / s[6] ** 2)
              if s[3] >= 8 and s[4] >= 8]
    sel = [int(i) for i in a.only.split(",")] if a.only else range(len(shapes))
    # (LDS-DMA, 128x256, 256x256)
    variants = ((1, 1, 0), (1, 1, 1)) if a.sq else ((0, 0, 0), (1, 0, 0), (1, 1, 0))
    tot = [0.0] * len(variants)
    torch.manual_seed(0)
    for i in sel:
        shape = shapes[i]
        times = [[] for _ in variants]
        outs, runs = [], []

        def tune(v):
            for key, val in enumerate(v):
                N.call("dmf_conv_wgrad_tune", key if key < 2 else 3, val)

        for v in variants:
            tune(v)  # the split count (and so the workspace) depends on the tile form
            torch.manual_seed(1)
            launch, reduce, flops = setup(shape)
            launch()
            outs.append(reduce())
            runs.append(launch)
        # the 256x256 form splits the pixels differently (fixed order per split count): close, not identical
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        close = all(((outs[0] - o).abs().max() <= 1e-5 * outs[0].abs().max()).item() for o in outs[1:])
        for _ in range(a.rounds):
            for vi, v in enumerate(variants):
                tune(v)
                times[vi].append(timed(runs[vi], a.reps))
        med = [statistics.median(t) for t in times]
        for vi in range(len(variants)):
            tot[vi] += med[vi] * cnt[shape]
        best = min(med)
        print(f"{i:2d} {str(shape):38s} x{cnt[shape]:2d} " + "  ".join(f"{v} {m * 1e3:7.1f}" for v, m in zip(variants, med))
              + f" us ({flops / best / 1e9:6.1f} TF/s best)  identical={same} close={close}", flush=True)
    tune((1, 1, 1, 0))
    print("weighted totals (ms per step, one encoder pair's forward shapes): " +
          "  ".join(f"{v} {t:.3f}" for v, t in zip(variants, tot)))


def reduce_ab(a):
    cnt = collections.Counter(tuple(json.loads(l)["shape"]) for l in open(a.src))
    shapes = [s for s in cnt if s[3] >= 8 and s[4] >= 8]
    tot = [0.0, 0.0]
    for i, shape in enumerate(shapes):
        launch, reduce, _ = setup(shape)
        launch()
        outs, times = [], [[], []]
        for v in (0, 1):
            N.call("dmf_conv_wgrad_tune", 4, v)
            outs.append(reduce())
        for _ in range(a.rounds):
            for v in (0, 1):
                N.call("dmf_conv_wgrad_tune", 4, v)
                times[v].append(timed(reduce, a.reps))
        med = [statistics.median(t) for t in times]
        for v in (0, 1):
            tot[v] += med[v] * cnt[shape]
        n, h, w, ci, co, k, st, dl = shape
        ho = (h + 2 * (k // 2) * dl - dl * (k - 1) - 1) // st + 1
        splits = N.load().dmf_conv2d_wgrad_splits(N.BF16, co, ci, k, k, n * ho * ho)
        close = ((outs[0] - outs[1]).abs().max() <= 1e-5 * outs[0].abs().max()).item()
        print(f"{i:2d} {str(shape):38s} x{cnt[shape]:2d} splits {splits:4d} weights {co * ci * k * k:8d}  "
              f"one-lane {med[0] * 1e3:6.1f} us  split-lane {med[1] * 1e3:6.1f} us  close={close}", flush=True)
    N.call("dmf_conv_wgrad_tune", 4, 1)
    print(f"weighted totals (ms per step): one-lane {tot[0]:.3f}  split-lane {tot[1]:.3f}")


if __name__ == "__main__":
    main()
