#!/usr/bin/env python3
"""Microbenchmark of the implicit-GEMM conv on the hot path's dominant
shapes (bf16, B=32 per GPU): per-shape TFLOP/s from HIP events over R
repetitions, with and without the BN partial-statistics epilogue.

    python tools/conv_bench.py [--reps 20] [--only i,j]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_ops as O  # noqa: E402

# (N, H, W, Cin, Cout, k, stride, dil) -- as dumped by bench.py DMF_CONV_DUMP, with call counts per step
SHAPES = [
    ((32, 32, 32, 3072, 256, 3, 1, 1), 2),
    ((32, 32, 32, 512, 2048, 1, 1, 1), 6),
    ((32, 32, 32, 512, 512, 3, 1, 4), 4),
    ((32, 32, 32, 256, 1024, 1, 1, 1), 12),
    ((32, 32, 32, 256, 256, 3, 1, 2), 10),
    ((32, 32, 32, 256, 256, 3, 1, 1), 8),
    ((32, 32, 32, 128, 128, 3, 1, 1), 14),
    ((32, 32, 32, 1024, 2048, 1, 1, 1), 2),
    ((32, 32, 32, 2048, 512, 1, 1, 1), 4),
    ((32, 32, 32, 1024, 256, 1, 1, 1), 10),
    ((32, 64, 64, 64, 256, 1, 1, 1), 8),
    ((32, 64, 64, 64, 64, 3, 1, 1), 6),
    ((32, 256, 256, 16, 64, 7, 2, 1), 1),
    ((32, 32, 32, 64, 64, 1, 1, 1), 9),
]


def run_shape(shape, reps, stats, dtype=torch.bfloat16):
    n, h, w, ci, co, k, st, dl = shape
    conv = torch.nn.Conv2d(ci, co, k, stride=st, padding=(k // 2) * dl, dilation=dl, bias=False).cuda()
    conv.weight.requires_grad_(False)
    x = torch.randn(n, ci, h, w, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    g = O.ConvGeom(conv)
    caches = (O.WeightCache(), O.WeightCache())
    with torch.no_grad():
        for _ in range(3):
            O._conv_forward_raw(x, conv.weight, None, g, caches, stats, "none")
        torch.cuda.synchronize()
        # replay R launches from a hipGraph: GPU time only (no Python launch overhead)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(reps):
                O._conv_forward_raw(x, conv.weight, None, g, caches, stats, "none")
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    ho, wo = g.out_hw(h, w)
    flops = 2.0 * n * ho * wo * co * k * k * ci
    return ms, flops / (ms * 1e-3) / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--nostats", action="store_true")
    ap.add_argument("--from", dest="src", default="", help="bench.py DMF_CONV_DUMP jsonl: every distinct shape, with counts")
    a = ap.parse_args()
    shapes = SHAPES
    if a.src:
        import collections
        import json
        cnt = collections.Counter(tuple(json.loads(l)["shape"]) for l in open(a.src))
        shapes = sorted(cnt.items(), key=lambda kv: -kv[1] * kv[0][0] * kv[0][1] * kv[0][2] * kv[0][3] * kv[0][4] * kv[0][5] ** 2 / kv[0][6] ** 2)
    sel = [int(i) for i in a.only.split(",")] if a.only else range(len(shapes))
    tot_ms = 0.0
    for i in sel:
        shape, cnt = shapes[i]
        ms, tf = run_shape(shape, a.reps, not a.nostats)
        tot_ms += ms * cnt
        print(f"{i:2d} {str(shape):38s} x{cnt:2d} {ms * 1e3:8.1f} us {tf:7.1f} TF/s", flush=True)
    print(f"weighted total (per step, these shapes): {tot_ms:.3f} ms")


if __name__ == "__main__":
    main()
