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
    ((32, 256, 256, 8, 64, 7, 2, 1), 1),
    ((32, 32, 32, 64, 64, 1, 1, 1), 9),
]


ACC = [False]  # --acc: BN statistics into a float64 arena (dmf_conv2d_fwd_acc), as the training forward does


def _fwd_acc(x, weight, g, caches, acc):
    import dmf_native as N
    n, cx, h, w, ldx = O.nhwc(x)
    co, ci, kh, kw = weight.shape
    ho, wo = g.out_hw(h, w)
    y = O.empty_nhwc(n, co, ho, wo, x.dtype, x.device)
    wk = caches[0].get(weight, x.dtype, cx, 0)
    N.call("dmf_conv2d_fwd_acc", O.dt(x), x.data_ptr(), n, h, w, cx, ldx, None, 0, 0, wk.data_ptr(), co, kh, kw,
           g.stride, g.pad, g.dil, None, y.data_ptr(), ho, wo, O.nhwc(y)[4], acc.data_ptr(), O.BN_ACC_REPLICAS, None,
           N.ACT_NONE, O._stream())
    return y


def run_shape(shape, reps, stats, dtype=torch.bfloat16):
    n, h, w, ci, co, k, st, dl = shape
    conv = torch.nn.Conv2d(ci, co, k, stride=st, padding=(k // 2) * dl, dilation=dl, bias=False).cuda()
    conv.weight.requires_grad_(False)
    x = torch.randn(n, ci, h, w, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    g = O.ConvGeom(conv)
    caches = (O.WeightCache(), O.WeightCache())
    acc = torch.zeros(2 * co * O.BN_ACC_REPLICAS, dtype=torch.float64, device="cuda")

    def launch():
        if ACC[0] and stats and O._is_mfma_conv(conv.weight, g):
            _fwd_acc(x, conv.weight, g, caches, acc)
        else:
            O._conv_forward_raw(x, conv.weight, None, g, caches, stats, "none")

    with torch.no_grad():
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        # replay R launches from a hipGraph: GPU time only (no Python launch overhead)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(reps):
                launch()
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


def _shapes(src):
    import collections
    import json
    cnt = collections.Counter(tuple(json.loads(l)["shape"]) for l in open(src))
    return sorted(cnt.items(), key=lambda kv: -kv[1] * kv[0][0] * kv[0][1] * kv[0][2] * kv[0][3] * kv[0][4] *
                  kv[0][5] ** 2 / kv[0][6] ** 2)


def ab(a):
    """Interleaved A/B of tuning variants (cdna_hip_programming.md 5.4 rule 24):
    per shape, rounds x variants, median time per variant."""
    import statistics

    import dmf_native as N
    variants = [[tuple(int(t) for t in kv.split(":")) for kv in grp.split(",") if kv] for grp in a.tunes.split(";")]
    shapes = _shapes(a.src) if a.src else SHAPES
    sel = [int(i) for i in a.only.split(",")] if a.only else range(len(shapes))
    tot = [0.0] * len(variants)
    print("variants:", variants)
    for i in sel:
        shape, cnt = shapes[i]
        times = [[] for _ in variants]
        for _ in range(a.rounds):
            for vi, var in enumerate(variants):
                for k, v in var:
                    N.call("dmf_conv_tune", k, v)
                times[vi].append(run_shape(shape, a.reps, not a.nostats)[0])
        med = [statistics.median(t) for t in times]
        for vi in range(len(variants)):
            tot[vi] += med[vi] * cnt
        print(f"{i:2d} {str(shape):38s} x{cnt:2d} " + " ".join(f"{m * 1e3:8.1f}" for m in med) + " us", flush=True)
    print("weighted totals (ms):", " ".join(f"{t:.3f}" for t in tot))
    for k, v in variants[0]:
        N.call("dmf_conv_tune", k, v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--nostats", action="store_true")
    ap.add_argument("--from", dest="src", default="", help="bench.py DMF_CONV_DUMP jsonl: every distinct shape, with counts")
    ap.add_argument("--tunes", default="", help="A/B variants, e.g. '0:0;0:1,1:0;0:1,1:1' (dmf_conv_tune key:value "
                                                "lists), timed interleaved in this process")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--acc", action="store_true", help="BN statistics into the float64 arena (the training forward's mode)")
    ap.add_argument("--shapes", default="", help="custom shapes 'N,H,W,Cin,Cout,k,stride,dil;...' (count 1 each) "
                                                 "instead of the hot-path list")
    a = ap.parse_args()
    if a.shapes:
        SHAPES[:] = [(tuple(int(v) for v in s.split(",")), 1) for s in a.shapes.split(";") if s]
    ACC[0] = a.acc
    if a.tunes:
        return ab(a)
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
