#!/usr/bin/env python3
"""Calibration of the conv-forward roofline target: the same bf16 shapes as
tools/conv_bench.py through the vendor libraries on this box (hipBLASLt via
torch.matmul for the 1x1 convs as plain [M,K]x[K,N] GEMMs, MIOpen via
F.conv2d channels_last for every shape) beside this library's conv (no BN
statistics), per-shape TFLOP/s from HIP events over a hipGraph replay.

    python tools/lib_ceiling.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import conv_bench as CB  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    big = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    ms = timed(lambda: big @ big, 10)
    print(f"hipBLASLt 8192^3 bf16: {ms * 1e3:8.1f} us {2 * 8192 ** 3 / ms / 1e9:7.1f} TF/s", flush=True)
    print(f"{'shape':40s} {'ours':>16s} {'MIOpen':>16s} {'hipBLASLt':>16s}")
    for shape, cnt in CB.SHAPES:
        n, h, w, ci, co, k, st, dl = shape
        ho, wo = (h + 2 * (k // 2) * dl - dl * (k - 1) - 1) // st + 1, (w + 2 * (k // 2) * dl - dl * (k - 1) - 1) // st + 1
        flops = 2.0 * n * ho * wo * co * k * k * ci
        ours, _ = CB.run_shape(shape, a.reps, False)
        x = torch.randn(n, ci, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(co, ci, k, k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            mio = timed(lambda: F.conv2d(x, wt, None, st, (k // 2) * dl, dl), a.reps)
        cell = lambda t: f"{t * 1e3:7.1f}us {flops / t / 1e9:6.0f}"  # noqa: E731
        line = f"{str(shape):40s} {cell(ours)} {cell(mio)}"
        if k == 1 and st == 1:
            xm = torch.randn(n * h * w, ci, device="cuda", dtype=torch.bfloat16)
            wm = torch.randn(ci, co, device="cuda", dtype=torch.bfloat16)
            line += f" {cell(timed(lambda: xm @ wm, a.reps))}"
        print(line + f"  x{cnt}", flush=True)


if __name__ == "__main__":
    main()
