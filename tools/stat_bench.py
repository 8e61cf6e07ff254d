#!/usr/bin/env python3
"""A/B of the conv epilogue's BN-statistics forms on hot-path shapes (bf16):
no statistics, the slab (one row per M tile), float64 atomics into [C][2],
float64 atomics into R replicas, float32 atomics. Interleaved rounds in one
process, median per variant (cdna_hip_programming.md 5.4 rule 24).

    python tools/stat_bench.py [--rounds 5] [--reps 20]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402

SHAPES = [(32, 32, 32, 1024, 256, 1), (32, 32, 32, 256, 256, 3), (32, 64, 64, 64, 64, 3), (32, 32, 32, 512, 2048, 1),
          (32, 64, 64, 256, 64, 1), (32, 32, 32, 128, 128, 3)]
VARIANTS = ["nostats", "slab", "f64", "f64r8", "f64r32", "f32"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for (n, h, w, ci, co, k) in SHAPES:
        conv = torch.nn.Conv2d(ci, co, k, padding=k // 2, bias=False).cuda()
        conv.weight.requires_grad_(False)
        x = torch.randn(n, ci, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        g = O.ConvGeom(conv)
        caches = (O.WeightCache(), O.WeightCache())
        wk = caches[0].get(conv.weight, x.dtype, ci, 0)
        y = O.empty_nhwc(n, co, h, w, x.dtype, x.device)
        tiles = N.load().dmf_conv2d_fwd_stat_tiles(1, n, h, w, ci, ci, 0, 0, co, k, k, 1, k // 2, h, w, 0)
        slab = torch.zeros(tiles * co * 2, dtype=torch.float32, device="cuda")
        acc = torch.zeros(64 * co * 2, dtype=torch.float64, device="cuda")

        def launch(v):
            if v == "nostats":
                N.call("dmf_conv2d_fwd", 1, x.data_ptr(), n, h, w, ci, ci, None, 0, 0, wk.data_ptr(), co, k, k, 1,
                       k // 2, 1, None, y.data_ptr(), h, w, co, None, 0, None, 0, N.stream_ptr())
            elif v == "slab":
                N.call("dmf_conv2d_fwd", 1, x.data_ptr(), n, h, w, ci, ci, None, 0, 0, wk.data_ptr(), co, k, k, 1,
                       k // 2, 1, None, y.data_ptr(), h, w, co, slab.data_ptr(), 0, None, 0, N.stream_ptr())
            else:
                N.call("dmf_conv_tune", 3, {"f64": 1, "f64r8": 8, "f64r32": 32, "f32": -1}[v])
                N.call("dmf_conv2d_fwd_acc", 1, x.data_ptr(), n, h, w, ci, ci, None, 0, 0, wk.data_ptr(), co, k, k,
                       1, k // 2, 1, None, y.data_ptr(), h, w, co, acc.data_ptr(), 1, None, 0, N.stream_ptr())

        graphs = {}
        for v in VARIANTS:
            for _ in range(2):
                launch(v)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(a.reps):
                    launch(v)
            graphs[v] = gr
        N.call("dmf_conv_tune", 3, 0)
        times = {v: [] for v in VARIANTS}
        for _ in range(a.rounds):
            for v in VARIANTS:
                graphs[v].replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graphs[v].replay()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps * 1e3)
        print((n, h, w, ci, co, k), "tiles", tiles, " ".join(f"{v}={statistics.median(times[v]):.1f}us" for v in VARIANTS),
              flush=True)


if __name__ == "__main__":
    main()
