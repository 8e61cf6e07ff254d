#!/usr/bin/env python3
"""Grid-barrier BatchNorm apply (dmf_conv2d_fwd_bn_act) against the conv + dmf_bn_apply form on the
frozen encoder's shapes (bf16, B=32): HIP events around a hipGraph of R forward-only conv_bn_act
calls per variant. Timing variants (dmf_conv_tune key 17, outputs wrong): 64 skips the barrier,
128 the arena reads, 192 both -- what is left is the K loop + the register epilogue.

    python tools/gbar_bench.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402

# (N, Cin, H, W, Cout, k, pad, dil, bias, act)
SHAPES = [(32, 2048, 32, 32, 512, 1, 0, 1, False, "relu"), (32, 1024, 32, 32, 512, 1, 0, 1, False, "relu"),
          (32, 512, 32, 32, 512, 3, 4, 4, False, "relu"), (32, 1024, 32, 32, 256, 1, 0, 1, False, "relu"),
          (32, 512, 32, 32, 256, 1, 0, 1, False, "relu"), (32, 256, 32, 32, 256, 3, 2, 2, False, "relu"),
          (32, 256, 32, 32, 256, 3, 1, 1, True, "gelu")]


def timed(fn, reps):
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
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for n, ci, h, w, co, k, pad, dil, bias, act in SHAPES:
        conv = nn.Conv2d(ci, co, k, padding=pad, dilation=dil, bias=bias).cuda().requires_grad_(False)
        bn = nn.BatchNorm2d(co).cuda().train().requires_grad_(False)
        x = torch.randn(n, ci, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        caches = (O.WeightCache(), O.WeightCache())

        def fwd():
            with torch.no_grad():
                return O.conv_bn_act(x, conv, caches, bn, act)

        res = {}
        for name, knob, dbg in (("conv+apply", 0, 0), ("barrier", 1, 0), ("no-arena", 1, 128), ("no-barrier", 1, 64),
                                ("loop+epi", 1, 192)):
            O.set_knobs(grid_barrier_bn=knob)
            N.call("dmf_conv_tune", 17, dbg)
            try:
                res[name] = timed(fwd, a.reps)
            finally:
                N.call("dmf_conv_tune", 17, 0)
                O.set_knobs(grid_barrier_bn=1)
        form = N.FORMS.get(N.load().dmf_conv_last_form())
        print(f"{ci:5d}->{co:4d} k{k} d{dil} {act} [{form}]: " + "  ".join(f"{k_} {v:7.1f}" for k_, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
