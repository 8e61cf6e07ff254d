#!/usr/bin/env python3
"""HBM-pass efficiency of the BN-backward kernels against plain streaming
copies of the same byte count (bf16, M = 32768 pixels = B=32 at 32x32):

* torch `a + b -> c` on contiguous tensors (2 reads + 1 write), and a float4
  copy (1 read + 1 write), as the achievable streaming rates;
* dmf_bn_bwd_apply_acc (reads dz, x; writes dx) and dmf_act_bwd_bn_reduce_acc
  (reads dy, x [, res, dy2]; writes dz; column sums into the arena).

HIP events around a hipGraph of R launches.

    python tools/bw_probe.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402


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
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    M = 32768
    for C in (128, 256, 1024, 2048):
        mb = M * C * 2 / 1e6
        t = [torch.randn(M, C, device=dev).to(torch.bfloat16) for _ in range(5)]
        save = torch.cat([torch.zeros(C), torch.ones(C)]).to(dev)
        ss = torch.cat([torch.ones(C), torch.zeros(C)]).to(dev)
        acc = torch.zeros(8 * C * 2, dtype=torch.float64, device=dev)
        gamma = torch.ones(C, device=dev)
        st = O._stream

        def add():
            torch.add(t[0], t[1], out=t[2])

        def copy():
            t[2].copy_(t[0])

        def apply():
            N.call("dmf_bn_bwd_apply_acc", N.BF16, t[0].data_ptr(), C, t[1].data_ptr(), C, acc.data_ptr(), 8,
                   float(M), 1, gamma.data_ptr(), save.data_ptr(), None, None, t[2].data_ptr(), C, M, C, st())

        def actbwd(res=False, dy2=False):
            def f():
                N.call("dmf_act_bwd_bn_reduce_acc", N.BF16, t[0].data_ptr(), C, t[3].data_ptr() if dy2 else None,
                       C if dy2 else 0, t[1].data_ptr(), C, ss.data_ptr(), t[4].data_ptr() if res else None,
                       C if res else 0, None, N.ACT_RELU, 0.0, None, 0, save.data_ptr(), t[2].data_ptr(), C, M, C,
                       acc.data_ptr(), 8, st())
            return f

        part = torch.empty((M + 255) // 256 * C * 2, dtype=torch.float32, device=dev)

        def actbwd_slab():
            N.call("dmf_act_bwd_bn_reduce", N.BF16, t[0].data_ptr(), C, None, 0, t[1].data_ptr(), C, ss.data_ptr(),
                   None, 0, None, N.ACT_RELU, 0.0, None, 0, save.data_ptr(), t[2].data_ptr(), C, M, C,
                   part.data_ptr(), st())

        rng = O.RNG.snapshot(dev)

        def affine(act, p=0.0):
            def f():
                N.call("dmf_affine_act", N.BF16, t[0].data_ptr(), C, ss.data_ptr(), None, 0, None, act, p,
                       rng.data_ptr() if p > 0 else None, 1, t[2].data_ptr(), C, M, C, st())
            return f

        rows = [("copy (1R+1W)", copy, 2), ("affine + relu (1R+1W)", affine(N.ACT_RELU), 2),
                ("affine + gelu (1R+1W)", affine(N.ACT_GELU), 2),
                ("affine + gelu + dropout 0.4 (1R+1W)", affine(N.ACT_GELU, 0.4), 2),
                ("act_bwd_bnred slab partials (2R+1W)", actbwd_slab, 3), ("torch add (2R+1W)", add, 3), ("bn_bwd_apply_acc (2R+1W)", apply, 3),
                ("act_bwd_bnred (2R+1W)", actbwd(), 3), ("act_bwd_bnred +res (3R+1W)", actbwd(True), 4),
                ("act_bwd_bnred +res+dy2 (4R+1W)", actbwd(True, True), 5)]
        for name, fn, passes in rows:
            us = timed(fn, a.reps)
            print(f"C={C:5d} {name:32s} {us:7.1f} us  {passes * mb / us:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
