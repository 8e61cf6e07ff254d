#!/usr/bin/env python3
"""BN-apply pass rates on the encoder forward's shapes (bf16, B=32): the
finalize-folded dmf_bn_apply (statistics from a float64 arena) against a
plain streaming copy of the same bytes. HIP events around a hipGraph of R
launches; each launch reads a freshly written arena (as in the forward).

    python tools/apply_bench.py [--reps 20]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402

# (M, C, act, residual kind 0/1/2) -- per encoder forward counts from profiles/r05d (x2 encoders)
SHAPES = [((131072, 64, 1, 0), 8), ((32768, 128, 1, 0), 8), ((32768, 256, 1, 0), 24), ((32768, 512, 1, 0), 12),
          ((131072, 128, 1, 0), 2), ((32768, 1024, 1, 1), 10), ((131072, 256, 1, 1), 4), ((32768, 512, 1, 1), 6),
          ((32768, 2048, 1, 1), 4), ((32768, 256, 2, 0), 12), ((32768, 1024, 1, 2), 2)]


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


def desc(c, acc, ss, save, m):
    d = N.BnDesc()
    d.acc = acc.data_ptr()
    d.gamma = d.beta = d.running_mean = d.running_var = d.num_batches_tracked = None
    d.scale_shift = ss.data_ptr()
    d.save_mean_invstd = save.data_ptr()
    d.count = float(m)
    d.unbias_count = 0.0
    d.momentum = 0.1
    d.eps = 1e-5
    d.replicas = O.BN_ACC_REPLICAS
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    tot_a = tot_c = 0.0
    for (m, c, act, rk), cnt in SHAPES:
        x = torch.randn(m, c, device="cuda").bfloat16()
        y = torch.empty_like(x)
        res = torch.randn(m, c, device="cuda").bfloat16() if rk else None
        acc = torch.rand(O.BN_ACC_REPLICAS * c * 2, device="cuda", dtype=torch.float64) + 1.0
        accr = torch.rand(O.BN_ACC_REPLICAS * c * 2, device="cuda", dtype=torch.float64) + 1.0
        ss = torch.empty(2 * c, device="cuda")
        save = torch.empty(2 * c, device="cuda")
        ssr = torch.empty(2 * c, device="cuda")
        saver = torch.empty(2 * c, device="cuda")
        d = desc(c, acc, ss, save, m)
        dr = desc(c, accr, ssr, saver, m) if rk == 2 else None

        def apply():
            N.call("dmf_bn_apply", N.BF16, x.data_ptr(), c, ctypes.byref(d), None, O._p(res), c,
                   ctypes.byref(dr) if dr is not None else None, None, act, 0.0, None, 0, y.data_ptr(), c, m, c,
                   N.stream_ptr())

        nbytes = x.numel() * 2 * (2 + (1 if rk else 0))
        src = torch.empty(nbytes // 4 // 2, dtype=torch.float32, device="cuda")
        dst = torch.empty_like(src)

        def copy():
            dst.copy_(src)

        ta, tc = timed(apply, a.reps), timed(copy, a.reps)
        tot_a += ta * cnt
        tot_c += tc * cnt
        print(f"M={m:6d} C={c:4d} act={act} res={rk}: apply {ta:7.2f} us ({nbytes / ta / 1e6:5.2f} TB/s)   "
              f"copy of the same bytes {tc:7.2f} us ({nbytes / tc / 1e6:5.2f} TB/s)  x{cnt}", flush=True)
    print(f"weighted per forward: apply {tot_a:.1f} us, copy {tot_c:.1f} us")


if __name__ == "__main__":
    main()
