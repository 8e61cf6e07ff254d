#!/usr/bin/env python3
"""SEBlock excitation (dmf_se_mlp) on the path's shapes (B=32; C = 128 / 256, mid = C/2; squeeze partial
planes S): the one-workgroup form against the three-launch form, HIP events over a hipGraph of R launches.

    python tools/se_bench.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402
from gemm_bench import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for n, c, s in ((32, 128, 1), (32, 128, 8), (32, 256, 1), (32, 256, 8), (32, 256, 32), (32, 512, 4)):
        mid = c // 2
        ws = torch.randn(s, n, c, device="cuda")
        w1, b1 = torch.randn(mid, c, device="cuda"), torch.randn(mid, device="cuda")
        w2, b2 = torch.randn(c, mid, device="cuda"), torch.randn(c, device="cuda")
        outs = [torch.empty(n, c, device="cuda"), torch.empty(n, mid, device="cuda"),
                torch.empty(n, mid, device="cuda"), torch.empty(n, c, device="cuda")]
        res = []
        for one in (1, 2, 0):
            N.call("dmf_se_mlp_tune", one)

            def run():
                N.call("dmf_se_mlp", ws.data_ptr(), s, n, c, 1.0 / s, w1.data_ptr(), b1.data_ptr(), mid, w2.data_ptr(),
                       b2.data_ptr(), outs[0].data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(),
                       O._stream())
            res.append(timed(run, a.reps))
        N.call("dmf_se_mlp_tune", 1)
        print(f"N={n} C={c} mid={mid} S={s}: two MFMA-tile launches {res[0]:6.1f} us   one workgroup {res[1]:6.1f} us"
              f"   three launches {res[2]:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
