#!/usr/bin/env python3
"""Token-GEMM microbench (config 5 shapes: 32 volumes x 576 tokens, E = 512,
4 heads): the linears and Q K^T through dmf_gemm_bf16, HIP events over a
hipGraph of R launches.

    python tools/gemm_bench.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")]

import torch  # noqa: E402

import dmf_tokens as D  # noqa: E402


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
    ap.add_argument("--only", default="", help="comma-separated case-name prefixes")
    a = ap.parse_args()
    dev = "cuda"
    r, e, hid, b, h, n = 32 * 576, 512, 2048, 32, 4, 576
    d = e // h
    bf = dict(dtype=torch.bfloat16, device=dev)
    x = torch.randn(r, e, **bf)
    hbuf = torch.randn(r, hid, **bf)
    qkv = torch.randn(r, 3 * e, **bf)
    cases = {
        "qkv  (18432x1536x512)": lambda: D.gemm(out_qkv, x, wq, r, 3 * e, e, lda=e, ldb=e, ldc=3 * e, bias=bq),
        "fc1  (18432x2048x512) gelu": lambda: D.gemm(out_h, x, w1, r, hid, e, lda=e, ldb=e, ldc=hid, bias=b1, act="gelu"),
        "fc2  (18432x512x2048) f32": lambda: D.gemm(out_f, hbuf, w2, r, e, hid, lda=hid, ldb=hid, ldc=e, bias=bp),
        "proj (18432x512x512) f32": lambda: D.gemm(out_f, x, wp, r, e, e, lda=e, ldb=e, ldc=e, bias=bp),
        "QK^T (576x576x128 x128)": lambda: D.gemm(S, qkv, qkv, n, n, d, lda=3 * e, ldb=3 * e, ldc=n, batch=(b, h),
                                                  sa=(n * 3 * e, d), sb=(n * 3 * e, d), sc=(h * n * n, n * n), b_off=e),
    }
    wq, w1, w2, wp = (torch.randn(3 * e, e, **bf), torch.randn(hid, e, **bf), torch.randn(e, hid, **bf),
                      torch.randn(e, e, **bf))
    bq, b1, bp = torch.randn(3 * e, device=dev), torch.randn(hid, device=dev), torch.randn(e, device=dev)
    out_qkv, out_h = torch.empty((r, 3 * e), **bf), torch.empty((r, hid), **bf)
    out_f = torch.empty((r, e), dtype=torch.float32, device=dev)
    S = torch.empty((b, h, n, n), dtype=torch.float32, device=dev)
    flops = {"qkv": 2 * r * 3 * e * e, "fc1": 2 * r * hid * e, "fc2": 2 * r * e * hid, "proj": 2 * r * e * e,
             "QK^T": 2 * b * h * n * n * d}
    # the same linears on the conv engine (a 1x1 conv over [r, e] rows viewed as NHWC (32, e, 24, 24)):
    # persistent 256x256 tiles, register epilogue (bias + act, bf16 out)
    import dmf_ops as O

    def conv_case(w, bias, k_in, act):
        conv = torch.nn.Conv2d(k_in, w.shape[0], 1).to(dev)
        with torch.no_grad():
            conv.weight.copy_(w.float()[:, :, None, None])
            conv.bias.copy_(bias)
        conv.requires_grad_(False)
        xin = (x if k_in == e else hbuf).view(b, 24, 24, k_in).permute(0, 3, 1, 2)
        caches = (O.WeightCache(), O.WeightCache())

        def run():
            with torch.no_grad():
                y, _ = O._conv_forward_raw(xin, conv.weight, conv.bias, O.ConvGeom(conv), caches, False, act)
            return y
        return run
    cases["qkv  conv-engine"] = conv_case(wq, bq, e, "none")
    cases["fc1  conv-engine gelu"] = conv_case(w1, b1, e, "gelu")
    lin1 = torch.nn.Linear(e, hid).to(dev)
    with torch.no_grad():
        lin1.weight.copy_(w1.float())
        lin1.bias.copy_(b1)
    lin1.requires_grad_(False)
    cases["fc1  gemm gelu + dropout 0.1"] = lambda: D.gemm(out_h, x, w1, r, hid, e, lda=e, ldb=e, ldc=hid, bias=b1,
                                                           act="gelu", dropout_p=0.1, rng=rng, site=3)
    cases["fc1  conv-engine gelu + dropout 0.1"] = lambda: D._linear_conv_drop(x, lin1, b, n, 0.1, rng, 3)
    cases["fc2  conv-engine (bf16 out)"] = conv_case(w2, bp, hid, "none")
    cases["proj conv-engine (bf16 out)"] = conv_case(wp, bp, e, "none")
    sm_p = torch.empty((b, h, n, n), **bf)

    def softmax():
        import dmf_native as N
        N.call("dmf_softmax_dropout", S.data_ptr(), n, b * h * n, n, n, float(d ** -0.5), 0.0, None, 0,
               sm_p.data_ptr(), sm_p.data_ptr(), n, O._stream())
    cases["softmax (128 x 576 rows)"] = softmax
    o = torch.empty((r, e), **bf)
    cases["PV   (576x128x576 x128)"] = lambda: D.gemm(o, sm_p, qkv, n, d, n, tb=1, lda=n, ldb=3 * e, ldc=e,
                                                        batch=(b, h), sa=(h * n * n, n * n), sb=(n * 3 * e, d),
                                                        sc=(n * e, d), b_off=2 * e)
    import dmf_native as N

    def flash(nq, p):
        def run():
            N.call("dmf_flash_attn_tune", nq)
            D.flash_attention(qkv, b, n, n, e, h, p, rng if p > 0 else None, 3)
        return run
    for var in (1, 2, 3):
        cases[f"flash QK^T.softmax.PV var={var}"] = flash(var, 0.0)
        cases[f"flash + dropout 0.1 var={var}"] = flash(var, 0.1)
    # the fp8 patch-embed GEMM (18432 x 512 x 1024, e4m3) in both forms
    kp = 1024
    qa = (torch.randn(r, kp, device=dev) * 100).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    qb = (torch.randn(e, kp, device=dev) * 100).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    ra_, rb_ = torch.rand(r, device=dev), torch.rand(e, device=dev)
    y8 = torch.empty((r, e), **bf)

    def fp8(var):
        def run():
            N.call("dmf_gemm_fp8_tune", var)
            N.call("dmf_gemm_fp8", r, e, kp, qa.data_ptr(), kp, ra_.data_ptr(), qb.data_ptr(), kp, rb_.data_ptr(),
                   bp.data_ptr(), y8.data_ptr(), e, O._stream())
        return run
    cases["fp8  (18432x512x1024) 128x128"] = fp8(0)
    cases["fp8  (18432x512x1024) scaled 144x256"] = fp8(1)
    flops["fp8"] = 2 * r * e * kp
    rng = O.RNG.snapshot(torch.device(dev))
    flops["flash"] = 2 * flops["QK^T"]
    flops["softmax"] = 1.0
    flops["PV"] = 2 * b * h * n * n * d
    only = [c for c in a.only.split(",") if c]
    for name, fn in cases.items():
        if only and not any(name.startswith(o) for o in only):
            continue
        us = timed(fn, a.reps)
        fl = flops[name.split()[0]]
        print(f"{name:30s} {us:7.1f} us ({fl / us / 1e6:6.1f} TF/s)", flush=True)
    N.call("dmf_gemm_fp8_tune", 1)


if __name__ == "__main__":
    main()
