#!/usr/bin/env python3
"""The fp32 GEMMs (dmf_sgemm) of one eager fusion step at the bench shape:
every (transA, transB, M, N, K, has-workspace) with its count, each timed
alone (HIP events over a hipGraph of R launches) -- the data for sizing a
small-tile f32 GEMM for the fusion's token linears.

    python tools/sgemm_shapes.py [--mode A] [--batch 32] [--reps 20]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import torch  # noqa: E402

import bench  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--mode", default="A")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import dmf_native as N
    import dmf_ops as O
    import parameters as PR
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    lm = bench.build(P, dev, torch.bfloat16, a.mode)
    tr = FusionTrainer(lm, world=1, use_graph=False)
    batch = bench.synthetic_batch(a.batch, 256, dev, 2)
    tr.step(batch)
    torch.cuda.synchronize()
    seen = collections.Counter()
    real = N.call

    def spy(name, *args):
        if name == "dmf_sgemm":
            tA, tB, M, Nn, K = args[:5]
            seen[(tA, tB, M, Nn, K, args[15] is not None, args[10] != 0.0)] += 1
        return real(name, *args)

    N.call = spy
    try:
        tr.step(batch)
        torch.cuda.synchronize()
    finally:
        N.call = real
    tot = 0.0
    for (tA, tB, M, Nn, K, ws, acc), cnt in sorted(seen.items(), key=lambda kv: -kv[1]):
        A = torch.randn((K, M) if tA else (M, K), device=dev)
        B = torch.randn((Nn, K) if tB else (K, Nn), device=dev)
        C = torch.empty(M, Nn, device=dev)
        W, wsn = None, 0

        def run():
            real("dmf_sgemm", tA, tB, M, Nn, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], 0.0,
                 C.data_ptr(), Nn, None, 0, W.data_ptr() if wsn else None, O._stream())

        wsn = N.load().dmf_sgemm_ws_size(M, Nn, K) if ws else 0
        W = torch.empty(max(wsn, 1), device=dev)
        us = timed(run, a.reps)
        tot += us * cnt
        print(f"tA={tA} tB={tB} M={M:5d} N={Nn:5d} K={K:5d} ws={int(ws)} beta={int(acc)} x{cnt:3d}  {us:6.1f} us",
              flush=True)
    print(f"total {tot / 1e3:.3f} ms per step ({sum(seen.values())} launches)")


if __name__ == "__main__":
    main()
