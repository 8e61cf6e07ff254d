#!/usr/bin/env python3
"""Test-time TTA x MC-dropout throughput: the batched
predict_tta_mc (4 flips x P passes as ceil(4*P*B/chunk) forwards) against the
reference's loop of 4*P separate forwards (train_fusion.py:591-632), on one
GPU, config-3 shapes, bf16, synthetic volumes. Prints one JSON line.

    python tools/predict_bench.py [--batch 32] [--passes 10] [--chunk 256]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import bench  # noqa: E402
import parameters as PR  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--passes", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = a.size
    lm = bench.build(P, dev, torch.bfloat16, "A")
    lm.eval()
    dwi, dce, _, _ = bench.synthetic_batch(a.batch, a.size, dev, 9)

    def batched():
        return lm.predict_tta_mc(dwi, dce, passes=a.passes, chunk=a.chunk)

    def loop():  # the reference's structure: one forward per (flip, pass)
        st = {m: m.training for m in lm.modules()}
        lm.mc_enable(lm.dwi_model)
        lm.mc_enable(lm.dce_model)
        outs = []
        with torch.no_grad():
            for t in lm.transforms_list:
                for _ in range(a.passes):
                    (_, da, dm), (_, ca, cm) = lm._encode(t(x=dwi), t(x=dce))
                    logits, _, _ = lm.forward(da["raw_feats"], ca["raw_feats"], dm, cm)
                    outs.append(torch.softmax(logits.float(), 1))
        for m, w in st.items():
            m.train(w)
        return outs

    tb = timed(batched, a.reps)
    tl = timed(loop, a.reps)
    n_fwd = len(lm.transforms_list) * a.passes * a.batch
    print(json.dumps({
        "metric": "TTA x MC-dropout test-time volumes/s (4 flips x passes forwards per volume)",
        "batched_volumes_per_s": round(a.batch / tb, 2), "loop_volumes_per_s": round(a.batch / tl, 2),
        "batched_forward_volumes_per_s": round(n_fwd / tb, 1), "speedup": round(tl / tb, 3),
        "batch": a.batch, "passes": a.passes, "flips": len(lm.transforms_list), "chunk": a.chunk,
        "size": a.size, "dtype": "bf16", "data": "synthetic config-3 volumes, random-init weights"}))


if __name__ == "__main__":
    main()
