#!/usr/bin/env python3
"""Interleaved A/B of the north-star workload (DWI + DCE encoder forward, B=32,
S=256, bf16, train-mode BN, two streams, hipGraph replay) over dmf_conv_tune
variants, in one process (cdna_hip_programming.md 5.4 rule 24): each variant
gets its own captured graph; rounds x variants, median ms per variant.

    python tools/enc_fwd_ab.py --tunes "7:0;7:1" [--rounds 4] [--reps 10]

A variant entry is KEY:VAL (dmf_conv_tune) or name=VAL (dmf_ops.set_knobs),
e.g. --tunes "two_pass_bn=1;two_pass_bn=0".
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import bench  # noqa: E402
import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402
import parameters as PR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tunes", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    variants = [[kv for kv in grp.split(",") if kv] for grp in a.tunes.split(";")]
    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    lm = bench.build(P, dev, torch.bfloat16, "A", seed=0)
    dwi, dce, _, _ = bench.synthetic_batch(32, 256, dev, 2)

    def fwd():
        with torch.no_grad():
            return lm._encode(dwi, dce)

    graphs = []
    for var in variants:
        for kv in var:
            if "=" in kv:
                k, v = kv.split("=")
                O.set_knobs(**{k: int(v)})
            else:
                k, v = (int(t) for t in kv.split(":"))
                N.call("dmf_conv_tune", k, v)
        g, _ = bench._graph(fwd)  # kernels are chosen at capture: the graph keeps this variant
        graphs.append(g)
    times = [[] for _ in variants]
    for _ in range(a.rounds):
        for vi, g in enumerate(graphs):
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            times[vi].append(e0.elapsed_time(e1) / a.reps)
    for vi, var in enumerate(variants):
        med = statistics.median(times[vi])
        print(json.dumps({"variant": var, "encoder_forward_ms_median": round(med, 3), "min": round(min(times[vi]), 3),
                          "frac": round(bench.T_ROOF_ENC_FWD_MS_B32 / med, 4), "all": [round(t, 3) for t in times[vi]]}))


if __name__ == "__main__":
    main()
