#!/usr/bin/env python3
"""How much would running the two encoders' backbones as ONE launch sequence
(the DWI and DCE batches concatenated, each half on its own weights) save over
the two-stream fork? Upper-bound probe, no new kernels: the DWI encoder's
forward at B=64 (the same work as both encoders at B=32 with grouped launches)
against the production two-stream forward at B=32 + 32 and the serial one.
Interleaved rounds in one process, hipGraph replays, no autograd.

    python tools/group_probe.py [--rounds 3] [--reps 10]
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
import dmf_ops as O  # noqa: E402
import parameters as PR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lm = bench.build(PR.default_parameters(), dev, torch.bfloat16, "A", seed=0)
    dwi, dce, _, _ = bench.synthetic_batch(32, 256, dev, 2)
    dwi64, _, _, _ = bench.synthetic_batch(64, 256, dev, 3)
    bb = lambda m: m.backbone_adapter.backbone  # noqa: E731

    def enc_pair():
        with torch.no_grad():
            return lm._encode(dwi, dce)

    def dwi_b64():
        with torch.no_grad():
            return lm.dwi_model(dwi64)

    def backbone_pair_serial():
        with torch.no_grad():
            xa, _ = lm.dwi_model._stage_input(dwi)
            xb, _ = lm.dce_model._stage_input(dce)
            return bb(lm.dwi_model)(xa), bb(lm.dce_model)(xb)

    def backbone_b64():
        with torch.no_grad():
            xa, _ = lm.dwi_model._stage_input(dwi64)
            return bb(lm.dwi_model)(xa)

    variants = {"encoders two-stream B=32+32": (enc_pair, {}),
                "encoders serial B=32+32": (enc_pair, {"parallel_encoders": 0}),
                "dwi encoder B=64": (dwi_b64, {}),
                "backbones serial B=32+32": (backbone_pair_serial, {}),
                "dwi backbone B=64": (backbone_b64, {})}
    graphs = {}
    for name, (fn, knobs) in variants.items():
        O.set_knobs(parallel_encoders=1)
        if knobs:
            O.set_knobs(**knobs)
        graphs[name], _ = bench._graph(fn)
    O.set_knobs(parallel_encoders=1)
    times = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for name, g in graphs.items():
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.reps)
    for name, t in times.items():
        print(json.dumps({"variant": name, "ms_median": round(statistics.median(t), 3), "all": [round(x, 3) for x in t]}))


if __name__ == "__main__":
    main()
