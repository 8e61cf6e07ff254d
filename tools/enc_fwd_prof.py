#!/usr/bin/env python3
"""The north-star workload alone: the DWI + DCE encoder forward of the fusion
step (a1-a10, train-mode BN, no autograd -- mode A at epoch 0), B=32, S=256,
bf16, captured once as a hipGraph and replayed --reps times. Run it under
`rocprofv3 --kernel-trace --stats` for a per-kernel split of one forward
(divide the totals by --reps); prints the HIP-event time per forward.

    python tools/enc_fwd_prof.py [--reps 20] [--batch 32] [--serial] [--knob name=VAL ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import bench  # noqa: E402
import parameters as PR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--serial", action="store_true", help="one stream (no DCE side stream)")
    ap.add_argument("--knob", action="append", default=[], help="dmf_ops.set_knobs name=VAL")
    a = ap.parse_args()
    import dmf_ops as O
    for kv in a.knob:
        k, v = kv.split("=")
        O.set_knobs(**{k: int(v)})
    if a.serial:
        O.set_knobs(parallel_encoders=0)
    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = a.size
    lm = bench.build(P, dev, torch.bfloat16, "A", seed=0)
    dwi, dce, _, _ = bench.synthetic_batch(a.batch, a.size, dev, 2)

    def fwd():
        with torch.no_grad():
            return lm._encode(dwi, dce)

    g, _ = bench._graph(fwd)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    t_roof = bench.T_ROOF_ENC_FWD_MS_B32 * a.batch / 32
    print(json.dumps({"encoder_forward_ms": round(ms, 3), "volumes_per_s": round(a.batch / ms * 1e3, 1),
                      "t_roof_ms": t_roof, "frac": round(t_roof / ms, 4), "reps": a.reps, "serial": a.serial}))


if __name__ == "__main__":
    main()
