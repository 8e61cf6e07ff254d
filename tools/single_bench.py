#!/usr/bin/env python3
"""Single-modality training-step throughput (reference
train.py:294-466): LightningSingleModel.training_step -> backward -> AdamW on
one encoder, every parameter trainable (the encoder pre-training phase before
fusion), config-3 shapes (B=32, S=256), bf16, synthetic volumes, random-init
weights. Eager launches (no hipGraph) -- the same kernels as bench.py's mode
B encoder half. Prints one JSON line.

    python tools/single_bench.py [--method dwi|dce] [--batch 32] [--steps 10]
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
    ap.add_argument("--method", choices=["dwi", "dce"], default="dwi")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import foundation_model as FM
    import model_module as MM
    import train as TR
    from dmf_optim import FusedAdamW
    from selector_helpers import get_classification_loss

    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = a.size
    P["dwi_model_parameters"]["compute_dtype"] = torch.bfloat16
    cin = P[f"{a.method}_channel_num"]
    torch.manual_seed(0)
    bb = FM.build_medical_backbone(P, "cpu", a.method, cin)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone(a.method, P, bb), True).to(dev)
    crit = get_classification_loss(P, torch.arange(1024) % P["class_num"], a.method, dev)
    lm = TR.LightningSingleModel(model=enc, method=a.method, criterion_clf=crit, parameters_dict=P)
    lm.train()
    opt = FusedAdamW(lm.parameters(), lr=1e-4, weight_decay=4e-5)
    dwi, dce, masks, labels = bench.synthetic_batch(a.batch, a.size, dev, 11, cd=P["dwi_channel_num"],
                                                    cc=P["dce_channel_num"])
    x = dwi if a.method == "dwi" else dce

    def step():
        opt.zero_grad(set_to_none=False)
        loss = lm.training_step((x, masks, labels))
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        loss = step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    print(json.dumps({
        "metric": f"single-modality ({a.method}) training volumes/s (fwd+bwd+AdamW, all trainable)",
        "value": round(a.batch / ms * 1e3, 2), "unit": "volumes/s", "ms_per_step": round(ms, 3),
        "batch": a.batch, "size": a.size, "channels": cin, "steps": a.steps, "dtype": "bf16",
        "hipgraph": False, "loss": round(loss.item(), 5),
        "data": "synthetic config-3 volumes, random-init weights"}))


if __name__ == "__main__":
    main()
