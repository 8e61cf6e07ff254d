#!/usr/bin/env python3
"""Mode-B gradient precision at the real widths (config-3 shapes, B=4 S=256,
dropout 0): per-tensor relative L2 error against a float64 evaluation of the
CPU oracle for
  * the oracle in fp32 (the conditioning yardstick),
  * the oracle under CPU bf16 autocast (the reference's own "bf16-mixed" AMP),
  * the HIP path in the f32 parity mode,
  * the HIP path in the bf16 throughput mode,
grouped by where the tensor sits in the backward (fusion, encoder heads,
backbone stages). Writes one JSON to gpurun_out/grad_precision.json.

    python tools/grad_precision.py [--batch 4] [--size 256]
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as MG  # noqa: E402
import model_module as MM  # noqa: E402
import parameters as PR  # noqa: E402
import train_fusion as TF  # noqa: E402
from oracle import losses as OL  # noqa: E402
from selector_helpers import get_classification_loss  # noqa: E402


def group_of(name):
    if name.startswith("fusion."):
        return "fusion"
    for tag in ("layer4", "layer3", "layer2", "layer1"):
        if f"._orig_mod.{tag}." in name:
            return "backbone." + tag
    if "._orig_mod." in name:
        return "backbone.stem"
    if "backbone_adapter.necks" in name:
        return "necks"
    if "modality_attention" in name:
        return "input_gate"
    return "heads"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--no-f64", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    P = copy.deepcopy(PR.default_parameters())
    P["dwi_model_parameters"]["dropout"] = 0.0
    P["dwi_model_parameters"]["input_size"] = a.size
    P["backbone_freeze_on_start"] = False
    dwi, dwi_r = MG.seeded_encoder(P, "dwi", 14, 61)
    dce, dce_r = MG.seeded_encoder(P, "dce", 6, 62)
    fm, fr = MG.seeded_fusion(P, 63)
    bt = MG.volume_batch(a.batch, a.size, 13)
    cw = OL.class_weights_from_labels(torch.arange(1024) % 4)
    dev = torch.device("cuda", 0)

    def oracle_grads(dtype=None, autocast=False):
        m = [copy.deepcopy(x) for x in (dwi_r, dce_r, fr)]
        b = bt
        c = cw
        if dtype is not None:
            m = [x.to(dtype) for x in m]
            b = tuple(t.to(dtype) if t.is_floating_point() else t for t in bt)
            c = cw.to(dtype)
        for x in m:
            x.train()
        t0 = time.time()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            out = OL.fusion_shared_step(m[0], m[1], m[2], b, P, c)
        out["total"].float().backward()
        g = {}
        for tag, x in zip(("dwi.", "dce.", "fusion."), m):
            for n, p in x.named_parameters():
                if p.grad is not None:
                    g[tag + n] = p.grad.double()
        return g, float(out["total"]), time.time() - t0

    def product_grads(dtype):
        ms = [copy.deepcopy(x) for x in (dwi, dce, fm)]
        for x in ms:
            MM.set_compute_dtype(x, dtype)
        crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", dev)
        lm = TF.LightningFusionModel(ms[0].to(dev), ms[1].to(dev), ms[2].to(dev), P, crit)
        lm.train()
        loss = lm.training_step(tuple(t.to(dev) for t in bt))
        loss.backward()
        g = {}
        for tag, x in zip(("dwi.", "dce.", "fusion."), ms):
            for n, p in x.named_parameters():
                if p.grad is not None:
                    g[tag + n] = p.grad.detach().double().cpu()
        return g, float(loss)

    runs = {}
    runs["oracle_fp32"] = oracle_grads()
    runs["oracle_bf16_autocast"] = oracle_grads(autocast=True)
    if not a.no_f64:
        runs["oracle_fp64"] = oracle_grads(torch.float64)
    runs["hip_f32"] = product_grads(torch.float32)
    runs["hip_bf16"] = product_grads(torch.bfloat16)
    truth_key = "oracle_fp64" if not a.no_f64 else "oracle_fp32"
    truth = runs[truth_key][0]
    report = {"truth": truth_key, "batch": a.batch, "size": a.size,
              "losses": {k: v[1] for k, v in runs.items()}}
    for k, (g, _, *rest) in runs.items():
        if k == truth_key:
            continue
        groups = {}
        num = den = 0.0
        for n, t in truth.items():
            if n not in g:
                continue
            d = (g[n].reshape(t.shape) - t)
            num += d.pow(2).sum().item()
            den += t.pow(2).sum().item()
            tn = t.norm().item()
            if tn == 0:
                continue
            groups.setdefault(group_of(n.split(".", 1)[1] if not n.startswith("fusion.") else n), []).append(
                d.norm().item() / tn)
        report[k] = {"all": (num / max(den, 1e-300)) ** 0.5,
                     "groups_median": {gk: float(np.median(v)) for gk, v in sorted(groups.items())}}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "grad_precision.json"), "w") as f:
        json.dump(report, f, indent=1)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
