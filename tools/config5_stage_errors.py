#!/usr/bin/env python3
"""Where config 5's bf16 error grows: the DWI encoder (hybrid TransformerStage, S=384, B=2, train-mode
BN) of tests/test_gpu_config5_full.py, forward hooks on every named module of the HIP model (bf16),
the fp32 oracle and the oracle under CPU bf16 autocast (the reference's mixed precision). Prints, in
call order, each module output's relative L2 error against the fp32 oracle for the HIP path and for
the autocast yardstick.

    python tools/config5_stage_errors.py [--depth 4]
"""
import argparse
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

import model_module as MM  # noqa: E402
import test_gpu_config5_full as T  # noqa: E402
from test_gpu_parity import batch, build_pair  # noqa: E402


def _first(o):
    if torch.is_tensor(o):
        return o
    if isinstance(o, (tuple, list)):
        for x in o:
            t = _first(x)
            if t is not None:
                return t
    return None


def record(model, depth):
    out, order = {}, []

    def hook(name):
        def f(_m, _i, o):
            t = _first(o)
            if t is not None and t.is_floating_point() and name not in out:
                out[name] = t.detach().float().cpu()
                order.append(name)
        return f
    hs = [m.register_forward_hook(hook(n)) for n, m in model.named_modules()
          if n and n.count(".") < depth]
    return out, order, hs


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--fusion", action="store_true", help="the FusionModel inside the whole shared step instead")
    a = ap.parse_args()
    if a.fusion:
        return fusion(a)
    P = T._config5_params()
    enc, ref, _ = build_pair(P, "dwi", 14, 51)
    T._no_dropout(enc, ref)
    enc.train()
    ref.train()
    amp = copy.deepcopy(ref)
    MM.set_compute_dtype(enc, torch.bfloat16)
    dwi, _, _, _ = batch(2, 384, 19)
    torch.set_num_threads(16)
    o_hip, order, h1 = record(enc, a.depth)
    o_ref, _, h2 = record(ref, a.depth)
    o_amp, _, h3 = record(amp, a.depth)
    with torch.no_grad():
        enc(dwi.to("cuda"))
        torch.cuda.synchronize()
        ref(dwi)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            amp(dwi)
    for h in h1 + h2 + h3:
        h.remove()
    report(order, o_hip, o_ref, o_amp)


def fusion(a):
    import train_fusion as TF
    from oracle import losses as OL
    from selector_helpers import get_classification_loss
    from test_gpu_parity import _fusion_pair

    P = T._config5_params()
    dwi_m, dwi_r, P1 = build_pair(P, "dwi", 14, 51)
    dce_m, dce_r, _ = build_pair(P, "dce", 6, 52)
    P = P1
    fm, fr = _fusion_pair(P, 53)
    T._no_dropout(dwi_m, dce_m, fm, dwi_r, dce_r, fr)
    labels = torch.arange(64) % 4
    crit = get_classification_loss(P, labels, "fusion", "cuda")
    lm = TF.LightningFusionModel(dwi_m, dce_m, fm, P, crit)
    lm.train()
    for m in (dwi_r, dce_r, fr):
        m.train()
    for m in (dwi_m, dce_m, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    bt = batch(2, 384, 19)
    bd = tuple(t.to("cuda") for t in bt)
    cw = OL.class_weights_from_labels(labels)
    torch.set_num_threads(16)
    mods = [copy.deepcopy(m) for m in (dwi_r, dce_r, fr)]
    o_hip, order, h1 = record(fm, a.depth)
    o_ref, _, h2 = record(fr, a.depth)
    o_amp, _, h3 = record(mods[2], a.depth)
    # the classifier head (AdaptiveAvgPool -> Flatten -> Linear): its pooled input and the logits; the HIP
    # model calls it functionally (O.gap + O.linear), so O.linear is wrapped for the head's weight
    import dmf_ops as O
    orig_linear = O.linear

    def linear(x, w, b=None, *args, **kw):
        y = orig_linear(x, w, b, *args, **kw)
        if w is fm.classifier[2].weight:
            o_hip.setdefault("classifier.pooled", x.detach().float().cpu())
            o_hip.setdefault("classifier.logits", y.detach().float().cpu())
        return y
    O.linear = linear
    order += ["classifier.pooled", "classifier.logits"]
    # the oracle calls F.linear on the head's weight (oracle/model.py FusionModel.forward)
    import torch.nn.functional as F
    orig_f_linear = F.linear
    heads = {id(fr.classifier[2].weight): o_ref, id(mods[2].classifier[2].weight): o_amp}

    def f_linear(x, w, b=None):
        y = orig_f_linear(x, w, b)
        d = heads.get(id(w))
        if d is not None:
            d.setdefault("classifier.pooled", x.detach().float())
            d.setdefault("classifier.logits", y.detach().float())
        return y
    F.linear = f_linear
    with torch.no_grad():
        lm._shared_step(bd, "train", return_preds=True)
        torch.cuda.synchronize()
        OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            OL.fusion_shared_step(mods[0], mods[1], mods[2], bt, P, cw, epoch=0)
    O.linear = orig_linear
    F.linear = orig_f_linear
    for h in h1 + h2 + h3:
        h.remove()
    report(order, o_hip, o_ref, o_amp)
    for k in ("classifier.pooled", "classifier.logits"):
        print(k, "hip", o_hip[k].flatten()[:8].tolist())
        print(k, "ref", o_ref[k].flatten()[:8].tolist())
        print(k, "amp", o_amp[k].flatten()[:8].tolist())


def report(order, o_hip, o_ref, o_amp):
    print(f"{'module':60s} {'shape':>22s} {'hip':>8s} {'amp':>8s} {'ratio':>6s}")
    for n in order:
        if n not in o_ref or n not in o_amp or o_ref[n].numel() != o_hip[n].numel():
            continue
        r = o_ref[n]
        eh = rel(o_hip[n].reshape(r.shape), r)
        ea = rel(o_amp[n].reshape(r.shape), r) if o_amp[n].numel() == r.numel() else float("nan")
        print(f"{n:60s} {str(tuple(r.shape)):>22s} {eh:8.4f} {ea:8.4f} {eh / max(ea, 1e-12):6.2f}", flush=True)


if __name__ == "__main__":
    main()
