#!/usr/bin/env python3
"""Config-5 bf16 logit error against the fp32 oracle under variants of the forward path
(tests/test_gpu_config5_full.py part 2, same weights, batch and yardstick), to find which
forward change moves the relative L2 error:

    python tools/config5_numerics_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

import dmf_ops as O  # noqa: E402
import dmf_tokens as D  # noqa: E402
import model_module as MM  # noqa: E402
import train_fusion as TF  # noqa: E402
from oracle import losses as OL  # noqa: E402
from selector_helpers import get_classification_loss  # noqa: E402
import test_gpu_config5_full as T  # noqa: E402
from test_gpu_parity import _fusion_pair, batch, build_pair  # noqa: E402


def main():
    P = T._config5_params()
    dwi_m, dwi_r, P1 = build_pair(P, "dwi", 14, 51)
    dce_m, dce_r, _ = build_pair(P, "dce", 6, 52)
    P = P1
    fm, fr = _fusion_pair(P, 53)
    T._no_dropout(dwi_m, dce_m, fm, dwi_r, dce_r, fr)
    train_labels = torch.arange(64) % 4
    crit = get_classification_loss(P, train_labels, "fusion", "cuda")
    lm = TF.LightningFusionModel(dwi_m, dce_m, fm, P, crit)
    lm.train()
    for m in (dwi_r, dce_r, fr):
        m.train()
    bt = batch(2, 384, 19)
    bd = tuple(t.to("cuda") for t in bt)
    cw = OL.class_weights_from_labels(train_labels)
    torch.set_num_threads(16)
    with torch.no_grad():
        want = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)["logits"].float()
    yard = T.amp_yardstick((dwi_r, dce_r, fr), bt, P, cw, False)
    y_rel = T.rel_l2(yard, want)
    print(f"reference AMP yardstick rel L2 {y_rel:.4f} (bar {1.5 * y_rel + 1e-2:.4f})", flush=True)
    for m in (dwi_m, dce_m, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    fa = D._FA_HEAD_DIM
    variants = [
        ("default", {}, fa),
        ("flash off (unfused attention, no-grad block)", {}, -1),
        ("token_fwd_fused off", {"token_fwd_fused": 0}, fa),
        ("two_pass_bn off", {"two_pass_bn": 0}, fa),
        ("token_fwd_fused off + two_pass_bn off", {"token_fwd_fused": 0, "two_pass_bn": 0}, fa),
    ]
    for name, knobs, fa_dim in variants:
        O.set_knobs(**knobs)
        D._FA_HEAD_DIM = fa_dim
        with torch.no_grad():
            _, lg, _, _ = lm._shared_step(bd, "train", return_preds=True)
        torch.cuda.synchronize()
        print(f"{name:45s} rel L2 {T.rel_l2(lg.float().cpu(), want):.4f}", flush=True)
        D._FA_HEAD_DIM = fa
        O.set_knobs(**{k: 1 for k in knobs})


if __name__ == "__main__":
    main()
