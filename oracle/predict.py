"""CPU restatement of the reference's test-time prediction
(code/train_fusion.py:484-632; flips code/train.py:916-923) -- TEST
INFRASTRUCTURE ONLY: imported by tests/ as the checker, never by the product.

The loops are the reference's: one forward per flip / MC pass, softmax,
mean and (unbiased) std over the stack, gating weights collapsed over any
spatial dims and averaged. The models are oracle.model modules; MC mode is
the reference's mc_enable (encoders' nn.Dropout modules on, BatchNorm eval,
train_fusion.py:445-481), the fusion model stays in eval.
Parity unpinned (the reference cannot be run here)."""
from __future__ import annotations

import torch


def tta_id(x):
    return x


def tta_flip_lr(x):
    return torch.flip(x, dims=[-1])


def tta_flip_ud(x):
    return torch.flip(x, dims=[-2])


def tta_flip_lrud(x):
    return torch.flip(torch.flip(x, dims=[-1]), dims=[-2])


TRANSFORMS = [tta_id, tta_flip_lr, tta_flip_ud, tta_flip_lrud]


def _collapse(gw):
    """train_fusion.py:514-524."""
    if gw.dim() == 5:
        return gw.mean(dim=(2, 3, 4))
    if gw.dim() == 4:
        return gw.mean(dim=(2, 3))
    if gw.dim() == 2:
        return gw
    raise ValueError(f"Unexpected gating weight shape: {gw.shape}")


def forward_from_inputs(dwi_model, dce_model, fusion_model, dwi, dce):
    """train_fusion.py:639-646 (masks=None)."""
    _, dwi_aux, dwi_mask = dwi_model(dwi)
    _, dce_aux, dce_mask = dce_model(dce)
    return fusion_model(dwi_aux["raw_feats"], dce_aux["raw_feats"], dwi_mask, dce_mask)


def mc_enable(model):
    """train_fusion.py:445-481: nn.Dropout modules train, BatchNorm eval."""
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.train()
    for m in model.modules():
        if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
            m.eval()


@torch.no_grad()
def predict_mc_dropout(dwi_model, dce_model, fusion_model, dwi, dce, passes=20, before_pass=None):
    """train_fusion.py:484-537. ``before_pass(i)`` (optional) runs before
    pass i -- the shared-mask check loads that pass's masks there."""
    states = {m: m.training for mod in (dwi_model, dce_model) for m in mod.modules()}
    mc_enable(dwi_model)
    mc_enable(dce_model)
    try:
        preds, gates = [], []
        for i in range(passes):
            if before_pass is not None:
                before_pass(i)
            logits, _, aux = forward_from_inputs(dwi_model, dce_model, fusion_model, dwi, dce)
            if aux["gating_weights"] is not None:
                gates.append(_collapse(aux["gating_weights"]))
            preds.append(torch.softmax(logits, dim=1))
    finally:
        for m, t in states.items():
            m.train(t)
    st = torch.stack(preds, 0)
    return st.mean(0), st.std(0), (torch.stack(gates, 0).mean(0) if gates else None)


@torch.no_grad()
def predict_tta(dwi_model, dce_model, fusion_model, dwi, dce, transforms=None):
    """train_fusion.py:541-587."""
    preds, gates = [], []
    for t in transforms or TRANSFORMS:
        logits, _, aux = forward_from_inputs(dwi_model, dce_model, fusion_model, t(dwi), t(dce))
        preds.append(torch.softmax(logits, dim=1))
        gates.append(_collapse(aux["gating_weights"]))
    st = torch.stack(preds, 0)
    return st.mean(0), st.std(0), torch.stack(gates, 0).mean(0)


@torch.no_grad()
def predict_tta_mc(dwi_model, dce_model, fusion_model, dwi, dce, transforms=None, passes=10):
    """train_fusion.py:591-632: per flip the MC mean, then mean / std over flips."""
    means, gates = [], []
    for t in transforms or TRANSFORMS:
        m, _, g = predict_mc_dropout(dwi_model, dce_model, fusion_model, t(dwi), t(dce), passes)
        means.append(m)
        gates.append(_collapse(g))
    st = torch.stack(means, 0)
    return st.mean(0), st.std(0), torch.stack(gates, 0).mean(0)
