"""Shared training helpers -- MI355X build of the pieces of the reference's
``code/train.py`` that the fusion step uses (train.py:287-288 encoder
wrapper forward, :916-923 TTA flips, :991-1048 loss helpers).

The Lightning single-model loop itself is outside the hot-path scope
(SURVEY.md 8(f) rank 4); ``LightningSingleModel`` here is the thin wrapper the
fusion step calls (``self.dwi_model(x)`` -> ``self.model(x, masks)``) and keeps
the ``model.`` state_dict prefix of the reference's checkpoints.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import dmf_ops as O


class LightningSingleModel(nn.Module):
    """Encoder wrapper (train.py:19-288 subset): forward(x, masks=None) -> model(x, masks)."""

    def __init__(self, model, parameters_dict=None, method="dwi", **kwargs):
        super().__init__()
        self.model = model
        self.parameters_dict = parameters_dict
        self.method = method

    def forward(self, x, masks=None):
        return self.model(x, masks)


# ------------------------------------------------------------------ TTA flips (train.py:916-923)
def tta_id(x):
    return x


def inv_tta_id(x):
    return x


def tta_flip_lr(x):
    return torch.flip(x, dims=[-1])


def inv_tta_flip_lr(x):
    return torch.flip(x, dims=[-1])


def tta_flip_ud(x):
    return torch.flip(x, dims=[-2])


def inv_tta_flip_ud(x):
    return torch.flip(x, dims=[-2])


def tta_flip_lrud(x):
    return torch.flip(torch.flip(x, dims=[-1]), dims=[-2])


def inv_tta_flip_lrud(x):
    return torch.flip(torch.flip(x, dims=[-1]), dims=[-2])


# ------------------------------------------------------------------ loss helpers
def compute_attn_energy_loss(aux, device):
    """train.py:991-1000 (off by default: attn_reg_enabled=False)."""
    a = aux.get("mask_attn_map", None)
    if a is None:
        return torch.zeros((), device=device)
    return a.float().abs().mean()


def compute_feature_consistency_loss(aux, device):
    """train.py:1001-1018 (off by default)."""
    if "proj_pairs" not in aux or aux["proj_pairs"] is None:
        return torch.zeros((), device=device)
    p1, _, p2, _ = aux["proj_pairs"]
    p1, p2 = p1.float(), p2.float()
    p2u = torch.nn.functional.interpolate(p2, size=p1.shape[-2:], mode="bilinear", align_corners=False)
    n1 = p1 / (p1.norm(dim=1, keepdim=True) + 1e-6)
    n2 = p2u / (p2u.norm(dim=1, keepdim=True) + 1e-6)
    return torch.nn.functional.mse_loss(n1, n2)


def compute_feat_norm_loss(aux, device):
    """train.py:1021-1030: sum of mean(f^2) over aux['raw_feats'] (0 when absent,
    as for the fusion aux)."""
    feats = aux.get("raw_feats", None)
    if feats is None:
        return torch.zeros((), device=device)
    return sum(f.float().pow(2).mean() for f in feats)


def mimic_feat_loss(s_feat, t_feat, eps=1e-6):
    """train.py:1033-1038: per-row (dim 0 of s_feat) cosine after flatten(1);
    teacher detached. Rows of a [C,H,W] item are channels."""
    return O.mimic(s_feat, t_feat.detach())


def charbonnier_loss(pred, target, eps=1e-3):
    """train.py:1041-1042 (generic tensors)."""
    return torch.mean(torch.sqrt((pred - target) ** 2 + eps ** 2))


def recon_image_loss(pred, target):
    """train.py:1043-1048 (generic tensors)."""
    return charbonnier_loss(torch.sigmoid(pred).clamp(0, 1), target.clamp(0, 1))
