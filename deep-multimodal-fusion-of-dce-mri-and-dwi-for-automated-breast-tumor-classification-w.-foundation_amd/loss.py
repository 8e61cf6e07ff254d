"""Criteria -- MI355X build of the reference's ``code/loss.py``.

Same class names, constructor arguments and forward(logits, targets)
contracts; forward and gradient are fused HIP kernels (csrc/losses.hip).
"""
from __future__ import annotations

import torch
import torch.nn as nn

import dmf_native as N
import dmf_ops as O


def proj_cosine_loss(a, b, eps=1e-8):
    """loss.py:7-9 (not on the fusion path; plain tensor math)."""
    na = a.norm(dim=1).clamp_min(eps)
    nb = b.norm(dim=1).clamp_min(eps)
    return (1.0 - (a * b).sum(1) / (na * nb)).mean()


class SoftDiceLoss(nn.Module):
    """loss.py:45-62: 1 - mean_b (2*sum(p*t) + eps) / (sum p + sum t + eps), p = sigmoid."""

    def __init__(self, eps=1e-6):
        super().__init__()
        self.eps = eps

    def forward(self, logits, targets):
        return O.soft_dice(logits, targets, self.eps)


class DiceBCELoss(nn.Module):
    """loss.py:11-43 (foreground Dice without eps in the numerator + BCE)."""

    def __init__(self, bce_weight=1.0, dice_weight=1.0, eps=1e-6):
        super().__init__()
        self.bce_weight = bce_weight
        self.dice_weight = dice_weight
        self.eps = eps

    def forward(self, pred_logits, target):
        return O.dice_bce(pred_logits, target, self.bce_weight, self.dice_weight, self.eps)


class SoftWeightedFocalLoss(nn.Module):
    """loss.py:157-187: -sum_c t_c * w_c * (1 - p_c)^gamma * log p_c, mean over rows."""

    def __init__(self, gamma=2.0, class_weights=None, reduction="mean"):
        super().__init__()
        self.gamma = gamma
        self.reduction = reduction
        self.class_weights = class_weights.reshape(1, -1) if class_weights is not None else None

    def forward(self, logits, targets):
        cw = None
        if self.class_weights is not None:
            cw = self.class_weights.to(device=logits.device, dtype=torch.float32).reshape(-1).contiguous()
        return O.focal_loss(logits, targets, self.gamma, cw, self.reduction)


class SoftFocalLoss(SoftWeightedFocalLoss):
    """loss.py:133-155 (no class weights)."""

    def __init__(self, gamma=2.0, reduction="mean"):
        super().__init__(gamma=gamma, class_weights=None, reduction=reduction)


class LabelSmoothing(nn.Module):
    """loss.py:190-213: dense targets filled with smoothing/(K-1), 1-smoothing at the label."""

    def __init__(self, classes, smoothing=0.0, dim=-1):
        super().__init__()
        self.confidence = 1.0 - smoothing
        self.smoothing = smoothing
        self.cls = classes
        self.dim = dim

    def forward(self, pred, target):
        return O.label_smooth(target, self.cls, self.smoothing)


class FocalLoss(nn.Module):
    """loss.py:66-84 (hard-label focal CE, scalar alpha)."""

    def __init__(self, alpha=1, gamma=2, reduction="mean"):
        super().__init__()
        self.alpha, self.gamma, self.reduction = alpha, gamma, reduction

    def forward(self, inputs, targets):
        return O.focal_ce(inputs, targets, self.gamma, self.alpha, None, self.reduction)


class WeightedFocalLoss(nn.Module):
    """loss.py:87-130 (hard-label focal CE with per-class alpha)."""

    def __init__(self, alpha=None, gamma=2, reduction="mean"):
        super().__init__()
        self.alpha, self.gamma, self.reduction = alpha, gamma, reduction

    def forward(self, inputs, targets):
        if targets.ndim > 1:
            return self._soft(inputs, targets)
        a = self.alpha
        if a is None:
            return O.focal_ce(inputs, targets, self.gamma, 1.0, None, self.reduction)
        if isinstance(a, (int, float)):
            return O.focal_ce(inputs, targets, self.gamma, float(a), None, self.reduction)
        return O.focal_ce(inputs, targets, self.gamma, 1.0, a.to(inputs.device).float().contiguous(), self.reduction)

    def _soft(self, inputs, targets):
        """loss.py:96-128 with soft / smoothed targets: ce = F.cross_entropy on
        the probabilities (-sum t log p), pt = exp(-ce), focal = alpha *
        (1 - pt)^gamma * ce, per-class alpha looked up at argmax(t). Off the
        default path (get_classification_loss builds SoftWeightedFocalLoss):
        device tensor ops."""
        N.require_cuda(inputs, targets)
        ce = -(targets.float() * torch.log_softmax(inputs.float(), dim=1)).sum(1)
        fl = (1 - torch.exp(-ce)) ** self.gamma * ce
        a = self.alpha
        if isinstance(a, (int, float)):
            fl = a * fl
        elif a is not None:
            fl = a.to(inputs.device).float().gather(0, targets.argmax(dim=1).long()) * fl
        if self.reduction == "mean":
            return fl.mean()
        if self.reduction == "sum":
            return fl.sum()
        return fl
