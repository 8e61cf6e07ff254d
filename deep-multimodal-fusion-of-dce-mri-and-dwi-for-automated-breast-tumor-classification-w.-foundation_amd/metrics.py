"""Epoch metrics of the fusion loop (train_fusion.py:56-79, :382-405):
macro one-vs-rest AUROC (torchmetrics MulticlassAUROC, average="macro"),
accuracy and the confusion matrix, over predictions all-gathered from every
data-parallel rank (dmf_dp.allgather_rows)."""
from __future__ import annotations

import torch


def _binary_auroc(score, target):
    """Exact AUROC with tie handling (average rank / Mann-Whitney U)."""
    n_pos = int(target.sum().item())
    n_neg = target.numel() - n_pos
    if n_pos == 0 or n_neg == 0:
        return float("nan")
    order = torch.argsort(score, stable=True)
    s = score[order]
    ranks = torch.empty_like(s, dtype=torch.float64)
    i = 0
    n = s.numel()
    vals = s.tolist()
    while i < n:
        j = i
        while j + 1 < n and vals[j + 1] == vals[i]:
            j += 1
        ranks[i:j + 1] = (i + j) / 2.0 + 1.0
        i = j + 1
    r = torch.empty_like(ranks)
    r[order] = ranks
    pos_rank_sum = r[target.bool()].sum().item()
    return (pos_rank_sum - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg)


def multiclass_auroc(probs, labels, num_classes=None):
    """Macro one-vs-rest AUROC; classes absent from ``labels`` are skipped
    (torchmetrics warns and scores them 0 -- noted in DESIGN.md)."""
    probs = probs.detach().double().cpu()
    labels = labels.detach().long().cpu()
    k = num_classes or probs.shape[1]
    aucs = []
    for c in range(k):
        a = _binary_auroc(probs[:, c], (labels == c).double())
        if a == a:
            aucs.append(a)
    return sum(aucs) / len(aucs) if aucs else float("nan")


def confusion_matrix(preds, labels, num_classes):
    cm = torch.zeros(num_classes, num_classes, dtype=torch.long)
    for p, t in zip(preds.tolist(), labels.tolist()):
        cm[t, p] += 1
    return cm
