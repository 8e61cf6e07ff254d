"""fp32 CPU restatement of the fusion training step's criteria and the
``_shared_step`` loss assembly. TEST INFRASTRUCTURE ONLY. PARITY UNPINNED.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def label_smoothing(logits, target, classes, smoothing):
    """loss.py:190-213: fill smoothing/(K-1), put 1-smoothing at the label."""
    t = torch.full_like(logits, smoothing / (classes - 1))
    t.scatter_(1, target.long().unsqueeze(1), 1.0 - smoothing)
    return t


def soft_weighted_focal(logits, targets, gamma, class_weights=None, reduction="mean"):
    """loss.py:157-187."""
    if targets.dim() == 1:
        targets = F.one_hot(targets, logits.size(1)).float()
    logp = F.log_softmax(logits, dim=1)
    fw = (1 - logp.exp()) ** gamma
    if class_weights is not None:
        fw = fw * class_weights.view(1, -1)
    per = -(targets * fw * logp).sum(dim=1)
    return per.mean() if reduction == "mean" else (per.sum() if reduction == "sum" else per)


def soft_focal(logits, targets, gamma=2.0, reduction="mean"):
    """loss.py:133-155 (SoftWeightedFocal without class weights)."""
    return soft_weighted_focal(logits, targets, gamma, None, reduction)


def soft_dice(logits, targets, eps=1e-6):
    """loss.py:45-62."""
    p = torch.sigmoid(logits)
    dims = tuple(range(2, p.ndim))
    inter = (p * targets).sum(dims)
    union = p.sum(dims) + targets.sum(dims)
    return 1.0 - ((2.0 * inter + eps) / (union + eps)).mean()


def dice_bce(logits, target, bce_weight=1.0, dice_weight=1.0, eps=1e-6):
    """loss.py:11-43."""
    bce = F.binary_cross_entropy_with_logits(logits, target)
    p = torch.sigmoid(logits).reshape(logits.size(0), -1)
    t = target.reshape(target.size(0), -1)
    dice = 2.0 * (p * t).sum(1) / (p.sum(1) + t.sum(1) + eps)
    return bce_weight * bce + dice_weight * (1.0 - dice.mean())


def class_weights_from_labels(train_labels):
    """selector_helpers.py:25-41 (inverse class frequency, 'wfl')."""
    counts = torch.bincount(train_labels.long())
    return train_labels.numel() / (len(counts) * (counts.float() + 1e-6))


def charbonnier(pred, target, eps=1e-3):
    """train.py:1041-1042."""
    return torch.sqrt((pred - target) ** 2 + eps ** 2).mean()


def recon_image_loss(pred, target):
    """train.py:1043-1048."""
    return charbonnier(torch.sigmoid(pred).clamp(0, 1), target.clamp(0, 1))


def recon_list_loss(recons, image):
    """train_fusion.py:709-744."""
    if isinstance(recons, torch.Tensor):
        recons = [recons]
    recons = [r for r in recons if r is not None]
    if not recons:
        return torch.zeros((), dtype=image.dtype)
    tot = torch.zeros((), dtype=image.dtype)
    for r in recons:
        up = F.interpolate(r, size=image.shape[-2:], mode="bilinear", align_corners=False)
        if up.size(1) != image.size(1):
            up, tgt = up.mean(1, keepdim=True), image.mean(1, keepdim=True)
        else:
            tgt = image
        tot = tot + recon_image_loss(up, tgt)
    return tot / len(recons)


def mimic_feat_loss(s, t, eps=1e-6):
    """train.py:1033-1038 (teacher detached)."""
    s = F.normalize(s.flatten(1), dim=1)
    t = F.normalize(t.detach().flatten(1), dim=1)
    return (1.0 - (s * t).sum(1).clamp(-1 + eps, 1 - eps)).mean()


def feat_norm_loss(aux):
    """train.py:1021-1030; the fusion aux has no raw_feats -> 0."""
    feats = aux.get("raw_feats")
    if feats is None:
        return torch.zeros(())
    return sum(f.pow(2).mean() for f in feats)


def fusion_shared_step(dwi_model, dce_model, fusion_model, batch, P, class_weights, epoch=0,
                       phase="train"):
    """train_fusion.py:204-321 -> dict of the loss terms and ``total``.

    ``P`` is the parameters dict (parameters_generate.py layout)."""
    fp = P["fusion_model_parameters"]
    dwi, dce, masks, labels = batch
    labels = labels.long()
    is_train = phase == "train"
    aux_w = max(0.0, 1 - epoch / P["aux_loss_weight_epoch_limit"]) if P["use_simple_aux_loss_scheduling"] else 1.0
    _, dwi_aux, dwi_mask = dwi_model(dwi)
    _, dce_aux, dce_mask = dce_model(dce)
    logits, fmask, aux = fusion_model(dwi_aux["raw_feats"], dce_aux["raw_feats"], dwi_mask, dce_mask)
    K = P["class_num"]
    gamma = fp["classification_loss_parameters"]["gamma"]
    if is_train:
        tgt = label_smoothing(logits, labels, K, fp["label_smoothing_alpha"])
    else:
        tgt = labels
    out = {"logits": logits, "fused_mask_logits": fmask, "aux": aux,
           "dwi_mask_pred": dwi_mask, "dce_mask_pred": dce_mask}
    cls = soft_weighted_focal(logits, tgt, gamma, class_weights)
    total = cls
    mk = fp["mask_parameters"]
    mask = (soft_dice(dwi_mask, masks) + soft_dice(dce_mask, masks) + soft_dice(fmask, masks)) / 3
    if is_train:
        total = total + mk["lambda_mask"] * mask
    if fp["feat_norm_reg_enabled"] and is_train:
        total = total + feat_norm_loss(aux) * fp["lambda_feat_norm"]
    recon = torch.zeros(())
    mimic = torch.zeros(())
    if aux_w > 0 and fp["recon_enabled"] and is_train:
        fused_in = torch.cat([dwi, dce], 1)
        recon = (recon_list_loss(dwi_aux["recon_feats"], dwi) + recon_list_loss(dce_aux["recon_feats"], dce)
                 + recon_list_loss(aux["recon_fused"], fused_in)) / 3
        total = total + fp["lambda_recon"] * recon * aux_w
        pf = aux["proj_fused"]
        if fp["mimic_enabled"] and pf is not None and len(pf) >= 4:
            mimic = (mimic_feat_loss(pf[0], pf[1]) + mimic_feat_loss(pf[2], pf[3])) / 2
            total = total + fp["lambda_mimic"] * mimic * aux_w
    out.update(cls=cls, mask=mask, recon=recon, mimic=mimic, total=total)
    return out


def single_shared_step(model, batch, P, class_weights, method="dwi", epoch=0, phase="train"):
    """train.py:294-466 (LightningSingleModel._shared_step + compute_aux_losses)
    -> dict of the loss terms and ``total``.

    Restated quirks: the recon/mimic values that compute_aux_losses returns in
    training are already multiplied by lambda * aux_w (train.py:458-460) and
    _shared_step multiplies them by lambda * aux_w again (:400-403); recon terms
    are SUMMED over recon_feats (:444-450), not averaged as in the fusion step;
    mimic pairs (p1, p1_r), (p2, p2_r) with rows = batch items (:453-455)."""
    mp = P[f"{method}_model_parameters"]
    inputs, masks, labels = batch
    labels = labels.long()
    is_train = phase == "train"
    aux_w = max(0.0, 1 - epoch / P["aux_loss_weight_epoch_limit"]) if P["use_simple_aux_loss_scheduling"] else 1.0
    logits, aux, mask_out = model(inputs, masks)
    K = P["class_num"]
    gamma = mp["classification_loss_parameters"]["gamma"]
    tgt = label_smoothing(logits, labels, K, mp["label_smoothing_alpha"]) if is_train else labels
    cls = soft_weighted_focal(logits, tgt, gamma, class_weights)
    total = cls
    feat_norm = torch.zeros(())
    if mp["feat_norm_reg_enabled"]:
        feat_norm = feat_norm_loss(aux)
        if is_train:
            total = total + feat_norm * mp["lambda_feat_norm"]
    mask = soft_dice(mask_out, masks)
    if is_train:
        total = total + mp["mask_parameters"]["lambda_mask"] * mask
    recon = torch.zeros(())
    mimic = torch.zeros(())
    if mp["recon_enabled"] and aux_w > 0:
        for r in aux["recon_feats"]:
            if r is None:
                continue
            up = F.interpolate(r, size=inputs.shape[-2:], mode="bilinear", align_corners=False)
            tgt_img = inputs.mean(1, keepdim=True) if up.size(1) == 1 and inputs.size(1) > 1 else inputs
            recon = recon + recon_image_loss(up, tgt_img)
        pp = aux.get("proj_pairs")
        if mp["mimic_enabled"] and pp is not None and len(pp) >= 4:
            mimic = mimic_feat_loss(pp[0], pp[1]) + mimic_feat_loss(pp[2], pp[3])
        if is_train:
            recon = recon * mp["lambda_recon"] * aux_w
            mimic = mimic * mp["lambda_mimic"] * aux_w
            total = total + mp["lambda_recon"] * recon * aux_w + mp["lambda_mimic"] * mimic * aux_w
    return {"logits": logits, "aux": aux, "mask_pred": mask_out, "cls": cls, "mask": mask, "recon": recon,
            "mimic": mimic, "feat_norm": feat_norm, "total": total}
