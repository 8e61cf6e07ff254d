"""Shared training helpers -- MI355X build of the pieces of the reference's
``code/train.py`` that the fusion step uses (train.py:287-288 encoder
wrapper forward, :916-923 TTA flips, :991-1048 loss helpers).

``LightningSingleModel`` carries the single-modality training step
(train.py:294-466) and is also the encoder wrapper
the fusion step calls (``self.dwi_model(x)`` -> ``self.model(x, masks)``),
keeping the ``model.`` state_dict prefix of the reference's checkpoints.
"""
from __future__ import annotations

import torch
import torch.nn as nn

import dmf_ops as O
from loss import LabelSmoothing


class LightningSingleModel(nn.Module):
    """Single-modality training module (train.py:19-466) without the Lightning
    runtime: same constructor, ``forward(x, masks)`` and
    ``_shared_step(batch, batch_idx, phase, return_preds)`` contract; a driver
    calls ``training_step`` -> backward -> optimizer step. Also the encoder
    wrapper the fusion step calls (``self.dwi_model(x)`` -> ``self.model(x,
    masks)``), keeping the ``model.`` state_dict prefix of the reference's
    checkpoints. Loss terms run in the fused criterion kernels
    (csrc/losses.hip): focal + smoothing, Dice, the recon terms of one step
    in one launch, and the item-row mimic in one launch per pair."""

    def __init__(self, model, method="dwi", criterion_clf=None, optimizer_fn=None, scheduler_fn=None,
                 parameters_dict=None, paths=None):
        super().__init__()
        self.model = model
        self.method = method
        self.criterion_clf = criterion_clf
        self.optimizer_fn = optimizer_fn
        self.scheduler_fn = scheduler_fn
        self.parameters_dict = parameters_dict
        self.paths = paths
        self.current_epoch = 0
        self.global_step = 0
        self.optimizer = None
        self.scheduler = None
        self.last_metrics = {}
        self.transforms_list = [tta_id, tta_flip_lr, tta_flip_ud, tta_flip_lrud]
        if parameters_dict is None:
            return
        mp = parameters_dict[f"{method}_model_parameters"]
        self.model_params = mp
        self.recon_enabled = mp["recon_enabled"]
        self.lambda_recon = mp["lambda_recon"]
        self.mimic_enabled = mp["mimic_enabled"]
        self.lambda_mimic = mp["lambda_mimic"]
        self.class_num = parameters_dict["class_num"]
        self.attn_reg_enabled = mp["attn_reg_enabled"]
        self.lambda_attn_energy = mp["lambda_attn_energy"]
        self.lambda_feature_consistency = mp["lambda_feature_consistency"]
        self.feat_norm_reg_enabled = mp["feat_norm_reg_enabled"]
        self.lambda_feat_norm = mp["lambda_feat_norm"]
        mk = mp["mask_parameters"]
        self.mask_enabled = mk["mask"]
        self.lambda_mask = mk["lambda_mask"]
        self.label_smoother = (LabelSmoothing(self.class_num, mp["label_smoothing_alpha"])
                               if mp["label_smoothing_enabled"] else None)
        from selector_helpers import mask_criterion_selector
        self.mask_criterion = mask_criterion_selector(parameters_dict, method)
        self.use_aux_loss_sched = parameters_dict["use_simple_aux_loss_scheduling"]
        self.aux_loss_limit = parameters_dict["aux_loss_weight_epoch_limit"]

    @property
    def device(self):
        return next(self.model.parameters()).device

    def forward(self, x, masks=None):
        return self.model(x, masks)

    def step_signature(self):
        """The captured step's structure beyond the optimizer: the aux-loss
        gate (train.py:391, aux_w > 0)."""
        return (aux_weight_value(self) > 0.0,)

    def sync_step_scalars(self):
        """Write the aux-loss weight the captured step reads before a replay."""
        sync_aux_weight(self)

    def configure_optimizers(self):
        """train.py:190-224 (the grad_clip keys are returned but never
        honoured, quirk Q10)."""
        self.optimizer = self.optimizer_fn(self.model.parameters())
        if self.scheduler_fn is None:
            return self.optimizer
        sched = self.scheduler_fn(self.optimizer)
        self.scheduler = sched["scheduler"] if isinstance(sched, dict) and "scheduler" in sched else sched
        return {"optimizer": self.optimizer, "lr_scheduler": sched}

    def _shared_step(self, batch, batch_idx=0, phase="train", return_preds=False):
        """train.py:294-418 with compute_aux_losses (:423-466)."""
        is_train = phase == "train"
        if self.mask_enabled:
            inputs, masks, labels = batch
        else:
            inputs, labels = batch
            masks = None
        dev = self.device
        inputs = inputs.to(dev, non_blocking=True)
        labels = labels.to(dev, non_blocking=True).long()
        if masks is not None:
            masks = masks.to(dev, non_blocking=True)
        aux_w = aux_weight_value(self)

        outputs, aux, mask_output = self(inputs, masks)

        if self.label_smoother is not None:
            smoothed = self.label_smoother(outputs, labels)
        # Q7: `smoothed` is undefined in training without label smoothing, as in the reference
        clf_loss = self.criterion_clf(outputs, smoothed) if is_train else self.criterion_clf(outputs, labels)
        batch_loss = clf_loss

        if self.attn_reg_enabled and is_train:
            batch_loss = batch_loss + compute_attn_energy_loss(aux, dev) * self.lambda_attn_energy \
                + compute_feature_consistency_loss(aux, dev) * self.lambda_feature_consistency
        feat_norm = torch.zeros((), device=dev)
        if self.feat_norm_reg_enabled:
            feat_norm = compute_feat_norm_loss(aux, dev)
            if is_train:
                batch_loss = batch_loss + feat_norm * self.lambda_feat_norm

        mask_out_resized = None
        mask_loss = torch.zeros((), device=dev)
        if self.mask_enabled:
            if mask_output.shape[-2:] != masks.shape[-2:]:
                mask_out_resized = O.bilinear(mask_output, *masks.shape[-2:])
            else:
                mask_out_resized = mask_output
            mask_loss = self.mask_criterion(mask_output, masks)
            if is_train:
                batch_loss = batch_loss + self.lambda_mask * mask_loss

        recon_loss_val = torch.zeros((), device=dev)
        mimic_loss_val = torch.zeros((), device=dev)
        if self.recon_enabled and aux_w > 0.0:
            # the device scalar, not the float: a captured step replays with the current epoch's weight
            w = aux_weight_tensor(self, dev) if inputs.is_cuda else aux_w
            recon_loss_val, mimic_loss_val = self.compute_aux_losses(aux, inputs, w, is_train)
            if is_train:
                # the values are already lambda * aux_w weighted (train.py:458-460): weighted twice, as there
                batch_loss = batch_loss + (self.lambda_recon * recon_loss_val * w
                                           + self.lambda_mimic * mimic_loss_val * w)

        preds = outputs.argmax(dim=1)
        acc = (preds == labels).float().mean()
        self.last_metrics = {"loss": batch_loss.detach(), "acc": acc.detach(), "cls": clf_loss.detach(),
                             "mask": mask_loss.detach(), "recon": recon_loss_val.detach(),
                             "mimic": mimic_loss_val.detach(), "feat_norm": feat_norm.detach()}
        if return_preds:
            return batch_loss.detach(), outputs.detach(), aux, mask_out_resized
        return batch_loss

    def compute_aux_losses(self, aux, inputs, aux_w, is_train):
        """train.py:423-466: recon terms SUMMED over recon_feats (bilinear up to
        the input size vs the input's channel mean), mimic over (p1, p1_r) and
        (p2, p2_r) with rows = batch items; lambda * aux_w applied in training."""
        dev = inputs.device
        recon = torch.zeros((), device=dev)
        mimic = torch.zeros((), device=dev)
        if not torch.is_tensor(aux_w) and aux_w <= 0.0:  # a device weight is only passed while aux_w > 0
            return recon, mimic
        maps = [r for r in (aux.get("recon_feats", []) if aux is not None else []) if r is not None]
        if maps:
            if any(r.shape[1] != 1 for r in maps):
                raise NotImplementedError("multi-channel reconstructions are not on the reference path")
            tgt = O.channel_mean_map(inputs.detach())
            recon = O.recon_terms(maps, [0] * len(maps), tgt).sum()
        pp = aux.get("proj_pairs", None) if aux is not None else None
        if self.mimic_enabled and pp is not None and len(pp) >= 4:
            mimic = O.mimic_items(pp[0], pp[1]) + O.mimic_items(pp[2], pp[3])
        if is_train:
            recon = recon * self.lambda_recon * aux_w
            mimic = mimic * self.lambda_mimic * aux_w
        return recon, mimic

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True, **kwargs):
        """Lightning-layout .ckpt -> module (run_training.py:123-131); see run_training.py."""
        from run_training import load_from_checkpoint
        return load_from_checkpoint(cls, checkpoint_path, map_location=map_location, strict=strict, **kwargs)

    def training_step(self, batch, batch_idx=0):
        # every trainable conv weight's re-layouts for this step in one launch (dmf_ops.PrepPlan)
        O.PREP.prep_step(self)
        return self._shared_step(batch, batch_idx, "train")

    def validation_step(self, batch, batch_idx=0):
        loss, _, _, _ = self._shared_step(batch, batch_idx, phase="val", return_preds=True)
        return loss


# ------------------------------------------------------------------ aux-loss schedule
def aux_weight_value(module):
    """train_fusion.py:221-224 / train.py:321-324: max(0, 1 - epoch / limit)
    under the simple aux-loss schedule, else 1."""
    if not module.use_aux_loss_sched:
        return 1.0
    return max(0.0, 1 - module.current_epoch / module.aux_loss_limit)


def aux_weight_tensor(module, device):
    """The aux-loss weight as a device fp32 scalar that the loss multiplies by.

    A Python float would be baked into a captured hipGraph (forward AND the
    saved backward), so a replay at epoch 10 would still weigh recon / mimic
    by the capture-time epoch's weight. The step reads this scalar instead;
    it is rewritten eagerly before every replay (``sync_aux_weight``) the way
    the optimizer's hyper table is. Outside a capture it is refreshed here."""
    w = module.__dict__.get("_aux_w_dev")
    if w is None or w.device != torch.device(device):
        if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("aux-loss weight scalar must be created by an eager step before capture")
        w = torch.empty((), dtype=torch.float32, device=device)
        module.__dict__["_aux_w_dev"] = w
    if not (device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
        w.fill_(aux_weight_value(module))
    return w


def sync_aux_weight(module):
    """Write the current epoch's aux weight into the captured step's scalar."""
    w = module.__dict__.get("_aux_w_dev")
    if w is not None:
        w.fill_(aux_weight_value(module))


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
