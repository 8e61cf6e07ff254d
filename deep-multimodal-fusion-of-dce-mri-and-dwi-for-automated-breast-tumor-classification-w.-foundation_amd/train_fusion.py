"""Fusion training step -- MI355X build of the reference's
``code/train_fusion.py`` (LightningFusionModel, :13-702; helpers :709-760).

``LightningFusionModel`` keeps the reference's constructor, hooks and
``_shared_step(batch, phase, return_preds)`` contract, without the Lightning
runtime: a driver (``bench.py``, ``dmf_dp.FusionDPTrainer``) calls
``training_step`` -> backward -> optimizer step, on one process per GPU.
The loss terms run in the fused criterion kernels (csrc/losses.hip); the five
reconstruction terms of one step share a single launch.
"""
from __future__ import annotations


import torch
import torch.nn as nn

import dmf_ops as O
from loss import LabelSmoothing
from selector_helpers import LightningFusionOptimizerFactory, mask_criterion_selector
from train import (aux_weight_tensor, aux_weight_value, compute_attn_energy_loss, compute_feat_norm_loss,
                   compute_feature_consistency_loss, sync_aux_weight, tta_flip_lr, tta_flip_lrud, tta_flip_ud, tta_id)


class LightningFusionModel(nn.Module):
    def __init__(self, dwi_model, dce_model, fusion_model, parameters_dict, criterion_clf, optimizer_fn=None,
                 scheduler_fn=None, paths=None):
        super().__init__()
        self.method = "fusion"
        self.dwi_model = dwi_model
        self.dce_model = dce_model
        self.fusion_model = fusion_model
        self.parameters_dict = parameters_dict
        self.criterion_clf = criterion_clf
        self.paths = paths
        fp = parameters_dict["fusion_model_parameters"]
        self.recon_enabled = fp["recon_enabled"]
        self.lambda_recon = fp["lambda_recon"]
        self.mask_enabled = fp["mask_parameters"]["mask"]
        self.lambda_mask = fp["mask_parameters"]["lambda_mask"]
        self.class_num = parameters_dict["class_num"]
        self.mimic_enabled = fp["mimic_enabled"]
        self.lambda_mimic = fp["lambda_mimic"]
        self.label_smoother = LabelSmoothing(self.class_num, fp["label_smoothing_alpha"]) \
            if fp["label_smoothing_enabled"] else None
        self.mask_criterion = mask_criterion_selector(parameters_dict, self.method)
        self.enable_modality_attention = fp["enable_modality_attention"]
        self.use_aux_loss_sched = parameters_dict["use_simple_aux_loss_scheduling"]
        self.aux_loss_limit = parameters_dict["aux_loss_weight_epoch_limit"]
        self.attn_reg_enabled = fp["attn_reg_enabled"]
        self.lambda_attn_energy = fp["lambda_attn_energy"]
        self.lambda_feature_consistency = fp["lambda_feature_consistency"]
        self.feat_norm_reg_enabled = fp["feat_norm_reg_enabled"]
        self.lambda_feat_norm = fp["lambda_feat_norm"]
        self.unfreeze_timer = int(parameters_dict["unfreeze_timer"])
        self.backbone_freeze_on_start = parameters_dict["backbone_freeze_on_start"]
        self.backbone_num_groups = parameters_dict["backbone_num_groups"]
        self.current_epoch = 0
        self.global_step = 0
        self.transforms_list = [tta_id, tta_flip_lr, tta_flip_ud, tta_flip_lrud]
        self.opt_factory = LightningFusionOptimizerFactory(dwi_model=dwi_model, dce_model=dce_model,
                                                           fusion_model=fusion_model, parameters=parameters_dict)
        self.optimizer_fn = self.opt_factory.optimizer_fn
        self.scheduler_fn = self.opt_factory.scheduler_fn
        self.optimizer = None
        self.last_metrics = {}

    @property
    def device(self):
        return next(self.fusion_model.parameters()).device

    # ---------------------------------------------------------------- hooks
    def configure_optimizers(self):
        self.optimizer = self.optimizer_fn(None)
        if self.scheduler_fn is None:
            return self.optimizer
        sched = self.scheduler_fn(self.optimizer)
        return {"optimizer": self.optimizer, "lr_scheduler": sched}

    def on_train_epoch_start(self):
        """train_fusion.py:155-169: gradual unfreeze."""
        if self.backbone_freeze_on_start and self.current_epoch <= (self.unfreeze_timer * self.backbone_num_groups
                                                                    + 1):
            new = self.opt_factory.gradual_unfreeze(epoch=self.current_epoch,
                                                    unfreeze_every_n_epochs=self.unfreeze_timer)
            if new and self.optimizer is not None:
                self.opt_factory.sync_unfrozen_params_to_optimizer(self.optimizer, new)

    def forward(self, dwi_feats, dce_feats, dwi_mask=None, dce_mask=None):
        return self.fusion_model(dwi_feats, dce_feats, dwi_mask, dce_mask)

    # ---------------------------------------------- captured-step hooks
    def step_signature(self):
        """What the captured step's graph STRUCTURE depends on beyond the
        optimizer layout: the aux-loss gate (train_fusion.py:274, aux_w > 0
        drops the recon and mimic nodes after epoch ``aux_loss_limit``)."""
        return (aux_weight_value(self) > 0.0,)

    def sync_step_scalars(self):
        """Write the epoch-dependent scalars the captured step reads (the
        aux-loss weight) before a replay."""
        sync_aux_weight(self)

    # ------------------------------------------------------------- encoders
    def _encode(self, dwi_inputs, dce_inputs):
        """The two encoder forwards (train_fusion.py:227-230). They are
        independent until FusionModel, so on the GPU the DCE encoder runs on a
        second HIP stream beside the DWI one (a fork/join that a captured
        hipGraph keeps as two branches): the small, latency-bound launches
        and the tails of one encoder overlap the other's. The dropout Philox
        snapshots are taken up front in the sequential order (DWI, DCE), so
        the masks match a sequential run; autograd replays each encoder's
        backward on the stream its forward ran on."""
        # read by dmf_dp.FusionTrainer: the backward's half-chip dgrad tiles only pay when the
        # two encoders' backwards really run on two streams, i.e. when this forward forked
        self.__dict__["_encoders_forked"] = False
        if not (dwi_inputs.is_cuda and O.PARALLEL_BRANCHES):
            return self.dwi_model(dwi_inputs), self.dce_model(dce_inputs)
        main = torch.cuda.current_stream(dwi_inputs.device)
        side = self.__dict__.get("_side_stream")
        if side is None or side.device != dwi_inputs.device:
            side = torch.cuda.Stream(dwi_inputs.device)
            self.__dict__["_side_stream"] = side
        # one snapshot per encoder whenever it draws dropout masks (train mode,
        # or MC dropout with only the Dropout modules on): the two streams then
        # never advance the shared Philox state concurrently
        snap_dwi = O.RNG.snapshot(dwi_inputs.device) if _draws_dropout(self.dwi_model) else None
        snap_dce = O.RNG.snapshot(dwi_inputs.device) if _draws_dropout(self.dce_model) else None
        side.wait_stream(main)
        prev = O.RNG_CURRENT[0]
        O.ORIGIN_STREAM[0] = main
        try:
            O.concurrent_tiles(True)
            O.RNG_CURRENT[0] = snap_dwi
            out_dwi = self.dwi_model(dwi_inputs)
            O.RNG_CURRENT[0] = snap_dce
            with torch.cuda.stream(side):
                O.record_tree([dce_inputs, snap_dce], side)
                out_dce = self.dce_model(dce_inputs)
        finally:
            O.RNG_CURRENT[0] = prev
            O.ORIGIN_STREAM[0] = None
            O.concurrent_tiles(False)  # idempotent: restores the single-stream tile sizing
        main.wait_stream(side)
        self.__dict__["_encoders_forked"] = True
        O.record_tree(out_dce, main)
        return out_dwi, out_dce

    # ---------------------------------------------------------------- step
    def _shared_step(self, batch, phase="train", return_preds=False):
        """train_fusion.py:204-321."""
        is_train = phase == "train"
        if self.mask_enabled:
            dwi_inputs, dce_inputs, masks_batch, labels = batch
        else:
            dwi_inputs, dce_inputs, labels = batch
            masks_batch = None
        dev = self.device
        dwi_inputs = dwi_inputs.to(dev, non_blocking=True)
        dce_inputs = dce_inputs.to(dev, non_blocking=True)
        labels = labels.long().to(dev, non_blocking=True)
        if masks_batch is not None:
            masks_batch = masks_batch.to(dev, non_blocking=True)
        aux_w = aux_weight_value(self)

        (_, dwi_aux, dwi_mask_pred), (_, dce_aux, dce_mask_pred) = self._encode(dwi_inputs, dce_inputs)
        logits, fused_mask_logits, aux = self.forward(dwi_aux["raw_feats"], dce_aux["raw_feats"], dwi_mask_pred,
                                                      dce_mask_pred)

        if self.label_smoother is not None:
            smoothed = self.label_smoother(logits, labels)
        if is_train:
            cls_loss = self.criterion_clf(logits, smoothed)  # Q7: undefined without smoothing, as in the reference
        else:
            cls_loss = self.criterion_clf(logits, labels)
        # the device assembly covers the default terms; the fusion aux has no raw_feats, so the
        # feat-norm term is the constant 0 of compute_feat_norm_loss and drops out
        feat_norm_zero = not self.feat_norm_reg_enabled or aux.get("raw_feats", None) is None
        if DEVICE_LOSS and dev.type == "cuda" and not self.attn_reg_enabled and feat_norm_zero and cls_loss.dim() == 0:
            return self._assemble_on_device(cls_loss, logits, labels, fused_mask_logits, aux, dwi_aux, dce_aux,
                                            dwi_mask_pred, dce_mask_pred, masks_batch, dwi_inputs, dce_inputs,
                                            aux_w, is_train, return_preds)
        total = cls_loss

        mask_loss_val = torch.zeros((), device=dev)
        if self.mask_enabled:
            mask_loss_val = (safe_mask_loss(dwi_mask_pred, masks_batch, self.mask_criterion)
                             + safe_mask_loss(dce_mask_pred, masks_batch, self.mask_criterion)
                             + safe_mask_loss(fused_mask_logits, masks_batch, self.mask_criterion)) / 3
            if is_train:
                total = total + self.lambda_mask * mask_loss_val

        if self.attn_reg_enabled and is_train:
            total = total + compute_attn_energy_loss(aux, dev) * self.lambda_attn_energy \
                + compute_feature_consistency_loss(aux, dev) * self.lambda_feature_consistency
        if self.feat_norm_reg_enabled and is_train:
            total = total + compute_feat_norm_loss(aux, dev) * self.lambda_feat_norm

        recon_loss_val = torch.zeros((), device=dev)
        mimic_loss_val = torch.zeros((), device=dev)
        if aux_w > 0.0 and self.recon_enabled and is_train:
            # the epoch-dependent weight as a device scalar: a captured step replays with the current
            # epoch's value (FusionTrainer.step writes it before every replay); the aux_w > 0 gate itself
            # is part of the trainer's capture signature
            w = aux_weight_tensor(self, dev) if dev.type == "cuda" else aux_w
            recon_loss_val = fused_recon_losses(dwi_aux["recon_feats"], dce_aux["recon_feats"], aux["recon_fused"],
                                                dwi_inputs.detach(), dce_inputs.detach())
            total = total + self.lambda_recon * recon_loss_val * w
            pf = aux.get("proj_fused", None)
            if self.mimic_enabled and pf is not None and len(pf) >= 4:
                mimic_loss_val = O.mimic_pairs(pf, npairs=2)
                total = total + self.lambda_mimic * mimic_loss_val * w

        preds = torch.argmax(logits, dim=1)
        acc = (preds == labels).float().mean()
        self.last_metrics = {"loss": total.detach(), "acc": acc.detach(), "cls": cls_loss.detach(),
                             "mask": mask_loss_val.detach(), "recon": recon_loss_val.detach(),
                             "mimic": mimic_loss_val.detach()}
        if return_preds:
            return total.detach(), logits.detach(), aux, fused_mask_logits
        return total

    def _assemble_on_device(self, cls_loss, logits, labels, fused_mask_logits, aux, dwi_aux, dce_aux, dwi_mask_pred,
                            dce_mask_pred, masks_batch, dwi_inputs, dce_inputs, aux_w, is_train, return_preds):
        """The rest of _shared_step (train_fusion.py:246-303) with the loss
        arithmetic in one launch (O.loss_combine) instead of ~40 scalar aten
        launches forward + backward: total = cls + lambda_mask * (m_dwi + m_dce
        + m_fused) / 3 + aux_w * (lambda_recon * recon + lambda_mimic * mimic),
        recon = ((t0 + t1) / 2 + (t2 + t3) / 2 + t4) / 3 over the five
        reconstruction terms; the logged mask / recon / mimic values are the
        launch's group sums."""
        dev = logits.device
        parts = [(cls_loss, (1.0,), False, -1, (0.0,))]
        if self.mask_enabled:
            lm = self.lambda_mask / 3.0 if is_train else 0.0
            for pred in (dwi_mask_pred, dce_mask_pred, fused_mask_logits):
                parts.append((safe_mask_loss(pred, masks_batch, self.mask_criterion), (lm,), False, 0, (1.0 / 3,)))
        w = None
        with_aux = aux_w > 0.0 and self.recon_enabled and is_train
        if with_aux:
            w = aux_weight_tensor(self, dev)
            t, rc = fused_recon_terms(dwi_aux["recon_feats"], dce_aux["recon_feats"], aux["recon_fused"],
                                      dwi_inputs.detach(), dce_inputs.detach())
            parts.append((t, tuple(self.lambda_recon * c for c in rc), True, 1, rc))
            pf = aux.get("proj_fused", None)
            if self.mimic_enabled and pf is not None and len(pf) >= 4:
                parts.append((O.mimic_pairs(pf, npairs=2), (self.lambda_mimic,), True, 2, (1.0,)))
        total, groups = O.loss_combine(parts, 3, w)
        # (a group with no term sums to 0, as the reference's torch.zeros placeholders)
        self.last_metrics = {"loss": total.detach(), "acc": O.batch_accuracy(logits, labels),
                             "cls": cls_loss.detach(), "mask": groups[0], "recon": groups[1], "mimic": groups[2]}
        if return_preds:
            return total.detach(), logits.detach(), aux, fused_mask_logits
        return total

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True, **kwargs):
        """Lightning-layout .ckpt -> module (run_training.py:123-131); see run_training.py."""
        from run_training import load_from_checkpoint
        return load_from_checkpoint(cls, checkpoint_path, map_location=map_location, strict=strict, **kwargs)

    def training_step(self, batch, batch_idx=0):
        # every trainable conv weight's re-layouts for this step in one launch (dmf_ops.PrepPlan)
        O.PREP.prep_step(self)
        return self._shared_step(batch, "train")

    def validation_step(self, batch, batch_idx=0):
        loss, _, _, _ = self._shared_step(batch, phase="val", return_preds=True)
        return loss

    # ------------------------------------------------------------- predict
    def forward_from_inputs(self, dwi_inputs, dce_inputs, masks=None):
        _, dwi_aux, dwi_mask = self.dwi_model(dwi_inputs)
        _, dce_aux, dce_mask = self.dce_model(dce_inputs)
        return self.forward(dwi_aux["raw_feats"], dce_aux["raw_feats"], dwi_mask, dce_mask)

    # ---- test-time MC dropout x TTA (train_fusion.py:445-632) -------------
    def enable_dropout(self, model):
        """train_fusion.py:445-449."""
        for m in model.modules():
            if isinstance(m, nn.Dropout):
                m.train()

    def set_batchnorm_eval(self, model):
        """train_fusion.py:455-459."""
        for m in model.modules():
            if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.SyncBatchNorm)):
                m.eval()

    def _get_module_train_states(self, model):
        return {m: m.training for m in model.modules()}

    def _restore_module_train_states(self, model, states):
        for m, was_training in states.items():
            m.train(was_training)

    def mc_enable(self, model):
        """train_fusion.py:479-481: Dropout on, BatchNorm in eval."""
        self.enable_dropout(model)
        self.set_batchnorm_eval(model)

    @torch.no_grad()
    def _replicated_forward(self, dwi_list, dce_list, chunk):
        """One batched forward over replicas of the batch (TTA views x MC
        passes, concatenated along the batch axis): BN is per-sample in eval
        mode and every replica row draws its own Philox dropout mask (the mask
        index runs over the batch rows), so R replicas of B volumes cost
        ceil(R*B/chunk) encoder+fusion launches instead of R sequential
        forwards. Returns (softmax probs [R, B, K], gating [R, B, 2])."""
        b = dwi_list[0].shape[0]
        r = len(dwi_list)
        per = max(1, chunk // b)
        probs, gates = [], []
        for i in range(0, r, per):
            x_dwi = torch.cat(dwi_list[i:i + per], 0)
            x_dce = torch.cat(dce_list[i:i + per], 0)
            (_, dwi_aux, dwi_mask), (_, dce_aux, dce_mask) = self._encode(x_dwi, x_dce)
            logits, _, aux = self.forward(dwi_aux["raw_feats"], dce_aux["raw_feats"], dwi_mask, dce_mask)
            probs.append(torch.softmax(logits.float(), dim=1).view(-1, b, logits.shape[1]))
            gw = aux["gating_weights"]
            gates.append(gw.float().reshape(-1, b, gw.shape[-1]) if gw is not None else None)
        gating = torch.cat(gates, 0) if all(g is not None for g in gates) else None
        return torch.cat(probs, 0), gating, dwi_aux, dce_aux

    def predict_mc_dropout(self, dwi_inputs, dce_inputs, masks=None, passes=20, chunk=256):
        """train_fusion.py:484-537: passes stochastic forwards (encoders'
        Dropout on, BN eval) -> mean / std of the softmax, mean gating; the
        passes run batched (_replicated_forward). The reference's
        masks-given branch feeds encoder *logits* back into the encoders
        (:500-503) and cannot run; it is not reproduced."""
        st_dwi = self._get_module_train_states(self.dwi_model)
        st_dce = self._get_module_train_states(self.dce_model)
        self.mc_enable(self.dwi_model)
        self.mc_enable(self.dce_model)
        try:
            probs, gating, dwi_aux, dce_aux = self._replicated_forward([dwi_inputs] * passes, [dce_inputs] * passes,
                                                                       chunk)
        finally:
            self._restore_module_train_states(self.dwi_model, st_dwi)
            self._restore_module_train_states(self.dce_model, st_dce)
        mean_gating = gating.mean(0).cpu() if gating is not None else None
        return probs.mean(0), probs.std(0), {"gating_weights": mean_gating, "dwi_aux": dwi_aux, "dce_aux": dce_aux}

    def predict_tta(self, dwi_inputs, dce_inputs, masks=None, transforms=None, chunk=256):
        """train_fusion.py:541-587: one forward per flip (identity, lr, ud,
        lr+ud; train.py:916-923) -> mean / std of the softmax, mean gating;
        the views run batched. As in the reference the aux of the fusion
        output has no dwi_aux / dce_aux keys, so those stay None."""
        transforms = transforms if transforms is not None else self.transforms_list
        probs, gating, _, _ = self._replicated_forward([t(x=dwi_inputs) for t in transforms],
                                                       [t(x=dce_inputs) for t in transforms], chunk)
        mean_gating = gating.mean(0).cpu() if gating is not None else None
        return probs.mean(0), probs.std(0), {"gating_weights": mean_gating, "dwi_aux": None, "dce_aux": None}

    def predict_tta_mc(self, dwi_inputs, dce_inputs, masks=None, transforms=None, passes=10, chunk=256):
        """train_fusion.py:591-632: per flip, the MC mean of passes
        stochastic forwards; then mean / std over the flips. All
        len(transforms) x passes forwards run batched."""
        transforms = transforms if transforms is not None else self.transforms_list
        st_dwi = self._get_module_train_states(self.dwi_model)
        st_dce = self._get_module_train_states(self.dce_model)
        self.mc_enable(self.dwi_model)
        self.mc_enable(self.dce_model)
        try:
            views_dwi = [t(x=dwi_inputs) for t in transforms for _ in range(passes)]
            views_dce = [t(x=dce_inputs) for t in transforms for _ in range(passes)]
            probs, gating, dwi_aux, dce_aux = self._replicated_forward(views_dwi, views_dce, chunk)
        finally:
            self._restore_module_train_states(self.dwi_model, st_dwi)
            self._restore_module_train_states(self.dce_model, st_dce)
        nt = len(transforms)
        per_t = probs.view(nt, passes, *probs.shape[1:]).mean(1)
        mean_gating = None
        if gating is not None:
            mean_gating = gating.view(nt, passes, *gating.shape[1:]).mean(1).mean(0).cpu()
        return per_t.mean(0), per_t.std(0), {"gating_weights": mean_gating, "dwi_aux": dwi_aux, "dce_aux": dce_aux}

    @torch.no_grad()
    def predict_custom(self, batch, mode="normal", mc_passes=10):
        """train_fusion.py:682-701."""
        dwi = batch[0].to(self.device)
        dce = batch[1].to(self.device)
        masks = batch[2] if len(batch) == 4 else None
        if mode == "normal":
            return self.forward_from_inputs(dwi, dce, masks)
        if mode == "tta":
            return self.predict_tta(dwi, dce, masks)
        if mode == "mc":
            return self.predict_mc_dropout(dwi, dce, passes=mc_passes)
        if mode == "tta_mc":
            return self.predict_tta_mc(dwi, dce, masks, passes=mc_passes)
        raise ValueError(f"Unknown predict mode: {mode}")


# ------------------------------------------------------------------ helpers



def _draws_dropout(model):
    return model.training or any(isinstance(m, nn.Dropout) and m.training and m.p > 0 for m in model.modules())


def compute_recon_list_loss(recon_list, input_img):
    """train_fusion.py:709-744 (2-D): mean over the valid maps of
    recon_image_loss(bilinear(r -> input size), channel-mean(input))."""
    if recon_list is None:
        return torch.zeros((), device=input_img.device)
    if isinstance(recon_list, torch.Tensor):
        recon_list = [recon_list]
    maps = [r for r in recon_list if r is not None]
    if not maps:
        return torch.zeros((), device=input_img.device)
    for r in maps:
        if r.shape[1] != 1:
            raise NotImplementedError("multi-channel reconstructions are not on the reference path")
    tgt = O.channel_mean_map(input_img)
    terms = O.recon_terms(maps, [0] * len(maps), tgt)
    return terms.sum() / len(maps)


DEVICE_LOSS = True  # knob "device_loss": the one-launch loss assembly (dmf_loss_combine)


def fused_recon_terms(dwi_recons, dce_recons, fused_recon, dwi_img, dce_img):
    """The five reconstruction terms of fused_recon_losses as a [5] tensor with
    the weights that make recon = sum(w * t), ((t0 + t1) / 2 + (t2 + t3) / 2 +
    t4) / 3 (train_fusion.py:281-285); other layouts: ([recon], (1,))."""
    dw = [r for r in dwi_recons if r is not None]
    dc = [r for r in dce_recons if r is not None]
    if fused_recon is None or len(dw) != 2 or len(dc) != 2:
        return fused_recon_losses(dwi_recons, dce_recons, fused_recon, dwi_img, dce_img).reshape(1), (1.0,)
    ta = O.channel_mean_map(dwi_img)
    tb = O.channel_mean_map(dce_img)
    ca, cb = dwi_img.shape[1], dce_img.shape[1]
    t = O.recon_terms([dw[0], dw[1], dc[0], dc[1], fused_recon], [0, 0, 1, 1, 2], ta, tb, ca / (ca + cb),
                      cb / (ca + cb))
    return t, (1.0 / 6, 1.0 / 6, 1.0 / 6, 1.0 / 6, 1.0 / 3)


def fused_recon_losses(dwi_recons, dce_recons, fused_recon, dwi_img, dce_img):
    """The three compute_recon_list_loss calls of train_fusion.py:281-285
    (dwi [r1,r2], dce [r1,r2], fused vs cat(dwi, dce)) / 3, in ONE launch."""
    dw = [r for r in dwi_recons if r is not None]
    dc = [r for r in dce_recons if r is not None]
    if fused_recon is None or len(dw) != 2 or len(dc) != 2:
        return (compute_recon_list_loss(dwi_recons, dwi_img) + compute_recon_list_loss(dce_recons, dce_img)
                + compute_recon_list_loss(fused_recon, torch.cat([dwi_img, dce_img], 1))) / 3
    ta = O.channel_mean_map(dwi_img)
    tb = O.channel_mean_map(dce_img)
    ca, cb = dwi_img.shape[1], dce_img.shape[1]
    t = O.recon_terms([dw[0], dw[1], dc[0], dc[1], fused_recon], [0, 0, 1, 1, 2], ta, tb, ca / (ca + cb),
                      cb / (ca + cb))
    return ((t[0] + t[1]) / 2 + (t[2] + t[3]) / 2 + t[4]) / 3


def safe_mask_loss(pred_logits, gt_mask, mask_criterion):
    """train_fusion.py:747-760 (quirk Q6: the resized mask is computed but the
    original one is passed to the criterion)."""
    if pred_logits is None:
        raise ValueError("pred_logits is None in safe_mask_loss")
    if gt_mask is None:
        raise ValueError("gt_mask is None in safe_mask_loss")
    return mask_criterion(pred_logits, gt_mask)
