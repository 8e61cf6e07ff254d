"""Criterion / optimizer / freeze-policy selection -- MI355X build of the
reference's ``code/selector_helpers.py`` (:14-46, :95-114, :356-742).

``LightningFusionOptimizerFactory`` keeps the reference's grouping by
parameter-name substrings, the freeze-on-start policy, the EFFECTIVE
``_build_optimizer`` (the second definition, :632-685, overrides the first),
``gradual_unfreeze`` (:541-584) and ``sync_unfrozen_params_to_optimizer``
(:588-613); the optimizer it returns is the device multi-tensor AdamW.
"""
from __future__ import annotations

import torch

from dmf_optim import FusedAdamW
from loss import DiceBCELoss, SoftDiceLoss, SoftFocalLoss, SoftWeightedFocalLoss


def get_classification_loss(parameters, train_labels, model_type, device):
    """selector_helpers.py:14-46. 'wfl' -> inverse-frequency class weights
    N / (K * (count + 1e-6)) from the TRAIN labels; 'fl' keeps the reference's
    argument mix-up (alpha passed as gamma, gamma as reduction; quirk Q8)."""
    clp = parameters[f"{model_type}_model_parameters"]["classification_loss_parameters"]
    code = clp["classification_loss_code"]
    if code == "fl":
        alpha = clp["alpha"] if clp["alpha"] is not None else 0.25
        gamma = clp["gamma"] if clp["gamma"] is not None else 2
        return SoftFocalLoss(alpha, gamma)
    if code == "wfl":
        gamma = clp["gamma"] if clp["gamma"] is not None else 2
        counts = torch.bincount(train_labels.long().cpu())
        weights = train_labels.numel() / (len(counts) * (counts.float() + 1e-6))
        return SoftWeightedFocalLoss(gamma, weights.to(device))
    raise ValueError(f"Invalid classification_loss_code '{code}'. Valid options: ['cel', 'fl', 'wfl']")


def mask_criterion_selector(parameters, model_type):
    """selector_helpers.py:95-114."""
    mk = parameters[f"{model_type}_model_parameters"]["mask_parameters"]
    if not mk["mask"]:
        return None
    if mk["mask_loss_type"] == "dice":
        return SoftDiceLoss()
    if mk["mask_loss_type"] == "dice_bce":
        return DiceBCELoss(bce_weight=1.0, dice_weight=1.0)
    raise ValueError(f"Invalid mask loss: {mk['mask_loss_type']}")


class LightningFusionOptimizerFactory:
    """selector_helpers.py:356-742."""

    def __init__(self, dwi_model, dce_model, fusion_model, parameters):
        self.dwi_model = dwi_model
        self.dce_model = dce_model
        self.fusion_model = fusion_model
        self.parameters = parameters
        self.num_backbone_groups = parameters.get("backbone_num_groups", 3)
        self.backbone_freeze_on_start = parameters.get("backbone_freeze_on_start", True)
        self.layers_unfrozen = 0
        self.dwi_named_groups = self.group_model_with_backbone_params(
            dwi_model, parameters["dwi_model_parameters"]["use_backbone"], self.num_backbone_groups)
        self.dce_named_groups = self.group_model_with_backbone_params(
            dce_model, parameters["dce_model_parameters"]["use_backbone"], self.num_backbone_groups)
        self.fusion_named = list(fusion_model.named_parameters())
        if self.backbone_freeze_on_start:
            self._freeze_all_backbone_groups()
        self.newly_unfrozen_groups = []
        self.optimizer_fn = self._build_optimizer()
        self.scheduler_fn = self._build_scheduler()

    @staticmethod
    def group_model_with_backbone_params(model, use_backbone=True, expected_num_groups=3):
        """[backbone, block1+block2, block3 + other] by name substring
        (classification heads skipped), selector_helpers.py:396-430."""
        bb, b1, b2, b3, other = [], [], [], [], []
        for name, p in model.named_parameters():
            if "classification_head" in name:
                continue
            if use_backbone and ("backbone" in name or "backbone_neck" in name):
                bb.append((name, p))
            elif "block1" in name:
                b1.append((name, p))
            elif "block2" in name:
                b2.append((name, p))
            elif "block3" in name:
                b3.append((name, p))
            else:
                other.append((name, p))
        if use_backbone:
            b2 = b1 + b2
            b1 = bb
        return [b1, b2, b3 + other]

    def _freeze_all_backbone_groups(self):
        for p in self.dwi_model.parameters():
            p.requires_grad = False
        for p in self.dce_model.parameters():
            p.requires_grad = False

    def _get_base_optimizer(self, params, cfg):
        op = cfg["optimizer_parameters"]
        name = op["name"].lower()
        if name not in ("adamw", "adam"):
            raise ValueError(f"Unsupported optimizer: {name}")
        if name == "adam":
            raise NotImplementedError("plain Adam (coupled L2) is not on the reference default path")
        return FusedAdamW(params, lr=op["lr"], eps=op["eps"], betas=op["betas"], amsgrad=op.get("amsgrad", False),
                          weight_decay=op["weight_decay"])

    def _build_optimizer(self):
        """The effective builder (selector_helpers.py:632-685): frozen start ->
        one group (fusion params, lr = base_lr, wd = reg_base); otherwise
        [g0, g1, g2, fusion] with lr = base/decay^(n-1-i), wd = reg*f^(n-1-i)."""
        cfg = self.parameters["fusion_model_parameters"]
        op = cfg["optimizer_parameters"]
        if not op.get("discriminative_lr", False):
            return lambda params: self._get_base_optimizer(params, cfg)
        lr_decay = op.get("lr_decay_factor", 2.0)
        wd_plain = op.get("weight_decay", 0.0)
        base_lr = op.get("lr", 1e-3)
        disc_reg = op.get("discriminative_reg", False)
        reg_base = op.get("reg_base", wd_plain)
        reg_decay = op.get("reg_decay_factor", 2.0)
        merged = []
        if not self.backbone_freeze_on_start:
            for i in range(max(len(self.dce_named_groups), len(self.dwi_named_groups))):
                g = []
                if i < len(self.dce_named_groups):
                    g += self.dce_named_groups[i]
                if i < len(self.dwi_named_groups):
                    g += self.dwi_named_groups[i]
                if g:
                    merged.append(g)
        merged.append(self.fusion_named)
        groups = []
        n = len(merged)
        for i, named in enumerate(merged):
            params = [p for _, p in named]
            if not params:
                continue
            lr = base_lr / (lr_decay ** (n - 1 - i))
            wd = reg_base * (reg_decay ** (n - 1 - i)) if disc_reg else wd_plain
            groups.append({"params": params, "lr": lr, "weight_decay": wd})
        if not groups:
            allp = ([p for _, p in self.dwi_model.named_parameters()] + [p for _, p in self.dce_model.named_parameters()]
                    + [p for _, p in self.fusion_named])
            groups = [{"params": allp, "lr": base_lr, "weight_decay": wd_plain}]
        self.param_groups_spec = groups
        return lambda _: self._get_base_optimizer(groups, cfg)

    def _unfreeze_named_group(self, named_group, model):
        mp = dict(model.named_parameters())
        newly = []
        for name, _ in named_group:
            if name in mp and not mp[name].requires_grad:
                mp[name].requires_grad = True
                newly.append(mp[name])
        return len(newly), newly

    def gradual_unfreeze(self, epoch, unfreeze_every_n_epochs=20):
        """selector_helpers.py:541-584: one group per multiple of the timer, deep -> shallow."""
        if epoch == 0 or unfreeze_every_n_epochs <= 0 or epoch % unfreeze_every_n_epochs != 0:
            return []
        if self.layers_unfrozen >= self.num_backbone_groups:
            return []
        gi = self.num_backbone_groups - 1 - self.layers_unfrozen
        if gi < 0 or gi >= self.num_backbone_groups:
            return []
        c1, n1 = self._unfreeze_named_group(self.dwi_named_groups[gi], self.dwi_model)
        c2, n2 = self._unfreeze_named_group(self.dce_named_groups[gi], self.dce_model)
        if c1 > 0 or c2 > 0:
            self.layers_unfrozen += 1
        return n1 + n2

    def sync_unfrozen_params_to_optimizer(self, optimizer, newly_unfrozen_params):
        """selector_helpers.py:588-613."""
        if not newly_unfrozen_params:
            return
        existing = {id(p) for g in optimizer.param_groups for p in g["params"]}
        add = [p for p in newly_unfrozen_params if isinstance(p, torch.nn.Parameter) and id(p) not in existing]
        if not add:
            return
        lr = self.parameters.get("backbone_unfreeze_lr", 1e-4) * (
            self.parameters.get("backbone_unfreeze_lr_factor", 1.0) ** (self.layers_unfrozen - 1))
        op = self.parameters["dwi_model_parameters"]["optimizer_parameters"]
        wd = op.get("reg_base", 0.0) * (op.get("reg_decay_factor", 1.0) ** (self.layers_unfrozen - 1))
        optimizer.add_param_group({"params": add, "lr": lr, "weight_decay": wd})

    def _build_scheduler(self):
        sch = self.parameters["fusion_model_parameters"].get("scheduler", None)
        if sch is None:
            return None
        name = sch["name"].lower()
        if name == "reduce_lr_on_plateau":
            def make(optimizer):
                s = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=sch["factor"],
                                                               patience=sch["patience"], min_lr=sch["min_lr"],
                                                               threshold=sch["threshold"])
                return {"scheduler": s, "monitor": sch["monitor"], "interval": "epoch"}
            return make
        if name == "cosine":
            def make(optimizer):
                return {"scheduler": torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=sch["T_max"],
                                                                                 eta_min=sch["eta_min"]),
                        "interval": "epoch"}
            return make
        raise ValueError(f"Unknown scheduler: {sch['name']}")
