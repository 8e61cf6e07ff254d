"""Default configuration dict, same schema as the reference's
``code/parameters_generate.py`` (which builds and torch.save()s it).

Only the keys read on the hot path are restated (model structure, criteria,
optimizer, freeze policy, aux-loss schedule, channel counts); values follow
parameters_generate.py line by line (cited inline). As in the reference,
``dce_model_parameters`` and ``fusion_model_parameters`` are the SAME dict
object as ``dwi_model_parameters`` (quirk Q1, :174, :183).
"""
from __future__ import annotations

import torch


def default_parameters():
    P = {}
    P["dim"] = 2                                        # :9
    P["compile"] = False                                # :14 (no tracing compiler here)
    P["dataloader_num_workers"] = 11                    # :15
    P["debug_training"] = False
    P["num_epochs"] = 900                               # :30
    P["batch_size"] = 32                                # :32
    P["segnum"] = 5                                     # :34
    P["class_num"] = 4                                  # :35
    P["methods"] = ["dwi", "dce"]
    P["namelist"] = ["train", "val", "test"]
    P["control_metric"] = "val_loss"                    # :46
    P["early_stop_metric"] = "val_roc_auc"              # :48
    P["patience"] = 90                                  # :50
    P["forced_mask_size"] = 32
    mp = {
        "input_size": 256,                              # :68
        "use_hybrid_transformer": False,                # :71
        "transformer_heads": 4,                         # :72
        "transformer_patch_size": 2,                    # :73
        "transformer_depth": 6,                         # :74
        "transformer_embed_dim": 512,                   # :75
        "patch_embed_fp8": False,                       # build option (config 5): PatchEmbed.proj on e4m3 MFMA
        "dropout": 0.2,                                 # :77
        "channels": (128, 256, 512),                    # :82
        "repeat_blocks": (1, 1, 1),                     # :83
        "downsample": (True, False, False),             # :84
        "downsample_each_repeat": False,                # :85
        "mid_squeeze": 2,                               # :86
        "backbone_index_lists": [],                     # :88 (set by build_medical_backbone)
        "backbone_out_channels": (),
        "proj_dim": 64,                                 # :90
        "use_se": True,                                 # :91
        "grad_clip": 5.0,
        "gradient_clip_algorithm": "norm",
        "enable_modality_attention": True,              # :96
        "use_backbone": True,                           # :97
        "use_input_adapt": False,                       # :98
        "use_advanced_adapt": False,                    # :99
        "transformer_backbone": False,
        "backbone_str": "radimagenet",                  # :101
        "label_smoothing_enabled": True,                # :103
        "label_smoothing_alpha": 0.1,                   # :104
        "mimic_enabled": True,                          # :107
        "lambda_mimic": 0.2,                            # :108
        "recon_enabled": True,                          # :111
        "reconstruction_loss_code": "mse",
        "lambda_recon": 0.1,                            # :113
        "classification_loss_parameters": {             # :116-120
            "classification_loss_code": "wfl", "gamma": 1.5, "alpha": None},
        "mask_parameters": {                            # :122-131
            "mask": True, "mask_stage": "f2", "lambda_mask": 0.2, "mask_loss_type": "dice",
            "mask_target_size": (32, 32), "mask_fusion_attention": True, "dice_weight": 0.5, "bce_weight": 0.5},
        "optimizer_parameters": {                       # :133-147
            "name": "adamW", "lr": 1e-4, "betas": (0.9, 0.999), "eps": 1e-08, "amsgrad": False,
            "weight_decay": 4e-5, "num_lr_groups": 3, "discriminative_lr": True, "lr_decay_factor": 1.2,
            "discrim_on": "all", "discriminative_reg": True, "reg_decay_factor": 0.8, "reg_base": 1e-4},
        "scheduler": {                                  # :148-164
            "name": "reduce_lr_on_plateau", "factor": 0.5, "patience": int(5 + 90 / 3), "min_lr": 4e-7,
            "threshold": 0.0001, "monitor": "val_loss", "T_max": 900, "eta_min": 0, "warmup_steps": 500,
            "max_steps": 10000},
        "attn_reg_enabled": False,                      # :166
        "lambda_attn_energy": 1e-4,
        "lambda_feature_consistency": 1e-4,
        "feat_norm_reg_enabled": True,                  # :169
        "lambda_feat_norm": 4e-5,                       # :170
    }
    P["dwi_model_parameters"] = mp
    P["dce_model_parameters"] = mp                       # :174 (alias)
    P["fusion_model_parameters"] = mp                    # :183 (alias)
    mp["fusion_specific_parameters"] = {                 # :185-194
        "mha_heads": 4, "use_cross_attention": True, "use_mask_attention": True, "token_pool": (4, 4),
        "fusion_channels": 128, "dwi_out_channels": mp["channels"][-1], "dce_out_channels": mp["channels"][-1],
        "fusion_recon_ch": 1}
    P["early_stopping_parameters"] = {"metric": "val_roc_auc", "mode": "max", "patience": 90, "min_delta": 1e-4}
    # :211 is "16-mixed" (fp16 autocast + GradScaler; run.py:59-76 keeps it on an
    # MI355X). Both 16-bit modes are built: "16-mixed" = IEEE fp16 activations
    # and MFMA operands with the device GradScaler (dmf_optim.DeviceGradScaler,
    # FusionTrainer), "bf16-mixed" = bf16 (fp32 range, no scaler) -- the
    # default here, as run.py:59-71 picks on bf16-capable GPUs. compute_dtype_of()
    # maps the precision to the kernels' compute dtype.
    P["precision"] = "bf16-mixed"
    P["test_mode"] = "tta_mc"                           # :215
    P["mc_passes"] = 10                                 # :216
    P["backbone_freeze_on_start"] = True                # :221
    P["backbone_num_groups"] = 3                        # :222
    P["unfreeze_timer"] = 40                            # :223
    P["foundation_model_unfreeze_timer"] = 40
    P["backbone_unfreeze_lr"] = mp["optimizer_parameters"]["lr"] * 0.1     # :225
    P["backbone_unfreeze_wd"] = mp["optimizer_parameters"]["reg_base"] * 0.1
    P["foundation_model_unfreeze_lr"] = 1e-5
    P["backbone_unfreeze_lr_factor"] = 0.25             # :228
    P["use_simple_aux_loss_scheduling"] = True          # :232
    P["aux_loss_weight_epoch_limit"] = max(100, P["unfreeze_timer"] * (P["backbone_num_groups"] + 2))  # :233
    P["dwi_bvals_to_use"] = tuple(range(13))            # :241
    P["dce_channels_to_use"] = tuple(range(6))          # :242
    P["dwi_add_adc_map"] = True
    P["dwi_base_channel_num"] = 13
    P["dwi_channel_num"] = 14                           # :245-249
    P["dce_channel_num"] = 6                            # :251
    P["min_epochs"] = 300
    return P


def small_parameters(channels=(16, 32, 64), input_size=64, dwi_c=14, dce_c=6, dropout=0.0, use_backbone=True):
    """Reduced config used by the parity tests (SURVEY.md 8(c) fixture shapes)."""
    P = default_parameters()
    mp = P["dwi_model_parameters"]
    mp["channels"] = tuple(channels)
    mp["input_size"] = input_size
    mp["dropout"] = dropout
    mp["use_backbone"] = use_backbone
    mp["fusion_specific_parameters"]["dwi_out_channels"] = channels[-1]
    mp["fusion_specific_parameters"]["dce_out_channels"] = channels[-1]
    P["dwi_channel_num"] = dwi_c
    P["dce_channel_num"] = dce_c
    return P


PRECISION_DTYPES = {"16-mixed": torch.float16, "16": torch.float16, "bf16-mixed": torch.bfloat16,
                    "bf16": torch.bfloat16, "32": torch.float32, "32-true": torch.float32}


def compute_dtype_of(P, mp=None):
    """The kernels' compute dtype: an explicit ``compute_dtype`` in the model
    parameters, else the one Lightning's ``precision`` names (fp16 for
    "16-mixed", bf16 for "bf16-mixed", fp32 for "32")."""
    mp = mp if mp is not None else P["dwi_model_parameters"]
    dt = mp.get("compute_dtype")
    if dt is not None:
        return dt
    return PRECISION_DTYPES.get(str(P.get("precision", "bf16-mixed")), torch.bfloat16)
