#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz from the CPU oracle restatement.

The reference itself could not be imported here (refused by
the environment), so these vectors are produced by ``oracle/`` -- they pin
the oracle (and, through the GPU tests, the HIP path) against silent drift;
they do NOT pin the reference ("parity unpinned").

Weights are not stored: each fixture records the seed recipe the tests
re-run (product-side seeded construction, state_dict loaded into the oracle).

    python tools/make_golden.py [small] [full] [ckpt]
"""
import copy
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import foundation_model as FM  # noqa: E402
import model_module as MM  # noqa: E402
import parameters as PR  # noqa: E402
from oracle import losses as OL  # noqa: E402
from oracle import model as OM  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def seeded_encoder(P, method, cin, seed):
    """Product-side seeded construction (same recipe the tests use)."""
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", method, cin)  # sets P's backbone_index_lists (reference side effect)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone(method, P, bb), True)
    ref = OM.ModelMaskHeadBackbone(method, P, OM.ResNet50OS8(cin))
    ref.load_state_dict(enc.state_dict())
    return enc, ref


def seeded_fusion(P, seed):
    torch.manual_seed(seed)
    fm = MM.FusionModel(P)
    fr = OM.FusionModel(P)
    fr.load_state_dict(fm.state_dict())
    return fm, fr


def volume_batch(B, S, seed, cd=14, cc=6):
    g = torch.Generator().manual_seed(seed)
    dwi = (0.5 + torch.randn(B, cd, S, S, generator=g) / 6).clamp(0, 1)
    dce = torch.rand(B, cc, S, S, generator=g)
    yy, xx = torch.meshgrid(torch.arange(32), torch.arange(32), indexing="ij")
    masks = torch.zeros(B, 1, 32, 32)
    for b in range(B):
        cy, cx = torch.randint(8, 24, (2,), generator=g).tolist()
        r = torch.randint(4, 11, (1,), generator=g).item()
        masks[b, 0] = (((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r).float()
    labels = torch.randint(0, 4, (B,), generator=g)
    return dwi, dce, masks, labels


def losses_fixture():
    g = torch.Generator().manual_seed(100)
    B, K = 16, 4
    logits = torch.randn(B, K, generator=g) * 2
    labels = torch.randint(0, K, (B,), generator=g)
    train_labels = torch.cat([torch.zeros(10), torch.ones(3), torch.full((6,), 2), torch.full((1,), 3)]).long()
    cw = OL.class_weights_from_labels(train_labels)
    tgt = OL.label_smoothing(logits, labels, K, 0.1)
    mlog = torch.randn(4, 1, 32, 32, generator=g) * 3
    mtgt = (torch.rand(4, 1, 32, 32, generator=g) > 0.7).float()
    rec = torch.randn(2, 6, 16, 16, generator=g)
    img = torch.rand(2, 6, 64, 64, generator=g)
    s = torch.randn(4, 64, 8, 8, generator=g)
    t = torch.randn(4, 64, 8, 8, generator=g)
    return dict(
        logits=logits.numpy(), labels=labels.numpy(), train_labels=train_labels.numpy(),
        class_weights=cw.numpy(), smooth_targets=tgt.numpy(),
        focal_w=OL.soft_weighted_focal(logits, tgt, 2.0, cw).numpy(),
        focal_w_hard=OL.soft_weighted_focal(logits, labels, 2.0, cw).numpy(),
        focal_rows=OL.soft_weighted_focal(logits, tgt, 2.0, cw, reduction="none").numpy(),
        mask_logits=mlog.numpy(), mask_target=mtgt.numpy(),
        dice=OL.soft_dice(mlog, mtgt).numpy(), dice_bce=OL.dice_bce(mlog, mtgt).numpy(),
        recon=rec.numpy(), image=img.numpy(),
        recon_same=OL.recon_list_loss([rec], img).numpy(),
        recon_mean=OL.recon_list_loss([rec[:, :1]], img).numpy(),
        mimic_s=s.numpy(), mimic_t=t.numpy(), mimic=OL.mimic_feat_loss(s, t).numpy(),
    )


def encoder_fixture():
    P = copy.deepcopy(PR.small_parameters(dropout=0.0))
    _, ref = seeded_encoder(P, "dwi", 14, 11)
    ref.eval()
    dwi, _, _, _ = volume_batch(2, 64, 5)
    with torch.no_grad():
        lo, aux, mp = ref(dwi)
    return dict(recipe=np.array("small_parameters(dropout=0); dwi encoder seed 11; eval"), dwi=dwi.numpy(),
                logits=lo.numpy(), mask_logits=mp.numpy(),
                raw_feat_sums=np.array([f.double().sum().item() for f in aux["raw_feats"]]))


def step_fixture():
    P = copy.deepcopy(PR.small_parameters(dropout=0.0))
    _, dwi_r = seeded_encoder(P, "dwi", 14, 21)
    _, dce_r = seeded_encoder(P, "dce", 6, 22)
    _, fr = seeded_fusion(P, 23)
    for m in (dwi_r, dce_r, fr):
        m.train()
    for p in list(dwi_r.parameters()) + list(dce_r.parameters()):
        p.requires_grad = False
    bt = volume_batch(4, 64, 7)
    train_labels = torch.arange(64) % 4
    out = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, OL.class_weights_from_labels(train_labels), epoch=0)
    out["total"].backward()
    gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for p in fr.parameters()])
    return dict(recipe=np.array("small_parameters(dropout=0); dwi seed 21, dce seed 22, fusion seed 23; train; "
                                "mode A; batch volume_batch(4,64,7); train_labels arange(64)%4"),
                dwi=bt[0].numpy(), dce=bt[1].numpy(), masks=bt[2].numpy(), labels=bt[3].numpy(),
                logits=out["logits"].detach().numpy(),
                terms=np.array([out[k].item() for k in ("cls", "mask", "recon", "mimic", "total")]),
                fusion_grad_norms=gn)


# ---------------------------------------------------------------------------
# SURVEY 8(c) fixtures (2), (4), (5) at the reference's real widths
# (channels 128/256/512, S=256, ResNet-50 OS8 at full width). Inputs are not
# stored: they are re-made from the seeded recipes below (volume_batch,
# backbone_input) with torch's CPU generator.
def feature_stats(f):
    """Per-channel mean and mean square (fp64 reductions) of an NCHW map."""
    f = f.double()
    return np.concatenate([f.mean((0, 2, 3)).numpy(), f.pow(2).mean((0, 2, 3)).numpy()]).astype(np.float64)


def full_encoders(seed_dwi=31, seed_dce=32, seed_fm=33):
    P = copy.deepcopy(PR.default_parameters())
    P["dwi_model_parameters"]["dropout"] = 0.0  # train-mode fixtures with p=0
    _, dwi_r = seeded_encoder(P, "dwi", 14, seed_dwi)
    _, dce_r = seeded_encoder(P, "dce", 6, seed_dce)
    _, fr = seeded_fusion(P, seed_fm)
    return P, dwi_r, dce_r, fr


def config3_forward_fixture():
    """(2) encoder + fusion forward at config-3 shapes, B=2, eval and train (p=0)."""
    P, dwi_r, dce_r, fr = full_encoders()
    dwi, dce, _, _ = volume_batch(2, 256, 9)
    out = {"recipe": np.array("default_parameters(), dropout 0; dwi seed 31, dce seed 32, fusion seed 33 "
                              "(seeded_encoder / seeded_fusion); batch volume_batch(2,256,9)")}
    for mode in ("eval", "train"):
        for m in (dwi_r, dce_r, fr):
            m.train(mode == "train")
        with torch.no_grad():
            lo_d, aux_d, mp_d = dwi_r(dwi)
            lo_c, aux_c, mp_c = dce_r(dce)
            logits, fmask, aux = fr(aux_d["raw_feats"], aux_c["raw_feats"], mp_d, mp_c)
        out.update({
            f"{mode}_dwi_logits": lo_d.numpy(), f"{mode}_dce_logits": lo_c.numpy(),
            f"{mode}_dwi_mask": mp_d.numpy(), f"{mode}_dce_mask": mp_c.numpy(),
            f"{mode}_fusion_logits": logits.numpy(), f"{mode}_fused_mask": fmask.numpy(),
            f"{mode}_gating": aux["gating_weights"].numpy(), f"{mode}_attn": aux["attn_weights"].numpy(),
        })
        for tag, a in (("dwi", aux_d), ("dce", aux_c)):
            for i, f in enumerate(a["raw_feats"]):
                out[f"{mode}_{tag}_f{i + 1}_stats"] = feature_stats(f)
        if mode == "train":
            rs = [b.double().sum().item() for m in (dwi_r, dce_r, fr) for n, b in m.named_buffers()
                  if n.endswith("running_mean") or n.endswith("running_var")]
            out["train_running_stat_sums"] = np.array(rs)
    return out


def config3_adamw_fixture():
    """(4) one mode-A fusion step at config-3 shapes (B=4 so the mimic term is
    on) and the AdamW delta of that step (selector_helpers.py:632-685 frozen
    start: one group, lr 1e-4, wd reg_base 1e-4, eps 1e-8)."""
    P, dwi_r, dce_r, fr = full_encoders(41, 42, 43)
    for m in (dwi_r, dce_r, fr):
        m.train()
    for p in list(dwi_r.parameters()) + list(dce_r.parameters()):
        p.requires_grad = False
    bt = volume_batch(4, 256, 12)
    train_labels = torch.arange(1024) % 4
    out = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, OL.class_weights_from_labels(train_labels), epoch=0)
    out["total"].backward()
    op = P["fusion_model_parameters"]["optimizer_parameters"]
    before = [p.detach().clone() for p in fr.parameters()]
    opt = torch.optim.AdamW([p for p in fr.parameters()], lr=op["lr"], betas=op["betas"], eps=op["eps"],
                            weight_decay=op["reg_base"])
    opt.step()
    gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for p in fr.parameters()])
    dn = np.array([(p.detach() - b).double().norm().item() for p, b in zip(fr.parameters(), before)])
    return dict(recipe=np.array("default_parameters(), dropout 0; dwi seed 41, dce seed 42, fusion seed 43; train; "
                                "mode A; batch volume_batch(4,256,12); train_labels arange(1024)%4; AdamW lr 1e-4 "
                                "wd 1e-4 eps 1e-8"),
                logits=out["logits"].detach().numpy(),
                terms=np.array([out[k].item() for k in ("cls", "mask", "recon", "mimic", "total")]),
                fusion_grad_norms=gn, fusion_delta_norms=dn)


def backbone_input(B, C, S, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, C, S, S, generator=g)


def seeded_backbone(cin, seed):
    """Product-side ResNet-50 OS8 with the encoder's BN re-initialisation
    (initialize_model, model_module.py:1002-1023, quirk Q3) -- timm's
    zero-initialised last BN of each block would leave every residual
    branch silent."""
    P = copy.deepcopy(PR.default_parameters())
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", "dce", cin)
    bb.apply(MM.init_parameter)
    ref = OM.ResNet50OS8(cin)
    ref.load_state_dict(bb.state_dict())
    return bb, ref


def resnet_maps_fixture():
    """(5) ResNet-50 OS8 feature maps at B=1, S=64 (full maps), eval, plus the
    config-2 shape (5 phases, S=256, B=2) as per-channel statistics."""
    _, ref = seeded_backbone(6, 51)
    ref.eval()
    x = backbone_input(1, 6, 64, 52)
    with torch.no_grad():
        feats = ref(x)
    out = {"recipe": np.array("seeded_backbone(6, 51) eval; backbone_input(1,6,64,52); config2: seeded_backbone(5, "
                              "53) eval, backbone_input(2,5,256,54)")}
    for i, f in enumerate(feats):
        out[f"C{i + 2}"] = f.numpy().astype(np.float32)
    _, ref5 = seeded_backbone(5, 53)
    ref5.eval()
    with torch.no_grad():
        feats5 = ref5(backbone_input(2, 5, 256, 54))
    for i, f in enumerate(feats5):
        out[f"config2_C{i + 2}_stats"] = feature_stats(f)
    return out


def reference_layout_ckpt_fixture():
    """A fusion .ckpt in the layout the REFERENCE writes (quirk Q2,
    run_training.py:66-74 / :123-131 / :175, ModelCheckpoint :93-99): the
    encoders are doubly Lightning-wrapped, so their keys read
    ``dwi_model.model.model.<encoder>``; fusion keys ``fusion_model.<...>``;
    Lightning 2.x top-level entries. No-backbone encoders (config 1 widths
    16/32/64) keep the file small. Returns (ckpt dict, expected-output npz
    dict): the oracle's eval-mode logits / fused mask on volume_batch(2,64,91)."""
    P = copy.deepcopy(PR.small_parameters(dropout=0.0, use_backbone=False))
    encs = {}
    for name, cin, seed in (("dwi", 14, 61), ("dce", 6, 62)):
        torch.manual_seed(seed)
        enc = MM.initialize_model(MM.ModelMaskHeadBackbone(name, P, None), True)
        ref = OM.ModelMaskHeadBackbone(name, P, None)
        ref.load_state_dict(enc.state_dict())
        encs[name] = ref
    _, fr = seeded_fusion(P, 63)
    sd = {}
    for name in ("dwi", "dce"):
        for k, v in encs[name].state_dict().items():
            sd[f"{name}_model.model.model.{k}"] = v.clone()
    for k, v in fr.state_dict().items():
        sd[f"fusion_model.{k}"] = v.clone()
    ckpt = {"epoch": 17, "global_step": 544, "pytorch-lightning_version": "2.5.1", "state_dict": sd,
            "loops": {}, "callbacks": {}, "optimizer_states": [], "lr_schedulers": []}
    dwi, dce, _, _ = volume_batch(2, 64, 91)
    for m in (encs["dwi"], encs["dce"], fr):
        m.eval()
    with torch.no_grad():
        _, aux_d, mp_d = encs["dwi"](dwi)
        _, aux_c, mp_c = encs["dce"](dce)
        logits, fmask, _ = fr(aux_d["raw_feats"], aux_c["raw_feats"], mp_d, mp_c)
    out = {"recipe": np.array("small_parameters(dropout=0, use_backbone=False); dwi seed 61, dce seed 62 "
                              "(initialize_model), fusion seed 63; eval; batch volume_batch(2,64,91)"),
           "logits": logits.numpy(), "fused_mask": fmask.numpy()}
    return ckpt, out


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    which = set(sys.argv[1:]) or {"small", "full"}
    if "small" in which:
        np.savez_compressed(os.path.join(OUT, "losses.npz"), **losses_fixture())
        np.savez_compressed(os.path.join(OUT, "encoder_small.npz"), **encoder_fixture())
        np.savez_compressed(os.path.join(OUT, "fusion_step_small.npz"), **step_fixture())
    if "ckpt" in which or "small" in which:
        ckpt, out = reference_layout_ckpt_fixture()
        torch.save(ckpt, os.path.join(OUT, "fusion_reference_layout.ckpt"))
        np.savez_compressed(os.path.join(OUT, "fusion_reference_layout.npz"), **out)
    if "full" in which:
        np.savez_compressed(os.path.join(OUT, "config3_forward.npz"), **config3_forward_fixture())
        np.savez_compressed(os.path.join(OUT, "config3_adamw_step.npz"), **config3_adamw_fixture())
        np.savez_compressed(os.path.join(OUT, "resnet50_os8_maps.npz"), **resnet_maps_fixture())
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
