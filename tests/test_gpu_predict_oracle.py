"""MC dropout x TTA against the CPU oracle (SURVEY 8(f)
rank 2; train_fusion.py:484-632, flips train.py:916-923).

* predict_tta (eval): the build's batched flips vs oracle.predict.predict_tta
  (the reference's per-flip loop) -- mean, std and mean gating;
* predict_mc_dropout / predict_tta_mc with p = 0: the stochastic passes
  collapse to the eval forward on both sides (std 0);
* one MC pass with p > 0 and SHARED masks: the build's encoders draw their
  Philox masks (dmf_dropout_keep_mask reproduces them from the snapshot and
  site), the oracle's ResNetLiteBlock dropouts take the same masks in call
  order (oracle.model.DROPOUT_MASKS) -- logits must agree to fp32 rounding.
f32 parity mode, small widths (16/32/64, S=64)."""
import copy

import pytest
import torch

import dmf_native as N
import dmf_ops as O
import make_golden as MG
import model_module as MM
import parameters as PR
import train_fusion as TF
from oracle import model as OM
from oracle import predict as OP
from selector_helpers import get_classification_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(p=0.2, seed=0):
    P = copy.deepcopy(PR.small_parameters(dropout=p))
    dwi, dwi_r = MG.seeded_encoder(P, "dwi", 14, 81 + seed)
    dce, dce_r = MG.seeded_encoder(P, "dce", 6, 82 + seed)
    fm, fr = MG.seeded_fusion(P, 83 + seed)
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.float32)
    crit = get_classification_loss(P, torch.arange(64) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi.to(DEV), dce.to(DEV), fm.to(DEV), P, crit)
    lm.eval()
    for m in (dwi_r, dce_r, fr):
        m.eval()
    return lm, (dwi_r, dce_r, fr)


def _zero_dropout(*mods):
    for mod in mods:
        for m in mod.modules():
            if hasattr(m, "p") and isinstance(getattr(m, "p"), float):
                m.p = 0.0


def _close(a, b, tol, what):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    err = (a - b).abs().max().item()
    assert err <= tol, f"{what}: max err {err:.3e}"


def test_tta_matches_oracle_loop():
    lm, (dr, cr, fr) = _pair()
    dwi, dce, _, _ = MG.volume_batch(3, 64, 21)
    mean, std, aux = lm.predict_tta(dwi.to(DEV), dce.to(DEV))
    om, os_, og = OP.predict_tta(dr, cr, fr, dwi, dce)
    _close(mean, om, 1e-4, "tta mean")
    _close(std, os_, 1e-4, "tta std")
    _close(aux["gating_weights"], og, 1e-4, "tta gating")
    assert std.abs().max().item() > 1e-5  # the flips matter


def test_mc_and_tta_mc_p0_match_oracle():
    lm, (dr, cr, fr) = _pair()
    _zero_dropout(lm, dr, cr, fr)
    dwi, dce, _, _ = MG.volume_batch(2, 64, 22)
    mean, std, aux = lm.predict_mc_dropout(dwi.to(DEV), dce.to(DEV), passes=3)
    om, os_, og = OP.predict_mc_dropout(dr, cr, fr, dwi, dce, passes=3)
    _close(mean, om, 1e-4, "mc mean")
    assert std.abs().max().item() < 1e-6 and os_.abs().max().item() < 1e-6
    _close(aux["gating_weights"], og, 1e-4, "mc gating")
    mean, std, aux = lm.predict_tta_mc(dwi.to(DEV), dce.to(DEV), passes=2)
    om, os_, og = OP.predict_tta_mc(dr, cr, fr, dwi, dce, passes=2)
    _close(mean, om, 1e-4, "tta_mc mean")
    _close(std, os_, 1e-4, "tta_mc std")
    _close(aux["gating_weights"], og, 1e-4, "tta_mc gating")


def _keep(rng, site, shape_nhwc, p):
    n = 1
    for s in shape_nhwc:
        n *= s
    keep = torch.empty(n, dtype=torch.uint8, device=DEV)
    N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, n, p, keep.data_ptr(), N.stream_ptr())
    # the build's element index is the NHWC linear index (row m = (n*H + h)*W + w, channel c)
    return (keep.float().cpu().view(*shape_nhwc) / (1 - p)).permute(0, 3, 1, 2).contiguous()


def test_mc_pass_with_shared_masks_matches_oracle():
    p = 0.2
    lm, (dr, cr, fr) = _pair(p, seed=1)
    dwi, dce, _, _ = MG.volume_batch(2, 64, 23)
    lm.mc_enable(lm.dwi_model)
    lm.mc_enable(lm.dce_model)
    OP.mc_enable(dr)
    OP.mc_enable(cr)
    masks = []
    for enc, x, ref in ((lm.dwi_model, dwi, dr), (lm.dce_model, dce, cr)):
        calls = []
        hooks = [m.register_forward_hook(lambda mod, inp, out: calls.append((mod, tuple(inp[0].shape),
                                                                              tuple(out[0].shape))))
                 for m in enc.modules() if isinstance(m, MM.ResNetLiteBlock_withRecon)]
        snap = O.RNG.snapshot(DEV)
        O.RNG_CURRENT[0] = snap
        try:
            with torch.no_grad():
                out = enc(x.to(DEV))
        finally:
            O.RNG_CURRENT[0] = None
            for h in hooks:
                h.remove()
        assert calls, "no ResNetLiteBlock_withRecon ran"
        enc_masks = []
        for mod, (n, _, h, w), (_, co, ho, wo) in calls:
            site_a, site_b = mod._sites[0]
            s = mod.bottlenecks[0][0].stride[0]
            mid = mod.bottlenecks[0][0].out_channels
            enc_masks.append(_keep(snap, site_a, (n, (h - 1) // s + 1, (w - 1) // s + 1, mid), p))
            enc_masks.append(_keep(snap, site_b, (n, ho, wo, co), p))
        OM.DROPOUT_MASKS = list(enc_masks)
        try:
            with torch.no_grad():
                ref_out = ref(x)
        finally:
            left = len(OM.DROPOUT_MASKS)
            OM.DROPOUT_MASKS = None
        assert left == 0, f"{left} masks unused: the oracle ran fewer dropouts than the build"
        _close(out[0], ref_out[0], 1e-3, "encoder logits (shared masks)")
        for i, (a, b) in enumerate(zip(out[1]["raw_feats"], ref_out[1]["raw_feats"])):
            _close(a, b, 1e-3 * max(1.0, b.abs().max().item()), f"raw_feats[{i}] (shared masks)")
        masks.append(enc_masks)
    # the masks are real dropout masks (some elements dropped, scale 1/(1-p))
    for m in (m for ms in masks for m in ms):
        assert (m == 0).any() and abs(m.max().item() - 1 / (1 - p)) < 1e-6
