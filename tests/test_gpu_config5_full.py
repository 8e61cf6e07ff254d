"""Config 5 at its own shape (VERDICT r02 "Next" 2).

The hybrid TransformerStage encoders (transformer_model.py:137-175 replacing
block3, model_module.py:564-579 / :701-703) at the configuration's real
shape -- S=384 (f2 48x48 -> 576 tokens), E=512, depth 6, 4 heads, patch 2,
widths 128/256/512 (parameters_generate.py:71-75, :82) -- inside the fusion
step, B=2, mode A (encoders frozen in train mode, reference default at
epoch 0):

1. f32 parity mode (every GEMM on the exact f32 MFMA) against the CPU oracle
   on one state_dict and one batch: logits within 1e-3, the loss within 1e-4
   relative, every fusion gradient within 2e-3 of its tensor's max.
2. The throughput numerics of config 5 on the same weights: bf16 everywhere,
   then bf16 with the fp8-e4m3 patch-embed (SURVEY 8(d) "fp8 patch-embed:
   report separately"): max-abs and relative logit error against the fp32
   oracle, printed side by side, gated at the bf16 bound of the other parity
   tests (5e-2).
"""
import json
import os

import pytest
import torch

import model_module as MM
import parameters as PR
import train_fusion as TF
from oracle import losses as OL
from selector_helpers import get_classification_loss
from test_gpu_parity import _fusion_pair, batch, build_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _config5_params():
    P = PR.small_parameters(channels=(128, 256, 512), input_size=384, dropout=0.0)
    mp = P["dwi_model_parameters"]
    mp["use_hybrid_transformer"] = True
    mp["transformer_embed_dim"] = 512
    mp["transformer_depth"] = 6
    mp["transformer_heads"] = 4
    mp["transformer_patch_size"] = 2
    return P


def _no_dropout(*models):
    for m in models:
        for mod in m.modules():
            if hasattr(mod, "p") and isinstance(getattr(mod, "p"), float):
                mod.p = 0.0


@pytest.mark.timeout(600)
def test_config5_full_shape_fusion_step_f32_and_fp8_report():
    P = _config5_params()
    dwi_m, dwi_r, P1 = build_pair(P, "dwi", 14, 51)
    dce_m, dce_r, _ = build_pair(P, "dce", 6, 52)
    P = P1
    fm, fr = _fusion_pair(P, 53)
    _no_dropout(dwi_m, dce_m, fm, dwi_r, dce_r, fr)
    assert len(dwi_m.transformer.transformer.layers) == 6 and dwi_m.transformer.transformer.layers[0].attn is not None
    train_labels = torch.arange(64) % 4
    crit = get_classification_loss(P, train_labels, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi_m, dce_m, fm, P, crit)
    lm.train()
    for m in (dwi_r, dce_r, fr):
        m.train()
    for p in list(dwi_r.parameters()) + list(dce_r.parameters()):
        p.requires_grad = False
    bt = batch(2, 384, 19)
    bd = tuple(t.to(DEV) for t in bt)

    # ---- 1. f32 parity
    with torch.no_grad():
        _, logits, aux, _ = lm._shared_step(bd, "train", return_preds=True)
    assert aux["attn_weights"] is not None
    loss = lm.training_step(bd)
    loss.backward()
    cw = OL.class_weights_from_labels(train_labels)
    ref = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
    ref["total"].backward()
    want = ref["logits"].detach()
    lerr = (logits.float().cpu() - want).abs().max().item()
    print(f"config 5 full shape f32: logits max err {lerr:.2e}; loss {loss.item():.6f} vs {ref['total'].item():.6f}")
    assert lerr <= 1e-3, lerr
    assert abs(loss.item() - ref["total"].item()) <= 1e-4 * max(1, abs(ref["total"].item()))
    for (n, p1), (_, p2) in zip(fm.named_parameters(), fr.named_parameters()):
        if p2.grad is None:
            continue
        tol = 2e-3 * max(1e-3, p2.grad.abs().max().item())
        err = (p1.grad.cpu().reshape(p2.grad.shape) - p2.grad).abs().max().item()
        assert err < tol, (n, err, tol)

    # ---- 2. bf16 and bf16 + fp8 patch-embed on the same weights
    report = {"shape": "S=384, 576 tokens, E=512, depth 6, 4 heads, widths 128/256/512, B=2",
              "f32_logits_max_abs": lerr}
    scale = want.abs().max().item()
    for tag, fp8 in (("bf16", False), ("bf16_fp8_patch_embed", True)):
        for m in (dwi_m, dce_m, fm):
            MM.set_compute_dtype(m, torch.bfloat16)
        for m in (dwi_m, dce_m):
            m.transformer.patch_embed.use_fp8 = fp8
        with torch.no_grad():
            _, lg, _, _ = lm._shared_step(bd, "train", return_preds=True)
        e = (lg.float().cpu() - want).abs().max().item()
        report[tag] = {"logits_max_abs": e, "logits_rel_to_max": e / max(scale, 1e-12)}
        assert torch.isfinite(lg).all()
        assert e <= 5e-2, (tag, e)
    print("config 5 numerics vs fp32 oracle:", json.dumps(report))
    # SURVEY 8(d) "Tolerances": fp8 reported separately -- always written (copied into profiles/ per round)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "config5_numerics.json"), "w") as f:
        json.dump(report, f, indent=1)
