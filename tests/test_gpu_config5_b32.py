"""GPU: configuration 5's PRODUCTION launch plan (B=32, S=384, fp8-e4m3
patch-embed, bf16 elsewhere) against the CPU oracle.

The hybrid TransformerStage encoders (transformer_model.py:137-175 in place of
block3; E=512, depth 6, 4 heads, patch 2 -> 576 tokens per volume) inside one
CAPTURED FusionTrainer mode-A step, as bench.py's config-5 line runs it. At
B=32 the 48x48 backbone maps give the 256-wide LDS-DMA conv forms >= 256
tiles, the token GEMMs run at M = 32 * 576 = 18,432 rows and the e4m3
patch-embed GEMM at M = 18,432, K = 1,024; at the B=2 of
test_gpu_config5_full none of that is exercised. The launch records
(dmf_ops.PROBE) must show those forms and GEMMs, and the step is compared with
oracle.losses.fusion_shared_step on the same state_dict and batch:

  * logits: relative L2 error against the fp32 oracle no larger than 1.5x the
    reference's own mixed precision (the fp32 oracle under CPU bf16 autocast
    with the e4m3-quantised PatchEmbed.proj, test_gpu_config5_full
    .fp8_patch_embed_oracle) + 1e-2 -- a zero output fails;
  * the loss within 3e-2 relative, and the fusion gradients no further from
    the fp32 oracle than 1.25x the yardstick's (+ 0.01), as
    test_gpu_config3_b32.
Reference: transformer_model.py:7-32, :68-134; train_fusion.py:204-321."""
import copy
import json
import os

import pytest
import torch

import dmf_ops as O
import make_golden as MG
import model_module as MM
import parameters as PR
import train_fusion as TF
from oracle import losses as OL
from selector_helpers import get_classification_loss
from test_gpu_config3_b32 import _fusion_grads, _rel_l2, _report
from test_gpu_config5_full import fp8_patch_embed_oracle, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, S = 32, 384
TOKENS = B * (S // 8 // 2) ** 2  # f2 at S/8 = 48, patch 2 -> 24 x 24 = 576 per volume


def _params():
    P = copy.deepcopy(PR.default_parameters())
    mp = P["dwi_model_parameters"]
    mp["dropout"] = 0.0
    mp["use_hybrid_transformer"] = True
    mp["patch_embed_fp8"] = True
    mp["input_size"] = S
    return P


@pytest.mark.timeout(1100)
def test_config5_b32_captured_step_production_plan_vs_oracle():
    from dmf_dp import FusionTrainer

    P = _params()
    dwi, dwi_r = MG.seeded_encoder(P, "dwi", 14, 61)
    dce, dce_r = MG.seeded_encoder(P, "dce", 6, 62)
    fm, fr = MG.seeded_fusion(P, 63)
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    assert dwi.transformer.patch_embed.use_fp8 and dce.transformer.patch_embed.use_fp8
    amp = [copy.deepcopy(m) for m in (dwi_r, dce_r, fr)]
    crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi.to(DEV), dce.to(DEV), fm.to(DEV), P, crit)
    lm.train()
    tr = FusionTrainer(lm, world=1, use_graph=True)
    bt = MG.volume_batch(B, S, 29)
    bd = tuple(t.to(DEV) for t in bt)
    recs = {k: [] for k in ("conv_fwd", "tok_gemm", "fp8_gemm")}
    for k, v in recs.items():
        O.PROBE[k] = v
    try:
        tr.capture(bd)  # eager warm-ups (recorded) + the captured graphs; the training state is restored
    finally:
        for k in recs:
            O.PROBE[k] = None
    forms = sorted({r["form"] for r in recs["conv_fwd"]})
    # token rows per record: dmf_gemm_* (batch, M, ...) / conv-engine linears (N, H, W, ...: the rows' NHWC
    # view) / the fused attention ("flash", b, n, ...)
    def _rows(r):
        sh = r["shape"]
        if r["fn"].startswith("dmf_conv2d"):
            return sh[0] * sh[1] * sh[2]
        if r["fn"] == "dmf_flash_attn_fwd":
            return sh[1] * sh[2]
        return sh[1]
    tok_m = sorted({_rows(r) for r in recs["tok_gemm"]})
    tok_fns = sorted({r["fn"] for r in recs["tok_gemm"]})
    fp8_shapes = sorted({tuple(r["shape"]) for r in recs["fp8_gemm"]})
    for v in recs.values():
        v.clear()
    # the production plan: 256-wide LDS-DMA forward forms and the 7x7 stem kernel on the 48x48 maps,
    # token GEMMs over all 18,432 token rows, the e4m3 patch-embed GEMM at M = 18,432
    assert {"ps", "stem"} <= set(forms) and ({"pp", "wide"} & set(forms)), forms
    assert tok_m == [TOKENS] and "dmf_flash_attn_fwd" in tok_fns, (TOKENS, tok_m, tok_fns)
    assert fp8_shapes and all(s[0] == TOKENS for s in fp8_shapes), fp8_shapes
    loss = tr.step(bd).item()  # one replay of the captured step
    assert tr.captures == 1 and tr.eager_steps == 0
    with torch.no_grad():
        _, logits, _, _ = lm._shared_step(bd, "train", return_preds=True)
    logits = logits.float().cpu()
    got = _fusion_grads(fm)

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cw = OL.class_weights_from_labels(torch.arange(1024) % 4)
    for m in (dwi_r, dce_r, *amp[:2]):
        for p in m.parameters():
            p.requires_grad = False
    for m in (dwi_r, dce_r, fr, *amp):
        m.train()
    # (the forward re-run above saw the post-step fusion weights: its logits are compared with an oracle
    # forward on those same weights below, the step's loss / gradients with the pre-step oracle step)
    ref = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
    ref["total"].backward()
    with torch.autocast("cpu", dtype=torch.bfloat16), fp8_patch_embed_oracle():
        ref_amp = OL.fusion_shared_step(amp[0], amp[1], amp[2], bt, P, cw, epoch=0)
    ref_amp["total"].float().backward()
    truth = _fusion_grads(fr)
    assert set(got) == set(truth), sorted(set(got) ^ set(truth))
    e_hip, med_hip = _rel_l2(got, truth)
    e_amp, med_amp = _rel_l2(_fusion_grads(amp[2]), truth)
    lrel = abs(loss - ref["total"].item()) / max(1.0, abs(ref["total"].item()))

    # logits on the post-step weights: the oracle and its AMP yardstick after loading them
    fr2 = copy.deepcopy(fr)
    fr2.load_state_dict({k: v.detach().float().cpu() for k, v in fm.state_dict().items()})
    amp2 = copy.deepcopy(fr2)
    with torch.no_grad():
        want = OL.fusion_shared_step(dwi_r, dce_r, fr2, bt, P, cw, epoch=0)["logits"].float()
        with torch.autocast("cpu", dtype=torch.bfloat16), fp8_patch_embed_oracle():
            yard = OL.fusion_shared_step(copy.deepcopy(dwi_r), copy.deepcopy(dce_r), amp2, bt, P, cw,
                                         epoch=0)["logits"].float()
    l_hip, l_amp = rel_l2(logits, want), rel_l2(yard, want)
    _report("config5_b32_captured_mode_a_step_bf16_fp8_vs_fp32_oracle",
            {"forms": forms, "token_gemm_rows": tok_m, "fp8_gemm_shapes": [list(s) for s in fp8_shapes],
             "loss": {"hip": loss, "oracle": ref["total"].item(), "rel": lrel},
             "logits_rel_l2": {"hip_bf16_fp8": l_hip, "reference_bf16_autocast_fp8_patch_embed": l_amp},
             "fusion_grads_rel_l2": {"hip_bf16_fp8": e_hip, "hip_median_tensor": med_hip,
                                     "reference_amp": e_amp, "reference_median_tensor": med_amp}})
    assert lrel < 3e-2, lrel
    bar = 1.5 * l_amp + 1e-2
    assert l_hip <= bar, (l_hip, l_amp)
    assert rel_l2(torch.zeros_like(logits), want) > bar
    assert e_hip <= 1.25 * e_amp + 0.01, (e_hip, e_amp)
    print(json.dumps({"logits_rel": [l_hip, l_amp], "grads_rel": [e_hip, e_amp], "loss_rel": lrel}))
