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
   report separately"): relative L2 logit error against the fp32 oracle, GATED
   against the reference's own mixed precision on the same weights and batch
   (an absolute bar above the logits' own magnitude let a
   zero forward pass) -- the fp32 oracle under CPU bf16 autocast
   (parameters_generate.py:211, run.py:59-76), and for the fp8 variant the same
   autocast with PatchEmbed.proj on the e4m3-quantised operands
   (``fp8_patch_embed_oracle``: per-token-row / per-output-channel amax / 448
   scales, torch.float8_e4m3fn rounding, fp32 product -- what k_gemm_fp8
   computes). Gated on the classifier head's input (the 2 x 128 pooled fused features):
   hip_rel <= 1.5 * yardstick_rel + 1e-2, and a zero output fails; the logits' error must be the head's
   image of that input error (<= its operator norm x the pooled error) and within 3x the yardstick's.
"""
import contextlib
import json
import os

import pytest
import torch

import dmf_ops as O
import model_module as MM
import parameters as PR
import train_fusion as TF
from oracle import losses as OL
from oracle import model as OM
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


def _q_e4m3_rows(m):
    """per-row amax / 448 scaling, OCP e4m3fn rounding, dequantised (fp32)."""
    sc = m.abs().amax(1, keepdim=True).clamp_min(1e-30) / 448.0
    return (m / sc).to(torch.float8_e4m3fn).float() * sc


@contextlib.contextmanager
def fp8_patch_embed_oracle():
    """The oracle's PatchEmbed (transformer_model.py:7-32) with its projection on
    e4m3-quantised operands, as config 5's fp8 patch-embed computes it: patch
    rows in (r, s, c) order quantised per token row, the weight per output
    channel, fp32 product of the dequantised operands + bias."""
    orig = OM.PatchEmbed.forward

    def fwd(self, x):
        n, c, h, w = x.shape
        p = self.proj.kernel_size[0]
        e = self.proj.out_channels
        with torch.autocast("cpu", enabled=False):
            rows = x.float().reshape(n, c, h // p, p, w // p, p).permute(0, 2, 4, 3, 5, 1).reshape(-1, p * p * c)
            wt = self.proj.weight.float().permute(0, 2, 3, 1).reshape(e, -1)
            y = _q_e4m3_rows(rows) @ _q_e4m3_rows(wt).t() + self.proj.bias.float()
        y = y.reshape(n, h // p, w // p, e).permute(0, 3, 1, 2)
        t = y.flatten(2).transpose(1, 2)
        return torch.nn.functional.layer_norm(t, t.shape[-1:], self.norm.weight, self.norm.bias, self.norm.eps), \
            (h // p, w // p)

    OM.PatchEmbed.forward = fwd
    try:
        yield
    finally:
        OM.PatchEmbed.forward = orig


@contextlib.contextmanager
def head_input(weight, rec, mod):
    """Record the classifier head's input (the pooled fused features, FusionModel.classifier[2]'s
    input; model_module.py:819 / oracle/model.py:740) when ``mod.linear`` runs on ``weight``."""
    orig = mod.linear

    def linear(x, w, b=None, *a, **k):
        if w is weight and "pooled" not in rec:
            rec["pooled"] = x.detach().float().cpu()
        return orig(x, w, b, *a, **k)
    mod.linear = linear
    try:
        yield rec
    finally:
        mod.linear = orig


def amp_yardstick(models, batch_cpu, P, cw, fp8, rec=None):
    """logits of the fp32 oracle under CPU bf16 autocast (+ the fp8 patch-embed), on copies of ``models``
    (``rec``: receives the head's pooled input)."""
    import copy as _copy
    import torch.nn.functional as F

    mods = [_copy.deepcopy(m) for m in models]
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16), \
            (fp8_patch_embed_oracle() if fp8 else contextlib.nullcontext()), \
            head_input(mods[2].classifier[2].weight, rec if rec is not None else {}, F):
        out = OL.fusion_shared_step(mods[0], mods[1], mods[2], batch_cpu, P, cw, epoch=0)
    return out["logits"].float()


def rel_l2(got, want):
    return ((got.float() - want).norm() / want.norm().clamp_min(1e-30)).item()


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
    import torch.nn.functional as F
    ref_rec = {}
    with head_input(fr.classifier[2].weight, ref_rec, F):
        ref = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
    ref["total"].backward()
    want = ref["logits"].detach()
    want_pooled = ref_rec["pooled"]
    w_head = fr.classifier[2].weight.detach().double()
    head_norm = torch.linalg.matrix_norm(w_head, ord=2).item()  # the head's operator norm
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

    # ---- 2. bf16 and bf16 + fp8 patch-embed on the same weights, gated against the reference's AMP
    report = {"shape": "S=384, 576 tokens, E=512, depth 6, 4 heads, widths 128/256/512, B=2",
              "f32_logits_max_abs": lerr}
    scale = want.abs().max().item()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    for tag, fp8 in (("bf16", False), ("bf16_fp8_patch_embed", True)):
        for m in (dwi_m, dce_m, fm):
            MM.set_compute_dtype(m, torch.bfloat16)
        for m in (dwi_m, dce_m):
            m.transformer.patch_embed.use_fp8 = fp8
        hip_rec, amp_rec = {}, {}
        with torch.no_grad(), head_input(fm.classifier[2].weight, hip_rec, O):
            _, lg, _, _ = lm._shared_step(bd, "train", return_preds=True)
        lg = lg.float().cpu()
        e = (lg - want).abs().max().item()
        yard = amp_yardstick((dwi_r, dce_r, fr), bt, P, cw, fp8, amp_rec)
        e_rel, y_rel = rel_l2(lg, want), rel_l2(yard, want)
        p_rel, py_rel = rel_l2(hip_rec["pooled"], want_pooled), rel_l2(amp_rec["pooled"], want_pooled)
        d_pooled = (hip_rec["pooled"].double() - want_pooled.double()).norm().item()
        d_logits = (lg.double() - want.double()).norm().item()
        report[tag] = {"logits_max_abs": e, "logits_rel_to_max": e / max(scale, 1e-12), "logits_rel_l2": e_rel,
                       "reference_amp_rel_l2": y_rel, "pooled_rel_l2": p_rel, "reference_amp_pooled_rel_l2": py_rel,
                       "logits_err_l2": d_logits, "head_norm_x_pooled_err_l2": head_norm * d_pooled,
                       "reference_amp": "fp32 oracle under CPU bf16 autocast" +
                                        (" + e4m3-quantised PatchEmbed.proj" if fp8 else "")}
        assert torch.isfinite(lg).all()
        # gate 1: the classifier head's input, the 2 x 128 pooled fused features, relative to the
        # reference's own mixed precision (the logits are only 8 numbers: their relative L2 is dominated
        # by how the input error happens to align with the head's rows -- r05: pooled 0.0161 vs AMP
        # 0.0162, logits 0.0556 vs AMP 0.0290, tools/config5_stage_errors.py)
        bar = 1.5 * py_rel + 1e-2
        assert p_rel <= bar, (tag, p_rel, py_rel)
        assert rel_l2(torch.zeros_like(hip_rec["pooled"]), want_pooled) > bar  # a zero forward fails
        # gate 2: the logits' error is the head's image of its input's error, nothing more (operator norm;
        # the head runs fp32 on the pooled features)
        assert d_logits <= 1.05 * head_norm * d_pooled + 1e-6, (tag, d_logits, head_norm * d_pooled)
        # and the logits stay within the reference-AMP yardstick's order of magnitude
        assert e_rel <= 3.0 * y_rel + 1e-2, (tag, e_rel, y_rel)
    print("config 5 numerics vs fp32 oracle:", json.dumps(report))
    # SURVEY 8(d) "Tolerances": fp8 reported separately -- always written (copied into profiles/ per round)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "config5_numerics.json"), "w") as f:
        json.dump(report, f, indent=1)
