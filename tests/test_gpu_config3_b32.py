"""GPU: the PRODUCTION bf16 launch plan at configuration 3's own shape (B=32,
S=256, default widths) against the CPU oracle.

The 256-wide LDS-DMA forward forms that carry the benchmark (k_conv_fwd_ps /
_pp / _wide and the 7x7 stem kernel) engage only at >= 256 output tiles
(conv.hip conv_plan, g_min_tiles): at B <= 4 -- every other model-level test
-- a layer-4 launch has 128 tiles and runs on the small buffer-load tiles. So
this file runs the model at the batch that selects them, asserts from the
launch records (dmf_conv_last_form) that they were chosen, and compares with
oracle.model / oracle.losses on the same state_dict and inputs:

  * encoder + fusion forward, eval and train mode (train-mode BN: batch
    statistics and running-stat updates; dropout 0), through the product's
    two-stream _encode as the training step runs it
    (reference model_module.py:645-733, :919-1000);
  * one CAPTURED FusionTrainer mode-A step (reference train_fusion.py:204-321,
    encoders frozen in train mode, backward + AdamW through FusionModel).

Tolerances: bf16 logits within 5e-2 absolute of the fp32 oracle (the gate;
the measured max-abs / relative errors go to gpurun_out/bf16_errors.json and
profiles/). Everything else against the reference's own bf16-mixed AMP (the
fp32 oracle under CPU bf16 autocast, parameters_generate.py:211): the masks,
gating / attention weights, per-channel f1..f3 statistics and running-stat
sums no further from the fp32 oracle than 1.5x the reference-AMP error (+ a
small floor) -- train-mode BN renormalises every layer by batch statistics,
so bf16 rounding moves e.g. the mask logits by ~0.1 in the reference's AMP
too. The step: loss within 3e-2 and the fusion gradients no further from the
fp32 oracle than 1.25x the reference-AMP gradients (+0.01), the yardstick of
test_gpu_golden_full.test_mode_b_bf16_full_width_step_vs_oracle."""
import copy
import json
import os

import numpy as np
import pytest
import torch

import dmf_ops as O
import make_golden as MG
import model_module as MM
import parameters as PR
import train_fusion as TF
from selector_helpers import get_classification_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, S = 32, 256
REPORT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "bf16_errors.json")
# the bodies that carry the benchmark's conv forward (r03t mode-A kernel stats)
BENCH_FORMS = {"ps", "pp", "wide", "stem"}


def _report(key, val):
    os.makedirs(os.path.dirname(REPORT), exist_ok=True)
    d = {}
    if os.path.exists(REPORT):
        with open(REPORT) as f:
            d = json.load(f)
    d[key] = val
    with open(REPORT, "w") as f:
        json.dump(d, f, indent=1)
    print(key, json.dumps(val))


def _models(P, seeds):
    dwi, dwi_r = MG.seeded_encoder(P, "dwi", 14, seeds[0])
    dce, dce_r = MG.seeded_encoder(P, "dce", 6, seeds[1])
    fm, fr = MG.seeded_fusion(P, seeds[2])
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    return (dwi.to(DEV), dce.to(DEV), fm.to(DEV)), (dwi_r, dce_r, fr)


def _params():
    P = copy.deepcopy(PR.default_parameters())
    P["dwi_model_parameters"]["dropout"] = 0.0  # aliases the dce / fusion dicts (quirk Q1)
    return P


def _err(got, want):
    g = got.float().cpu().numpy()
    w = want.detach().float().numpy()
    return {"max_abs": float(np.abs(g - w).max()), "rel": float(np.linalg.norm(g - w) / max(1e-12, np.linalg.norm(w)))}


def _stats_err(got, want):
    a, b = MG.feature_stats(got.float().cpu()), MG.feature_stats(want.detach())
    c = b.shape[0] // 2
    return max(float(np.abs(a[:c] - b[:c]).max() / max(1e-6, np.abs(b[:c]).max())),
               float(np.abs(a[c:] - b[c:]).max() / max(1e-6, np.abs(b[c:]).max())))


def _forms(recs):
    return sorted({r["form"] for r in recs})


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["eval", "train"])
def test_config3_b32_bf16_forward_vs_oracle(mode):
    P = _params()
    (dwi, dce, fm), (dwi_r, dce_r, fr) = _models(P, (71, 72, 73))
    crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi, dce, fm, P, crit)
    lm.train(mode == "train")
    for m in (dwi_r, dce_r, fr):
        m.train(mode == "train")
    x_dwi, x_dce, _, _ = MG.volume_batch(B, S, 19)
    recs = []
    O.PROBE["conv_fwd"] = recs
    try:
        with torch.no_grad():
            (lo_d, aux_d, mp_d), (lo_c, aux_c, mp_c) = lm._encode(x_dwi.to(DEV), x_dce.to(DEV))
            logits, fmask, aux = fm(aux_d["raw_feats"], aux_c["raw_feats"], mp_d, mp_c)
        torch.cuda.synchronize()
    finally:
        O.PROBE["conv_fwd"] = None
    forms = _forms(recs)
    recs.clear()
    assert BENCH_FORMS <= set(forms), forms

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    # the reference's own bf16-mixed (parameters_generate.py:211, run.py:59-76): the fp32 oracle under CPU bf16
    # autocast, from the same state (copied before the fp32 forward moves the running statistics)
    amp = [copy.deepcopy(m) for m in (dwi_r, dce_r, fr)]

    def oracle(mods):
        with torch.no_grad():
            lo1, a1, m1 = mods[0](x_dwi)
            lo2, a2, m2 = mods[1](x_dce)
            lf, mf, af = mods[2](a1["raw_feats"], a2["raw_feats"], m1, m2)
        return (lo1, lo2, lf, m1, m2, mf, af["gating_weights"], af["attn_weights"]), (a1, a2)

    want, (ar_d, ar_c) = oracle((dwi_r, dce_r, fr))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ref_amp, (am_d, am_c) = oracle(amp)
    names = ("dwi_logits", "dce_logits", "fusion_logits", "dwi_mask", "dce_mask", "fused_mask", "gating", "attn")
    mine = (lo_d, lo_c, logits, mp_d, mp_c, fmask, aux["gating_weights"], aux["attn_weights"])
    out = {"forms": forms, "hip_bf16": {}, "reference_bf16_autocast": {}}
    for name, got, w, r in zip(names, mine, want, ref_amp):
        out["hip_bf16"][name] = _err(got, w)
        out["reference_bf16_autocast"][name] = _err(r, w)
    out["hip_bf16"]["feature_stats_rel"] = {f"{tag}_f{i + 1}": _stats_err(a, b)
                                            for tag, ga, wa in (("dwi", aux_d, ar_d), ("dce", aux_c, ar_c))
                                            for i, (a, b) in enumerate(zip(ga["raw_feats"], wa["raw_feats"]))}
    out["reference_bf16_autocast"]["feature_stats_rel"] = {
        f"{tag}_f{i + 1}": _stats_err(a, b) for tag, ga, wa in (("dwi", am_d, ar_d), ("dce", am_c, ar_c))
        for i, (a, b) in enumerate(zip(ga["raw_feats"], wa["raw_feats"]))}

    def stat_sums(mods):
        return np.array([b.double().sum().item() for m in mods for n, b in m.named_buffers()
                         if n.endswith("running_mean") or n.endswith("running_var")])

    if mode == "train":
        w = stat_sums((dwi_r, dce_r, fr))
        for tag, mods in (("hip_bf16", (dwi, dce, fm)), ("reference_bf16_autocast", amp)):
            g = stat_sums(mods)
            assert g.shape == w.shape
            out[tag]["running_stat_sums_rel"] = float((np.abs(g - w) / np.maximum(1.0, np.abs(w))).max())
    _report(f"config3_b32_{mode}_forward_bf16_vs_fp32_oracle", out)
    h, r = out["hip_bf16"], out["reference_bf16_autocast"]
    for name in ("dwi_logits", "dce_logits", "fusion_logits"):
        assert h[name]["max_abs"] < 5e-2, (name, h[name])
    # everything else: no further from the fp32 oracle than the reference's own bf16 autocast (x1.5, + a floor)
    for name in names:
        assert h[name]["rel"] <= 1.5 * r[name]["rel"] + 1e-2, (name, h[name], r[name])
    for k, v in h["feature_stats_rel"].items():
        assert v <= 1.5 * r["feature_stats_rel"][k] + 1e-2, (k, v, r["feature_stats_rel"][k])
    if mode == "train":
        assert h["running_stat_sums_rel"] <= 1.5 * r["running_stat_sums_rel"] + 1e-3, (h, r)


def _fusion_grads(fm):
    return {n: p.grad.detach().float().cpu() for n, p in fm.named_parameters() if p.grad is not None}


def _rel_l2(got, truth):
    num = den = 0.0
    per = []
    for n, t in truth.items():
        d = got[n].reshape(t.shape) - t
        num += d.pow(2).sum().item()
        den += t.pow(2).sum().item()
        if t.norm() > 0:
            per.append((d.norm() / t.norm()).item())
    return (num / max(den, 1e-30)) ** 0.5, float(np.median(per))


@pytest.mark.timeout(900)
def test_config3_b32_captured_mode_a_step_vs_oracle():
    from dmf_dp import FusionTrainer
    from oracle import losses as OL

    P = _params()
    P["backbone_freeze_on_start"] = True  # the reference default at epoch 0 (mode A)
    (dwi, dce, fm), (dwi_r, dce_r, fr) = _models(P, (81, 82, 83))
    amp = [copy.deepcopy(m) for m in (dwi_r, dce_r, fr)]
    crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi, dce, fm, P, crit)
    lm.train()
    tr = FusionTrainer(lm, world=1, use_graph=True)
    bt = MG.volume_batch(B, S, 23)
    bd = tuple(t.to(DEV) for t in bt)
    recs = []
    O.PROBE["conv_fwd"] = recs
    try:
        tr.capture(bd)  # eager warm-ups (recorded) + the captured graphs; the training state is restored
    finally:
        O.PROBE["conv_fwd"] = None
    forms = _forms(recs)
    recs.clear()
    assert BENCH_FORMS <= set(forms), forms
    assert all(not p.requires_grad for m in (dwi, dce) for p in m.parameters())
    loss = tr.step(bd).item()  # one replay of the captured step
    assert tr.captures == 1 and tr.eager_steps == 0
    got = _fusion_grads(fm)

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cw = OL.class_weights_from_labels(torch.arange(1024) % 4)
    for m in (dwi_r, dce_r, *amp[:2]):
        for p in m.parameters():
            p.requires_grad = False
    for m in (dwi_r, dce_r, fr, *amp):
        m.train()
    ref = OL.fusion_shared_step(dwi_r, dce_r, fr, bt, P, cw, epoch=0)
    ref["total"].backward()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ref_amp = OL.fusion_shared_step(amp[0], amp[1], amp[2], bt, P, cw, epoch=0)
    ref_amp["total"].float().backward()
    truth = _fusion_grads(fr)
    assert set(got) == set(truth), sorted(set(got) ^ set(truth))
    e_hip, med_hip = _rel_l2(got, truth)
    e_amp, med_amp = _rel_l2(_fusion_grads(amp[2]), truth)
    lrel = abs(loss - ref["total"].item()) / max(1.0, abs(ref["total"].item()))
    terms = {k: {"hip": lm.last_metrics[k].item(), "oracle": ref[k].item()} for k in ("cls", "mask", "recon", "mimic")}
    _report("config3_b32_captured_mode_a_step_bf16_vs_fp32_oracle",
            {"forms": forms, "loss": {"hip": loss, "oracle": ref["total"].item(), "rel": lrel}, "terms": terms,
             "fusion_grads_rel_l2": {"hip_bf16": e_hip, "hip_bf16_median_tensor": med_hip,
                                     "reference_bf16_autocast": e_amp, "reference_median_tensor": med_amp}})
    assert lrel < 3e-2, lrel
    assert e_hip <= 1.25 * e_amp + 0.01, (e_hip, e_amp)
