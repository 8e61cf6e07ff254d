"""GPU: every weight gradient of one PRODUCTION mode-B step against float64
(reference selector_helpers.py:541-584 -- after the
unfreeze, mode B is the steady state).

The model-level mode-B check (test_gpu_golden_full) can only bound the
backbone gradients by the reference AMP's own error, which is ~1.4 relative:
ill-conditioned, so it cannot see a wrong weight gradient. This test pins the
kernels instead, inside the real step: configuration 3 at B=32, S=256,
default widths, bf16, everything trainable. One eager step records every MFMA
weight-gradient launch (dmf_ops.PROBE["conv_wgrad"]: dmf_conv2d_wgrad with its
production split plan -- wgrad_fill, the 256x256 / 128x256 / 128x128 tiles --
and the split reduce) together with its bf16 operands x (x2 for the dual-source
neck conv) and dY. Each launch is re-run into a fresh output and compared with
torch.nn.grad.conv2d_weight's contraction evaluated in float64 on the same
bf16 operands (unfold + GEMM, on the GPU): relative L2 <= 1e-3 per launch
(fp32 accumulation over up to 131,072 pixels). Negative control: the same
check on a zeroed output must fail."""
import copy

import pytest
import torch
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O
import make_golden as MG
import model_module as MM
import parameters as PR
import train_fusion as TF
from selector_helpers import get_classification_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, S = 32, 256
BAR = 1e-3


def _truth(x, x2, dy, co, kh, kw, stride, pad, dil):
    """float64 dW [co][C][kh][kw] = sum over pixels of dY (x) unfold(x)."""
    xs = torch.cat([x, x2], 1) if x2 is not None else x
    n, c = xs.shape[:2]
    acc = torch.zeros(co, c * kh * kw, dtype=torch.float64, device=DEV)
    for i in range(0, n, 8):  # bounded memory: 8 volumes at a time
        cols = F.unfold(xs[i:i + 8].double(), (kh, kw), dilation=dil, padding=pad, stride=stride)  # [b][c*kh*kw][L]
        g = dy[i:i + 8].double().reshape(cols.shape[0], co, -1)  # [b][co][L]
        acc += torch.einsum("bol,bkl->ok", g, cols)
    return acc.view(co, c, kh, kw)


def _rel(got, want):
    return ((got.double() - want).norm() / want.norm().clamp_min(1e-300)).item()


@pytest.mark.timeout(900)
def test_mode_b_b32_every_weight_gradient_launch_vs_float64():
    P = copy.deepcopy(PR.default_parameters())
    P["backbone_freeze_on_start"] = False  # mode B: everything trainable
    dwi, _ = MG.seeded_encoder(P, "dwi", 14, 41)
    dce, _ = MG.seeded_encoder(P, "dce", 6, 42)
    fm, _ = MG.seeded_fusion(P, 43)
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi.to(DEV), dce.to(DEV), fm.to(DEV), P, crit)
    lm.train()
    from dmf_dp import FusionTrainer

    tr = FusionTrainer(lm, world=1, use_graph=False)
    bd = tuple(t.to(DEV) for t in MG.volume_batch(B, S, 31))
    tr.eager_step(bd)  # weight caches, optimizer tables
    recs = []
    O.PROBE["conv_wgrad"] = recs
    try:
        tr.eager_step(bd)
        torch.cuda.synchronize()
    finally:
        O.PROBE["conv_wgrad"] = None
    assert len(recs) > 100, len(recs)  # both ResNet-50 OS8 encoders + heads
    splits_seen, worst, checked = set(), (0.0, None), 0
    for r in recs:
        (fw, wargs), (fr_, rargs) = r["calls"]
        assert fw == "dmf_conv2d_wgrad" and fr_ == "dmf_conv2d_wgrad_reduce"
        x, x2, dy = r["keep"][0], r["keep"][1], r["keep"][2]
        (_, _, n, h, w, cx, ldx, _, cx2, ldx2, _, ho, wo, co, lddy, kh, kw, stride, pad, dil, splits, _) = wargs
        ws_ptr, _, co_r, ci, ct, kh_r, kw_r, _, _ = rargs
        assert (co_r, kh_r, kw_r) == (co, kh, kw)
        splits_seen.add(splits)
        out = torch.empty((co, ci, kh, kw), dtype=torch.float32, device=DEV)
        N.call(fw, *wargs, N.stream_ptr())
        N.call(fr_, ws_ptr, splits, co, ci, ct, kh, kw, out.data_ptr(), 0, N.stream_ptr())
        want = _truth(x, x2, dy, co, kh, kw, stride, pad, dil)[:, :ci]
        e = _rel(out, want)
        assert e <= BAR, (r["shape"], splits, e)
        assert _rel(torch.zeros_like(out), want) > BAR  # negative control: a zeroed dW fails
        if e > worst[0]:
            worst = (e, r["shape"])
        checked += 1
    print(f"{checked} weight-gradient launches of one B=32 mode-B step vs float64: worst rel L2 {worst[0]:.2e} "
          f"at {worst[1]}; split counts {sorted(splits_seen)}")
    assert max(splits_seen) > 1  # the production split plan (pixel splits + reduce) ran
