"""Criteria off the default path (ADVICE r01 lows) and the conv channel
check: WeightedFocalLoss with soft / smoothed targets follows loss.py:96-128
(cross entropy on the soft targets, alpha at argmax); a reduction that is
neither 'mean' nor 'sum' returns per-row losses (loss.py:151-155, the 'fl'
selector passes gamma there, quirk Q8); a conv input whose channel count is
neither the weight's nor its zero-padded staging width is refused."""
import pytest
import torch
import torch.nn.functional as F

import dmf_ops as O
from loss import SoftFocalLoss, WeightedFocalLoss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_wfl(x, t, alpha, gamma, reduction):
    ce = F.cross_entropy(x, t, reduction="none")
    pt = torch.exp(-ce)
    if alpha is None:
        fl = (1 - pt) ** gamma * ce
    elif isinstance(alpha, (int, float)):
        fl = alpha * (1 - pt) ** gamma * ce
    else:
        idx = t.argmax(1) if t.ndim > 1 else t
        fl = alpha.gather(0, idx.long()) * (1 - pt) ** gamma * ce
    return fl.mean() if reduction == "mean" else fl.sum() if reduction == "sum" else fl


@pytest.mark.parametrize("alpha", [None, 0.5, "vec"])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_weighted_focal_soft_targets(alpha, reduction):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(16, 4, generator=g) * 2
    lab = torch.randint(0, 4, (16,), generator=g)
    t = F.one_hot(lab, 4).float() * 0.9 + 0.025  # label smoothing 0.1
    a = torch.tensor([0.1, 0.2, 0.3, 0.4]) if alpha == "vec" else alpha
    got = WeightedFocalLoss(a.to(DEV) if alpha == "vec" else a, 2, reduction)(x.to(DEV), t.to(DEV))
    want = _ref_wfl(x, t, a, 2, reduction)
    assert torch.allclose(got.cpu(), want, rtol=1e-5, atol=1e-6)
    # hard labels keep the fused kernel path and agree too
    got_h = WeightedFocalLoss(a.to(DEV) if alpha == "vec" else a, 2, reduction)(x.to(DEV), lab.to(DEV))
    assert torch.allclose(got_h.cpu(), _ref_wfl(x, lab, a, 2, reduction), rtol=1e-5, atol=1e-6)


def test_non_string_reduction_returns_rows():
    x = torch.randn(8, 4, device=DEV)
    lab = torch.randint(0, 4, (8,), device=DEV)
    out = SoftFocalLoss(2.0, 2)(x, lab)  # the 'fl' selector's (alpha, gamma) mix-up: reduction = 2
    assert out.shape == (8,)


def test_conv_refuses_wrong_channel_count():
    conv = torch.nn.Conv2d(6, 16, 3, padding=1).to(DEV)
    ok = O.as_nhwc(torch.randn(2, 8, 12, 12, device=DEV))  # 6 channels staged (padded) to 8
    O.conv2d(ok, conv, (O.WeightCache(), O.WeightCache()))
    bad = O.as_nhwc(torch.randn(2, 12, 12, 12, device=DEV))
    with pytest.raises(RuntimeError):
        O.conv2d(bad, conv, (O.WeightCache(), O.WeightCache()))
