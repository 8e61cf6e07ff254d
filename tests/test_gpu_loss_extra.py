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


def test_loss_combine_and_batch_accuracy_match_torch():
    """dmf_loss_combine (total + group sums in one launch, term gradients in one
    more) and dmf_batch_accuracy against plain torch arithmetic."""
    import dmf_ops as O

    torch.manual_seed(3)
    dev = "cuda"
    a = torch.rand((), device=dev, requires_grad=True)
    m = [torch.rand((), device=dev, requires_grad=True) for _ in range(3)]
    t = torch.rand(5, device=dev, requires_grad=True)
    mi = torch.rand((), device=dev, requires_grad=True)
    w = torch.tensor(0.8, device=dev)
    rc = (1 / 6, 1 / 6, 1 / 6, 1 / 6, 1 / 3)
    parts = [(a, (1.0,), False, -1, (0.0,))] + [(x, (0.2 / 3,), False, 0, (1 / 3,)) for x in m] + \
        [(t, tuple(0.1 * c for c in rc), True, 1, rc), (mi, (0.2,), True, 2, (1.0,))]
    total, groups = O.loss_combine(parts, 3, w)
    g = torch.tensor(1.7, device=dev)
    total.backward(g)
    grads = [a.grad.clone()] + [x.grad.clone() for x in m] + [t.grad.clone(), mi.grad.clone()]
    for x in [a, *m, t, mi]:
        x.grad = None
    recon = ((t[0] + t[1]) / 2 + (t[2] + t[3]) / 2 + t[4]) / 3
    ref = a + 0.2 * (m[0] + m[1] + m[2]) / 3 + 0.1 * recon * w + 0.2 * mi * w
    ref.backward(g)
    torch.testing.assert_close(total, ref.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(groups[0], ((m[0] + m[1] + m[2]) / 3).detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(groups[1], recon.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(groups[2], mi.detach(), rtol=1e-6, atol=1e-7)
    for got, x in zip(grads, [a, *m, t, mi]):
        torch.testing.assert_close(got, x.grad, rtol=1e-6, atol=1e-7)
    # accuracy: first maximum on ties, NaN counts as the maximum (torch.argmax)
    z = torch.randn(37, 4, device=dev)
    z[3] = torch.tensor([1.0, 1.0, 0.0, -1.0])
    z[5, 2] = float("nan")
    lab = torch.randint(0, 4, (37,), device=dev)
    lab[3], lab[5] = 0, 2
    ref_acc = (torch.argmax(z, dim=1) == lab).float().mean()
    torch.testing.assert_close(O.batch_accuracy(z, lab), ref_acc)
