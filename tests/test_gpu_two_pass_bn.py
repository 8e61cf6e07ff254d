"""GPU: the two-pass BatchNorm fusion of a forward-only Bottleneck conv3
(dmf_conv2d_fwd_stats -> dmf_bn_finalize_acc -> dmf_conv2d_fwd_affine, or with the finalize folded
into the second pass: dmf_conv2d_fwd_affine_acc) against
a float64 CPU restatement of conv -> BN(batch statistics) -> + shortcut -> ReLU
(foundation_model.py Bottleneck.forward, the reference's timm Bottleneck), and
against the conv + dmf_bn_apply form it replaces (knob two_pass_bn off):
outputs, running statistics, eval mode, identity and projection shortcuts, and
that the frozen encoder's forward takes the path."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _to_dev(x):
    return x.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _bn64(z, bn, training):
    """BatchNorm2d in float64: returns (out, batch mean, unbiased batch var)."""
    if training:
        mean = z.mean((0, 2, 3))
        var = z.var((0, 2, 3), unbiased=False)
        m = z.numel() // z.shape[1]
        uvar = var * m / (m - 1)
    else:
        mean, var = bn.running_mean.double(), bn.running_var.double()
        uvar = var
    inv = (var + bn.eps).rsqrt()
    out = (z - mean[None, :, None, None]) * (inv * bn.weight.double())[None, :, None, None] \
        + bn.bias.double()[None, :, None, None]
    return out, mean, uvar


def _case(shape, proj, training, seed=7):
    n, ci, h, w, co, cr, stride = shape
    torch.manual_seed(seed)
    conv = nn.Conv2d(ci, co, 1, bias=False)
    bn = nn.BatchNorm2d(co)
    x = torch.randn(n, ci, h // stride, w // stride).bfloat16().float().relu()
    mods = [conv, bn]
    if proj:
        conv_r = nn.Conv2d(cr, co, 1, stride=stride, bias=False)
        bn_r = nn.BatchNorm2d(co)
        xr = torch.randn(n, cr, h, w).bfloat16().float()
        mods += [conv_r, bn_r]
    else:
        xr = torch.randn(n, co, h // stride, w // stride).bfloat16().float()
    for m in mods:
        if isinstance(m, nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.5, 0.5)
            m.running_mean.uniform_(-0.2, 0.2)
            m.running_var.uniform_(0.5, 2.0)
            m.train(training)
        else:
            m.weight.data = m.weight.data.bfloat16().float()
    return x, xr, mods


def _ref(x, xr, mods, training):
    conv, bn = mods[0], mods[1]
    with torch.no_grad():
        z, mean, uvar = _bn64(F.conv2d(x.double(), conv.weight.double()), bn, training)
        stats = [(mean, uvar)]
        if len(mods) > 2:
            r, mr, vr = _bn64(F.conv2d(xr.double(), mods[2].weight.double(), stride=mods[2].stride), mods[3],
                              training)
            stats.append((mr, vr))
        else:
            r = xr.double()
    return (z + r).relu(), stats


def _run(x, xr, mods, two_pass, fold=True, finalizes=None):
    dm = [copy.deepcopy(m).to(DEV) for m in mods]
    calls = []
    orig, orig_fin = O._conv_bn_two_pass, O._finalize_acc

    def counted(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    def counted_fin(*a, **k):
        if finalizes is not None:
            finalizes.append(1)
        return orig_fin(*a, **k)

    O.set_knobs(two_pass_bn=two_pass, two_pass_fold=fold)
    O._conv_bn_two_pass = counted
    O._finalize_acc = counted_fin
    try:
        with torch.no_grad():
            xd, xrd = _to_dev(x), _to_dev(xr)
            c = (O.WeightCache(), O.WeightCache())
            if len(dm) > 2:
                y = O.conv_bn_act(xd, dm[0], c, dm[1], "relu", skip=(xrd, dm[2], (O.WeightCache(), O.WeightCache()),
                                                                     dm[3]))
            else:
                y = O.conv_bn_act(xd, dm[0], c, dm[1], "relu", res=xrd)
        torch.cuda.synchronize()
    finally:
        O._conv_bn_two_pass, O._finalize_acc = orig, orig_fin
        O.set_knobs(two_pass_bn=True, two_pass_fold=True)
    return y.float().cpu(), dm, len(calls)


# (N, Cin, H, W, Cout, Cin of the projection, its stride): M = N*H*W/stride^2 a multiple of 256 and
# M/256 * Cout/256 >= 256 tiles (the persistent 256x256 plan)
SHAPES = [(16, 256, 32, 32, 1024, 0, 1), (32, 128, 64, 64, 512, 256, 2), (32, 64, 64, 64, 256, 64, 1)]


# fold: the BatchNorm finalize between the passes folded into pass 2 (dmf_conv2d_fwd_affine_acc) or the
# separate dmf_bn_finalize_acc launch + dmf_conv2d_fwd_affine
@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("shape", SHAPES)
def test_two_pass_conv3(shape, training, fold):
    proj = shape[5] > 0
    x, xr, mods = _case(shape, proj, training)
    dev_ok = N.load().dmf_conv2d_fwd_affine_ok(N.BF16, shape[0], shape[2] // shape[6], shape[3] // shape[6],
                                               shape[1], shape[4], 1)
    assert dev_ok, "test shape must take the persistent plan"
    ref, stats = _ref(x, xr, mods, training)
    fins = []
    y2, dm2, n2 = _run(x, xr, mods, True, fold=fold, finalizes=fins)
    y1, dm1, n1 = _run(x, xr, mods, False)
    assert (n2, n1) == (1, 0)
    # the main BatchNorm's finalize launch only without the fold; a projection shortcut's BN keeps its own
    assert len(fins) == (int(not fold) + int(proj) if training else 0), fins
    scale = ref.abs().max().item()
    e2 = (y2.double() - ref).abs().max().item() / scale
    e1 = (y1.double() - ref).abs().max().item() / scale
    # bf16 output rounding (2^-9 relative) bounds both; the two-pass form applies the BN to the fp32
    # accumulator instead of the bf16-rounded raw output, so it is no worse
    assert e2 <= 8e-3, (e2, e1)
    assert e2 <= e1 * 1.25 + 1e-4, (e2, e1)
    bns = [(dm2[1], dm1[1], mods[1])] + ([(dm2[3], dm1[3], mods[3])] if proj else [])
    for (b2, b1, b0), (mean, uvar) in zip(bns, stats):
        if training:
            mom = b0.momentum
            rm = (1 - mom) * b0.running_mean.double() + mom * mean
            rv = (1 - mom) * b0.running_var.double() + mom * uvar
            assert int(b2.num_batches_tracked) == 1
        else:
            rm, rv = b0.running_mean.double(), b0.running_var.double()
        for got, want in ((b2.running_mean, rm), (b2.running_var, rv)):
            torch.testing.assert_close(got.cpu().double(), want, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(b2.running_mean.cpu(), b1.running_mean.cpu(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(b2.running_var.cpu(), b1.running_var.cpu(), rtol=1e-4, atol=1e-5)


def test_two_pass_needs_no_grad_and_relu():
    """Autograd, a non-ReLU activation or dropout keep the conv + apply form."""
    x, xr, mods = _case(SHAPES[0], False, True)
    conv, bn = (m.to(DEV) for m in mods[:2])
    xd, xrd = _to_dev(x), _to_dev(xr)
    assert O._two_pass_ok(xd, conv, bn, "relu", 0.0, xrd, None, None, None, 1) is False  # params need grad
    with torch.no_grad():
        assert O._two_pass_ok(xd, conv, bn, "relu", 0.0, xrd, None, None, None, 1) is True
        assert O._two_pass_ok(xd, conv, bn, "gelu", 0.0, xrd, None, None, None, 1) is False
        assert O._two_pass_ok(xd, conv, bn, "relu", 0.1, xrd, None, None, None, 1) is False
        assert O._two_pass_ok(xd, conv, bn, "relu", 0.0, None, None, None, None, 1) is False
        assert O._two_pass_ok(xd[:3], conv, bn, "relu", 0.0, xrd[:3], None, None, None, 1) is False  # < 256 tiles


def test_frozen_encoder_forward_takes_two_pass():
    """The production plan: the frozen ResNet-50 encoder's forward (mode A,
    train-mode BN, no autograd) runs every eligible conv3 in two passes."""
    import foundation_model as FM

    torch.manual_seed(0)
    enc = FM.ResNet50OS8().to(DEV).train()
    for p in enc.parameters():
        p.requires_grad_(False)
    calls = []
    orig = O._conv_bn_two_pass

    def counted(*a, **k):
        calls.append(a[1].out_channels)
        return orig(*a, **k)

    O._conv_bn_two_pass = counted
    try:
        with torch.no_grad():
            feats = enc(torch.randn(32, 3, 256, 256, device=DEV))
        torch.cuda.synchronize()
    finally:
        O._conv_bn_two_pass = orig
    assert all(torch.isfinite(f.float()).all() for f in feats)
    # layer1-3 conv3s (3 + 4 + 6 blocks; K <= TWO_PASS_MAX_K) at B=32, 256x256 input, output stride 8
    assert len(calls) == 13 and max(calls) == 1024, calls
