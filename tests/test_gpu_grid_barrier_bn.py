"""GPU: the grid-barrier BatchNorm apply (dmf_conv2d_fwd_bn_act) of a forward-only
conv -> BN(batch statistics) -> act, the frozen encoders' non-residual apply
passes (timm Bottleneck conv1 / conv2 + bn + act, foundation_model.py Bottleneck;
the neck conv -> BN -> GELU, model_module.py BackboneAdapter): outputs against
an fp32 conv (GPU, TF32 off) with the BatchNorm finished in float64, against the
conv + dmf_bn_apply form it replaces (knob grid_barrier_bn off), the running
statistics, repeated launches and hipGraph replays of the self-resetting barrier
words, and that the serial encoder forward takes the path. The form is a measured
variant, off by default (dmf_ops.GRID_BARRIER_BN): these tests switch it on."""
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


# (N, Cin, Cin2, H, W, Cout, k, pad, dil, bias, act, form): 256 output tiles = one per CU
CASES = [
    (32, 2048, 0, 32, 32, 512, 1, 0, 1, False, "relu", "pp"),   # layer4 conv1
    (32, 512, 0, 32, 32, 512, 3, 4, 4, False, "relu", "pp"),    # layer4 conv2 (dilated)
    (32, 1024, 0, 32, 32, 256, 1, 0, 1, False, "relu", "wide"),  # layer3 conv1
    (32, 256, 0, 32, 32, 256, 3, 2, 2, False, "relu", "wide"),   # layer3 conv2 (dilated)
    (32, 256, 0, 32, 32, 256, 3, 1, 1, True, "gelu", "wide"),    # neck conv2 (bias, GELU)
    (32, 512, 256, 32, 32, 256, 3, 1, 1, True, "gelu", "wide"),  # a two-source neck conv (no concat)
]


def _case(case, seed=3):
    n, ci, ci2, h, w, co, k, pad, dil, bias, act, _ = case
    torch.manual_seed(seed)
    conv = nn.Conv2d(ci + ci2, co, k, padding=pad, dilation=dil, bias=bias)
    conv.weight.data = conv.weight.data.bfloat16().float()
    if bias:
        conv.bias.data.uniform_(-0.2, 0.2)
    bn = nn.BatchNorm2d(co)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.5, 0.5)
    bn.running_mean.uniform_(-0.2, 0.2)
    bn.running_var.uniform_(0.5, 2.0)
    x = torch.randn(n, ci + ci2, h, w).bfloat16().float()
    return x, conv, bn


def _ref(x, conv, bn, act):
    """fp32 conv on the GPU (TF32 off) -> BatchNorm in float64 -> act."""
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.no_grad():
            z = F.conv2d(x.to(DEV), conv.weight.to(DEV), conv.bias.to(DEV) if conv.bias is not None else None,
                         padding=conv.padding, dilation=conv.dilation).double()
    finally:
        torch.backends.cudnn.allow_tf32 = prev
    mean = z.mean((0, 2, 3))
    var = z.var((0, 2, 3), unbiased=False)
    m = z.numel() // z.shape[1]
    inv = (var + bn.eps).rsqrt()
    y = (z - mean[None, :, None, None]) * (inv * bn.weight.to(DEV).double())[None, :, None, None] \
        + bn.bias.to(DEV).double()[None, :, None, None]
    y = F.relu(y) if act == "relu" else F.gelu(y)
    return y, mean.cpu(), (var * m / (m - 1)).cpu()


def _run(x, conv, bn, case, gbar, reps=1):
    ci2, act = case[2], case[10]
    cd, bd = copy.deepcopy(conv).to(DEV), copy.deepcopy(bn).to(DEV).train()
    for p in list(cd.parameters()) + list(bd.parameters()):
        p.requires_grad_(False)
    calls = []
    orig = O._conv_bn_gbar

    def counted(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    prev = O.GRID_BARRIER_BN
    O.set_knobs(grid_barrier_bn=gbar)
    O._conv_bn_gbar = counted
    try:
        with torch.no_grad():
            xd = _to_dev(x)
            x1, x2 = (xd[:, :xd.shape[1] - ci2], xd[:, xd.shape[1] - ci2:]) if ci2 else (xd, None)
            if ci2:
                x1, x2 = O.as_nhwc(x1.contiguous(memory_format=torch.channels_last)), \
                    O.as_nhwc(x2.contiguous(memory_format=torch.channels_last))
            caches = (O.WeightCache(), O.WeightCache())
            for _ in range(reps):
                y = O.conv_bn_act(x1, cd, caches, bd, act, x2=x2)
            form = N.FORMS.get(N.load().dmf_conv_last_form())
        torch.cuda.synchronize()
    finally:
        O._conv_bn_gbar = orig
        O.set_knobs(grid_barrier_bn=prev)
    return y.float(), bd, len(calls), form


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[1]}+{c[2]}-{c[5]}-k{c[6]}d{c[8]}-{c[10]}-{c[11]}")
def test_grid_barrier_bn_apply(case):
    x, conv, bn = _case(case)
    ref, mean, uvar = _ref(x, conv, bn, case[10])
    y2, bn2, n2, form2 = _run(x, conv, bn, case, True)
    y1, bn1, n1, _ = _run(x, conv, bn, case, False)
    assert (n2, n1) == (1, 0) and form2 == case[11], (n2, n1, form2)
    scale = ref.abs().max().item()
    e2 = (y2.double() - ref).abs().max().item() / scale
    e1 = (y1.double() - ref).abs().max().item() / scale
    # bf16 output rounding bounds both; the barrier form applies the BN to the fp32 accumulator, the
    # two-kernel form to the bf16-rounded raw output
    assert e2 <= 8e-3, (e2, e1)
    assert e2 <= e1 * 1.25 + 1e-4, (e2, e1)
    mom = bn.momentum
    rm = (1 - mom) * bn.running_mean.double() + mom * mean
    rv = (1 - mom) * bn.running_var.double() + mom * uvar
    torch.testing.assert_close(bn2.running_mean.cpu().double(), rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn2.running_var.cpu().double(), rv, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn2.running_mean.cpu(), bn1.running_mean.cpu(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn2.running_var.cpu(), bn1.running_var.cpu(), rtol=1e-5, atol=1e-6)
    assert int(bn2.num_batches_tracked) == 1


def test_grid_barrier_repeated_and_graph_replay():
    """The barrier words reset themselves: five eager launches in a row, then a captured hipGraph
    replayed three times, all agree with the first launch (statistics are float64 sums of fp32
    tile partials, so only the last bits may differ)."""
    case = CASES[3]
    x, conv, bn = _case(case)
    y_once, _, _, _ = _run(x, conv, bn, case, True)
    y5, bn5, n5, _ = _run(x, conv, bn, case, True, reps=5)
    assert n5 == 5 and int(bn5.num_batches_tracked) == 5
    torch.testing.assert_close(y5, y_once, rtol=1e-2, atol=1e-2)
    cd, bd = copy.deepcopy(conv).to(DEV).requires_grad_(False), copy.deepcopy(bn).to(DEV).train()
    bd.requires_grad_(False)
    xd = _to_dev(x)
    caches = (O.WeightCache(), O.WeightCache())
    owner = nn.Sequential(cd, bd)

    def fwd():
        # the forward's statistics arena (zeroed at each scope entry after the first: captured)
        with O.bn_scope(owner, DEV):
            return O.conv_bn_act(xd, cd, caches, bd, "relu")

    prev = O.GRID_BARRIER_BN
    O.set_knobs(grid_barrier_bn=True)
    with torch.no_grad():
        fwd()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            yg = fwd()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    O.set_knobs(grid_barrier_bn=prev)
    assert int(bd.num_batches_tracked) == 4
    torch.testing.assert_close(yg.float(), y_once, rtol=1e-2, atol=1e-2)


def test_grid_barrier_not_in_concurrent_region_or_with_grad():
    case = CASES[3]
    x, conv, bn = _case(case)
    cd, bd = conv.to(DEV), bn.to(DEV)
    xd = _to_dev(x)
    prev = O.GRID_BARRIER_BN
    O.set_knobs(grid_barrier_bn=True)
    try:
        _check_gbar_ok(xd, cd, bd)
    finally:
        O.set_knobs(grid_barrier_bn=prev)
    with torch.no_grad():
        assert O._gbar_ok(xd, cd, bd, "relu", 0.0, None, None, None, None) is prev  # the default


def _check_gbar_ok(xd, cd, bd):
    assert O._gbar_ok(xd, cd, bd, "relu", 0.0, None, None, None, None) is False  # parameters need grad
    with torch.no_grad():
        assert O._gbar_ok(xd, cd, bd, "relu", 0.0, None, None, None, None) is True
        O.CONCURRENT[0] += 1
        try:
            assert O._gbar_ok(xd, cd, bd, "relu", 0.0, None, None, None, None) is False
        finally:
            O.CONCURRENT[0] -= 1
        assert O._gbar_ok(xd, cd, bd, "relu", 0.1, None, None, None, None) is False  # dropout
        bd.eval()
        assert O._gbar_ok(xd, cd, bd, "relu", 0.0, None, None, None, None) is False  # running statistics
        bd.train()
        assert O._gbar_ok(xd[:8], cd, bd, "relu", 0.0, None, None, None, None) is False  # < one tile per CU


def test_serial_encoder_forward_takes_grid_barrier():
    """The production plan with the encoders on one stream (knob parallel_encoders off): the frozen
    ResNet-50's layer3 / layer4 conv1 + conv2 BatchNorms run in the barrier form."""
    import foundation_model as FM

    torch.manual_seed(0)
    enc = FM.ResNet50OS8().to(DEV).train()
    for p in enc.parameters():
        p.requires_grad_(False)
    calls = []
    orig = O._conv_bn_gbar

    def counted(*a, **k):
        calls.append((a[1].out_channels, a[1].kernel_size[0]))
        return orig(*a, **k)

    prev = O.GRID_BARRIER_BN
    O.set_knobs(grid_barrier_bn=True)
    O._conv_bn_gbar = counted
    try:
        with torch.no_grad():
            feats = enc(torch.randn(32, 3, 256, 256, device=DEV))
        torch.cuda.synchronize()
    finally:
        O._conv_bn_gbar = orig
        O.set_knobs(grid_barrier_bn=prev)
    assert all(torch.isfinite(f.float()).all() for f in feats)
    # layer3: 6 blocks x (conv1 1x1 -> 256, conv2 3x3 -> 256); layer4: 3 x (conv1 -> 512, conv2 -> 512)
    assert sorted(set(calls)) == [(256, 1), (256, 3), (512, 1), (512, 3)], calls
    assert len(calls) == 18, calls
