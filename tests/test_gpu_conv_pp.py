"""The ping-pong 256x256 forward conv (csrc/conv_pp.hip) and the persistent
form at 128x128 with two workgroups per CU (k_conv_fwd_ps<..., 128, 128, 2>)
against a float64 torch reference of the same bf16 operands, and bit for bit
against the 256x256 persistent form they share operand order, K order and
register epilogue with (k_conv_fwd_ps). Shapes cover a plain 1x1, padded / dilated 3x3 with an M
tail, the neck's two-source 3x3 (channel concat in the K loop), the bias +
activation epilogue, and K = 64 (a single K-tile: prologue-only staging)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (N, Cin, H, W, Cout, k, pad, dil, Cin2, act)
    (34, 512, 32, 32, 1024, 1, 0, 1, 0, None),
    (65, 256, 32, 32, 256, 3, 2, 2, 0, None),
    (65, 64, 31, 31, 512, 3, 4, 4, 0, None),
    (36, 64, 31, 31, 512, 3, 1, 1, 64, None),
    (64, 64, 32, 32, 256, 1, 0, 1, 0, None),
    (66, 128, 32, 32, 256, 1, 0, 1, 0, "gelu"),
]


def _q(t):
    return t.bfloat16().float()


# (dmf_conv_tune key, value forcing the form on every legal shape, library default)
FORMS = {"pp": (7, 2, 1)}  # (the 128x128 two-workgroup persistent form was removed in round 4)


@pytest.fixture(params=sorted(FORMS))
def pp_mode(request):
    key, on, default = FORMS[request.param]
    N.call("dmf_conv_tune", key, on)
    yield
    N.call("dmf_conv_tune", key, default)


@pytest.mark.parametrize("case", CASES)
def test_pp_forward_matches_reference_and_bn_stats(case, pp_mode):
    n, ci, h, w, co, k, p, d, ci2, act = case
    torch.manual_seed(11)
    conv = nn.Conv2d(ci + ci2, co, k, padding=p, dilation=d, bias=act is not None)
    a = _q(torch.randn(n, ci, h, w))
    b = _q(torch.randn(n, ci2, h, w)) if ci2 else None
    wq = _q(conv.weight.detach())
    xin = torch.cat([a, b], 1) if ci2 else a
    cd = copy.deepcopy(conv).to(DEV)
    with torch.no_grad():
        cd.weight.copy_(wq)
    xa = a.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xb = b.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last) if ci2 else None
    caches = (O.WeightCache(), O.WeightCache())
    with torch.no_grad():
        if act is None:
            bn = nn.BatchNorm2d(co)
            bd = nn.BatchNorm2d(co).to(DEV)
            raw = F.conv2d(xin.double(), wq.double(), None, 1, p, d).float()
            ref = F.relu(bn(raw))
            y = O.conv_bn_act(xa, cd, caches, bd, "relu", x2=xb)
        else:
            raw = F.conv2d(xin.double(), wq.double(), conv.bias.double(), 1, p, d).float()
            ref = F.gelu(raw)
            y = O.conv2d(xa, cd, caches, act="gelu")
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-2 * scale, (err, scale)
    if act is None:
        assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=1e-2, atol=1e-3 * raw.abs().max().item())
        assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=2e-2, atol=1e-3)


@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("case", [c for c in CASES if c[5] == 1 and c[8] == 0])
def test_pp_bitwise_equals_persistent_form(case, form):
    """k_conv_fwd_pp / the 128x128 two-workgroup form and the 256x256
    k_conv_fwd_ps accumulate the same MFMAs in the same K order into the same
    registers: identical raw outputs."""
    key, on, default = FORMS[form]
    n, ci, h, w, co, k, p, d, _, act = case
    torch.manual_seed(12)
    conv = nn.Conv2d(ci, co, k, bias=act is not None).to(DEV)
    x = torch.randn(n, ci, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = O.ConvGeom(conv)
    outs = []
    for mode in ((7, 0), (key, on)):
        N.call("dmf_conv_tune", *mode)
        try:
            with torch.no_grad():
                y, _ = O._conv_forward_raw(x, conv.weight, conv.bias, g, (O.WeightCache(), O.WeightCache()), False,
                                           act or "none")
            torch.cuda.synchronize()
            outs.append(y.clone())
        finally:
            N.call("dmf_conv_tune", 7, 1)
            N.call("dmf_conv_tune", key, default)
    assert torch.equal(outs[0], outs[1])
