"""The 7x7 / stride-2 stem kernel (csrc/conv_stem.hip) against a float64
torch reference of the same bf16 operands, in eval (plain store) and
training (BN batch statistics from the conv epilogue, then the BN apply +
ReLU) form, and against the general implicit GEMM it replaces
(dmf_conv_tune key 10 off). Shapes: the DWI stem (14 -> 16 padded channels)
and the DCE stem (6 -> 8) at S=256, config 2's 5-phase stem at S=128 (64
output columns: one column block), a config-5-size S=384 input (three
column blocks, a 7-KiB ring plane), and a batch whose workgroups take fewer
output rows each (B=1)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (batch, real input channels, input size)
CASES = [(4, 14, 256), (4, 6, 256), (3, 5, 128), (2, 14, 384), (1, 14, 256)]


def _q(t):
    return t.bfloat16().float()


def _inputs(b, ci, s, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(ci, 64, 7, stride=2, padding=3, bias=False)
    x = _q(torch.randn(b, ci, s, s))
    wq = _q(conv.weight.detach())
    cp = O.channel_pad(ci, torch.bfloat16)
    xp = torch.cat([x, torch.zeros(b, cp - ci, s, s)], 1)
    xd = xp.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cd = copy.deepcopy(conv).to(DEV)
    with torch.no_grad():
        cd.weight.copy_(wq)
    raw = F.conv2d(x.double(), wq.double(), None, 2, 3).float()
    return cd, xd, raw


def _stem(on):
    N.call("dmf_conv_tune", 10, 1 if on else 0)


@pytest.fixture(autouse=True)
def _restore():
    yield
    _stem(True)


@pytest.mark.parametrize("case", CASES)
def test_stem_forward_matches_reference(case):
    b, ci, s = case
    cd, xd, raw = _inputs(b, ci, s, 21)
    outs = []
    for on in (True, False):
        _stem(on)
        with torch.no_grad():
            y = O.conv2d(xd, cd, (O.WeightCache(), O.WeightCache()))
        torch.cuda.synchronize()
        outs.append(y.float().cpu())
    scale = raw.abs().max().item()
    err = (outs[0] - raw).abs().max().item()
    assert err <= 1e-2 * scale, (err, scale)
    # the general implicit GEMM it replaces: same bf16 rounding of fp32 sums over a different K order
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-2 * scale


@pytest.mark.parametrize("case", CASES)
def test_stem_training_bn_stats(case):
    b, ci, s = case
    cd, xd, raw = _inputs(b, ci, s, 22)
    bn = nn.BatchNorm2d(64)
    bd = nn.BatchNorm2d(64).to(DEV)
    ref = F.relu(bn(raw))
    with torch.no_grad():
        y = O.conv_bn_act(xd, cd, (O.WeightCache(), O.WeightCache()), bd, "relu")
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=1e-2, atol=1e-3 * raw.abs().max().item())
    assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=1e-2, atol=1e-3)


def test_stem_is_selected_for_the_hot_shape():
    """The stem path is the one a DWI stem launch takes (statistics slab rows = its workgroups)."""
    n = N.load().dmf_conv2d_fwd_stat_tiles(N.dtype_code(torch.bfloat16), 32, 256, 256, 16, 16, 0, 0, 64, 7, 7, 2, 3,
                                           128, 128, 0)
    assert n == 32 * 128 // 16  # 16 output rows of 128 pixels per workgroup
