"""GPU: the packed-fp32 GELU of the BatchNorm apply (gelu_f2, v_pk_fma_f32 on value pairs; k_bn_apply
with act GELU -- the necks' conv -> BN -> GELU, model_module.py:440-447) against the scalar gelu_f of
k_affine_act8 on the same bf16 inputs, and both against torch's exact erf GELU in float64."""
import pytest
import torch
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(fn, x, m, c):
    y = torch.empty_like(x)
    if fn == "dmf_bn_apply":
        N.call("dmf_bn_apply", N.BF16, x.data_ptr(), c, None, None, None, 0, None, None, O.ACT["gelu"], 0.0, None, 0,
               y.data_ptr(), c, m, c, N.stream_ptr())
    else:
        N.call("dmf_affine_act", N.BF16, x.data_ptr(), c, None, None, 0, None, O.ACT["gelu"], 0.0, None, 0,
               y.data_ptr(), c, m, c, N.stream_ptr())
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("m,c", [(32768, 256), (1000, 72)])
def test_packed_gelu_matches_scalar(m, c):
    torch.manual_seed(0)
    x = (torch.randn(m, c, device=DEV) * 3).to(torch.bfloat16)
    x[0, :8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 8.0, -8.0, 30.0, -30.0], device=DEV).bfloat16()
    yp = _run("dmf_bn_apply", x, m, c)
    ys = _run("dmf_affine_act", x, m, c)
    ref = F.gelu(x.double())
    # same formula, packed vs scalar instruction forms: equal up to one bf16 rounding step of the fp32 result
    d = (yp.float() - ys.float()).abs()
    ulp = ys.float().abs().clamp_min(1e-30) * 2 ** -7
    assert (d <= ulp).all(), d.max().item()
    assert (yp != ys).float().mean().item() < 1e-3
    for y in (yp, ys):
        err = (y.double() - ref).abs()
        assert (err <= ref.abs() * 2 ** -8 + 1e-6).all(), err.max().item()
