"""GPU: k_bn_apply with 2 / 4 rows of loads in flight per thread (dmf_bn_apply_tune) against the
one-row form -- bitwise equal for every residual kind, activation and dropout, on full and ragged
row ranges (the BatchNorm -> act [-> + shortcut] pass of model_module.py / foundation_model.py)."""
import pytest
import torch

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _apply(x, ss, res, ssr, act, p, rng, m, c):
    y = torch.empty_like(x)
    N.call("dmf_bn_apply", N.BF16, x.data_ptr(), c, None, ss.data_ptr(), O._p(res), c, None,
           O._p(ssr), O.ACT[act], p, O._p(rng), 5, y.data_ptr(), c, m, c, N.stream_ptr())
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("m,c", [(32768, 256), (1000, 72), (131072, 64), (4133, 2048)])
@pytest.mark.parametrize("rk", [0, 1, 2])
@pytest.mark.parametrize("act,p", [("relu", 0.0), ("gelu", 0.0), ("none", 0.3)])
def test_rows_in_flight_bitwise(m, c, rk, act, p):
    torch.manual_seed(1)
    x = torch.randn(m, c, device=DEV).bfloat16()
    ss = torch.cat([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)])
    res = torch.randn(m, c, device=DEV).bfloat16() if rk else None
    ssr = torch.cat([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)]) if rk == 2 else None
    rng = O.RNG.snapshot(torch.device(DEV)) if p > 0 else None
    try:
        N.call("dmf_bn_apply_tune", 1)
        y1 = _apply(x, ss, res, ssr, act, p, rng, m, c)
        for u in (2, 4):
            N.call("dmf_bn_apply_tune", u)
            yu = _apply(x, ss, res, ssr, act, p, rng, m, c)
            assert torch.equal(y1, yu), (u, (y1.float() - yu.float()).abs().max().item())
    finally:
        N.call("dmf_bn_apply_tune", 1)
    # and the one-row form against a torch statement of the same pass
    z = x.float() * ss[:c] + ss[c:]
    if rk:
        z = z + (res.float() * ssr[:c] + ssr[c:] if rk == 2 else res.float())
    if act == "relu":
        z = z.relu()
    elif act == "gelu":
        z = torch.nn.functional.gelu(z)
    if p > 0:
        kept = y1.float() != 0
        z = torch.where(kept, z / (1 - p), torch.zeros_like(z))
        assert abs(kept.float().mean().item() - (1 - p)) < 0.02
    assert torch.allclose(y1.float(), z, rtol=2 ** -7, atol=1e-5)
