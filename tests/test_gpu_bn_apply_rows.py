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


@pytest.mark.parametrize("m,c", [(32768, 256), (1000, 72), (4133, 2048)])
def test_bwd_apply_rows_in_flight(m, c):
    """dmf_bn_bwd_apply_acc (training BN backward, finalize from the float64 arena) against the
    torch statement dx = g*inv*(dz - mean(dz) - xhat*mean(dz*xhat)), and its 2 / 4 rows-in-flight
    forms bitwise against the one-row form."""
    torch.manual_seed(2)
    reps = O.BN_ACC_REPLICAS
    x = (torch.randn(m, c, device=DEV) * 2 + 0.5).bfloat16()
    dz = torch.randn(m, c, device=DEV).bfloat16()
    xf = x.double()
    mean = xf.mean(0)
    inv = (xf.var(0, unbiased=False) + 1e-5).rsqrt()
    xhat = (xf - mean) * inv
    s, q = dz.double().sum(0), (dz.double() * xhat).sum(0)
    w = torch.rand(reps, 1, device=DEV, dtype=torch.float64)
    w = w / w.sum()
    acc = torch.stack([w * s, w * q], -1).contiguous()  # [reps][C][2], sums to (s, q)
    save = torch.cat([mean, inv]).float()
    gamma = torch.rand(c, device=DEV) + 0.5

    def run(u):
        N.call("dmf_bn_bwd_apply_tune", u)
        dx = torch.empty_like(x)
        dg, db = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
        N.call("dmf_bn_bwd_apply_acc", N.BF16, dz.data_ptr(), c, x.data_ptr(), c, acc.data_ptr(), reps, float(m), 1,
               gamma.data_ptr(), save.data_ptr(), dg.data_ptr(), db.data_ptr(), dx.data_ptr(), c, m, c,
               N.stream_ptr())
        torch.cuda.synchronize()
        return dx, dg, db

    try:
        dx1, dg1, db1 = run(1)
        for u in (2, 4):
            dxu, dgu, dbu = run(u)
            assert torch.equal(dx1, dxu) and torch.equal(dg1, dgu) and torch.equal(db1, dbu), u
    finally:
        N.call("dmf_bn_bwd_apply_tune", 1)
    ref = gamma.double() * inv * (dz.double() - s / m - xhat * q / m)
    assert torch.allclose(dx1.double(), ref, rtol=2 ** -7, atol=2e-3 * ref.abs().max().item())
    assert torch.allclose(db1.double(), s, rtol=1e-6, atol=1e-3)
    assert torch.allclose(dg1.double(), q, rtol=1e-6, atol=1e-3)
