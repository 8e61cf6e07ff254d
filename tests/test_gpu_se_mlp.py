"""GPU: the SEBlock excitation (model_module.py:63-80 SEBlock; dmf_se_mlp) in its three forms -- two
launches of fp32-MFMA tiles (k_se_dense, default), one workgroup (k_se_mlp1) and three launches
(k_sum_planes + k_dense_rows) -- against a float64 restatement: squeeze partial planes with a scale, every output
(pooled, hpre, hact, gate), ragged N / C / mid, and a shape that keeps the three-launch form."""
import pytest
import torch
import torch.nn.functional as F

import dmf_native as N

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(ws, s, n, c, scale, w1, b1, w2, b2, one):
    mid = w1.shape[0]
    out = [torch.full((n, c), float("nan"), device=DEV), torch.full((n, mid), float("nan"), device=DEV),
           torch.full((n, mid), float("nan"), device=DEV), torch.full((n, c), float("nan"), device=DEV)]
    N.call("dmf_se_mlp_tune", one)
    try:
        N.call("dmf_se_mlp", ws.data_ptr(), s, n, c, float(scale), w1.data_ptr(), b1.data_ptr(), mid, w2.data_ptr(),
               b2.data_ptr(), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(),
               N.stream_ptr())
    finally:
        N.call("dmf_se_mlp_tune", 1)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("n,c,mid,s", [(32, 128, 64, 1), (32, 128, 64, 8), (5, 72, 36, 3), (32, 256, 128, 4),
                                       (32, 14, 7, 1)])
def test_se_mlp_one_launch(n, c, mid, s):
    torch.manual_seed(n + c + mid)
    ws = torch.randn(s, n, c, device=DEV)
    scale = 1.0 / (s * 7)
    w1, b1 = torch.randn(mid, c, device=DEV) / c ** 0.5, torch.randn(mid, device=DEV) * 0.1
    w2, b2 = torch.randn(c, mid, device=DEV) / mid ** 0.5, torch.randn(c, device=DEV) * 0.1
    pooled = ws.double().sum(0) * scale
    hpre = pooled @ w1.double().t() + b1.double()
    hact = F.gelu(hpre)
    gate = torch.sigmoid(hact @ w2.double().t() + b2.double())
    want = [pooled, hpre, hact, gate]
    forms = {mode: _run(ws, s, n, c, scale, w1, b1, w2, b2, mode) for mode in (1, 2, 0)}
    for mode, outs in forms.items():
        for name, a, ref in zip(("pooled", "hpre", "hact", "gate"), outs, want):
            assert torch.isfinite(a).all(), (mode, name)
            tol = 2e-5 * max(1.0, ref.abs().max().item())
            assert (a.double() - ref).abs().max().item() <= tol, (mode, name, (a.double() - ref).abs().max().item())
