"""GPU: dmf_sgemm (the fusion's fp32 token linears and their gradients, FusionModel model_module.py:821-1000)
in both forms -- 16 x 16 fp32-MFMA tiles (k_sgemm_mfma, default for M * N <= 512^2) and the 64 x 64 VALU
tile with split-K (k_sgemm) -- against float64: every op(A) / op(B) layout, alpha, an accumulating beta,
bias and activation, ragged M / N / K."""
import pytest
import torch
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(ta, tb, a, b, alpha, beta, c0, bias, act):
    A = a.double().t() if ta else a.double()
    B = b.double().t() if tb else b.double()
    v = alpha * (A @ B) + beta * c0.double()
    if bias is not None:
        v = v + bias.double()
    return {"none": v, "relu": F.relu(v), "gelu": F.gelu(v), "sigmoid": torch.sigmoid(v)}[act]


@pytest.mark.parametrize("mfma", [1, 0])
@pytest.mark.parametrize("ta,tb,m,n,k,beta,act", [(0, 1, 512, 128, 128, 0.0, "none"), (0, 0, 512, 128, 384, 0.0, "gelu"),
                                                  (1, 0, 384, 128, 512, 1.0, "none"), (0, 1, 37, 61, 53, 0.5, "sigmoid"),
                                                  (1, 1, 32, 4, 512, 0.0, "relu")])
def test_sgemm_forms(mfma, ta, tb, m, n, k, beta, act):
    torch.manual_seed(m + n + k)
    a = torch.randn((k, m) if ta else (m, k), device=DEV)
    b = torch.randn((n, k) if tb else (k, n), device=DEV)
    c = torch.randn(m, n, device=DEV)
    bias = torch.randn(n, device=DEV)
    alpha = 0.75
    want = _ref(ta, tb, a, b, alpha, beta, c, bias, act)
    ws_n = N.load().dmf_sgemm_ws_size(m, n, k)
    ws = torch.empty(max(ws_n, 1), device=DEV)
    N.call("dmf_sgemm_tune", mfma)
    try:
        N.call("dmf_sgemm", ta, tb, m, n, k, alpha, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1], beta,
               c.data_ptr(), n, bias.data_ptr(), O.ACT[act], ws.data_ptr(), N.stream_ptr())
    finally:
        N.call("dmf_sgemm_tune", 1)
    torch.cuda.synchronize()
    err = (c.double() - want).abs().max().item()
    assert err <= 2e-5 * max(1.0, want.abs().max().item()) * (k / 128) ** 0.5, err
