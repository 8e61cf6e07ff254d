"""GPU: the e4m3 patch-embed GEMM (dmf_gemm_fp8, csrc/fp8.hip) in both forms -- the 128x128
non-scaled v_mfma_f32_16x16x32_fp8_fp8 tile and the 144x256 block-scaled
v_mfma_scale_f32_16x16x128_f8f6f4 tile (unit E8M0 scales) -- against the fp64 product of the
dequantised operands: configuration 5's production shape (18432 x 512 x 1024: 32 volumes x 576
tokens, PatchEmbed P = 2 over 256 channels, transformer_model.py:17-22), ragged M / N / K tails
(rows past M, a partial 256-column tile, K not a multiple of the 128-B K-step), and the two forms
against each other. Which form ran is read from dmf_gemm_fp8_last_form."""
import pytest
import torch

import dmf_native as N

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(m, n, k, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    a = (torch.randn(m, k, generator=g) * 100).clamp(-448, 448).to(torch.float8_e4m3fn)
    b = (torch.randn(n, k, generator=g) * 100).clamp(-448, 448).to(torch.float8_e4m3fn)
    asc = torch.rand(m, generator=g) * 0.01 + 1e-3
    bsc = torch.rand(n, generator=g) * 0.01 + 1e-3
    bias = torch.randn(n, generator=g)
    return a, b, asc, bsc, bias


def _ref(a, b, asc, bsc, bias):
    ad, bd = a.to(DEV).double(), b.to(DEV).double()
    return (ad @ bd.t()) * asc.to(DEV).double()[:, None] * bsc.to(DEV).double()[None, :] + bias.to(DEV).double()


def _run(a, b, asc, bsc, bias, var):
    m, k = a.shape
    n = b.shape[0]
    ad, bd = a.view(torch.uint8).to(DEV).contiguous(), b.view(torch.uint8).to(DEV).contiguous()
    asd, bsd, biasd = asc.to(DEV), bsc.to(DEV), bias.to(DEV)
    c = torch.full((m, n), float("nan"), dtype=torch.bfloat16, device=DEV)
    N.call("dmf_gemm_fp8_tune", var)
    try:
        N.call("dmf_gemm_fp8", m, n, k, ad.data_ptr(), k, asd.data_ptr(), bd.data_ptr(), k, bsd.data_ptr(),
               biasd.data_ptr(), c.data_ptr(), n, N.stream_ptr())
        form = N.load().dmf_gemm_fp8_last_form()
    finally:
        N.call("dmf_gemm_fp8_tune", 1)
    torch.cuda.synchronize()
    return c, form


@pytest.mark.parametrize("m,n,k,form", [
    (18432, 512, 1024, 1),        # configuration 5, B = 32: 128 x 2 tiles of 144 x 256
    (18432 + 77, 520, 1040, 1),   # ragged rows, a 8-column third tile, K % 128 == 16
    (36864, 256, 128, 1),         # one K-step
    (300, 512, 1024, 0),          # too few 144 x 256 tiles to fill the chip: the 128 x 128 form
])
def test_fp8_gemm_forms(m, n, k, form):
    a, b, asc, bsc, bias = _operands(m, n, k, seed=m + n + k)
    ref = _ref(a, b, asc, bsc, bias)
    c, got_form = _run(a, b, asc, bsc, bias, 1)
    assert got_form == form
    assert torch.isfinite(c.float()).all()
    err = (c.double() - ref).abs()
    # bf16 output rounding (2^-8 relative) over fp32 accumulation of exact e4m3 products
    assert (err <= ref.abs() * 2 ** -8 + 1e-3 * ref.abs().max()).all(), err.max().item()


def test_fp8_gemm_forms_agree():
    m, n, k = 18432, 512, 1024
    a, b, asc, bsc, bias = _operands(m, n, k, seed=5)
    c1, f1 = _run(a, b, asc, bsc, bias, 1)
    c0, f0 = _run(a, b, asc, bsc, bias, 0)
    assert (f1, f0) == (1, 0)
    # same products, different fp32 summation order: at most one bf16 ulp apart
    d = (c1.float() - c0.float()).abs()
    assert (d <= c0.float().abs() * 2 ** -7 + 1e-6).all(), d.max().item()
