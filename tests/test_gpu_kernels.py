"""Kernel-level numerics: each HIP op against a plain PyTorch fp32 reference of
the same op (computed on the CPU), in the f32 parity mode (tight tolerance)
and the bf16 throughput mode (bf16 tolerance)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _to_dev(x, dtype):
    return x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)


def _tol(dtype):
    return (2e-4, 2e-4) if dtype == torch.float32 else (3e-2, 3e-2)


CONV_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, dil)
    (2, 64, 16, 16, 64, 1, 1, 0, 1),
    (2, 64, 16, 16, 128, 3, 1, 1, 1),
    (2, 128, 17, 13, 64, 3, 2, 1, 1),
    (1, 64, 20, 20, 256, 3, 1, 2, 2),
    (1, 256, 12, 12, 128, 3, 1, 4, 4),
    (2, 16, 32, 32, 64, 7, 2, 3, 1),
    (2, 256, 8, 8, 512, 1, 2, 0, 1),
    (3, 8, 9, 9, 8, 3, 1, 1, 1),
    # large enough for the 128-row tiles of the buffer-load forward kernel
    (64, 64, 32, 32, 128, 3, 1, 1, 1),
    (64, 128, 32, 32, 64, 1, 1, 0, 1),
    # more blocks than resident slots: the persistent forward kernel
    (64, 128, 32, 32, 256, 1, 1, 0, 1),
    (48, 64, 32, 32, 256, 3, 1, 1, 1),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case, dtype):
    n, ci, h, w, co, k, s, p, d = case
    torch.manual_seed(0)
    conv = nn.Conv2d(ci, co, k, stride=s, padding=p, dilation=d, bias=True)
    x = torch.randn(n, ci, h, w)
    xr = x.clone().requires_grad_(True)
    yr = F.conv2d(xr, conv.weight, conv.bias, s, p, d)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    cd = copy.deepcopy(conv).to(DEV)
    cd.zero_grad(set_to_none=True)
    xd = _to_dev(x, dtype).requires_grad_(True)
    caches = (O.WeightCache(), O.WeightCache())
    y = O.conv2d(xd, cd, caches)
    rtol, atol = _tol(dtype)
    scale = yr.abs().max().item()
    assert torch.allclose(y.float().cpu(), yr.detach(), rtol=rtol, atol=atol * scale), \
        (y.float().cpu() - yr.detach()).abs().max()
    y.backward(_to_dev(gy, dtype))
    gscale = xr.grad.abs().max().item()
    assert torch.allclose(xd.grad.float().cpu(), xr.grad, rtol=rtol, atol=atol * gscale), \
        (xd.grad.float().cpu() - xr.grad).abs().max()
    wscale = conv.weight.grad.abs().max().item() if conv.weight.grad is not None else 1
    ref_w = torch.nn.grad.conv2d_weight(x, conv.weight.shape, gy, s, p, d)
    assert torch.allclose(cd.weight.grad.cpu(), ref_w, rtol=rtol, atol=atol * ref_w.abs().max().item()), \
        (cd.weight.grad.cpu() - ref_w).abs().max()
    assert torch.allclose(cd.bias.grad.cpu(), gy.sum((0, 2, 3)), rtol=rtol, atol=atol * gy.abs().sum((0, 2, 3)).max())


# shapes that take the 256x128 LDS-DMA forward kernel (bf16, Cout % 128 == 0,
# K >= 512, >= 256 blocks): dilated 3x3 with zero padding and an M tail, a
# plain 1x1, and the neck's channel-concat (two-source) 3x3
WIDE_CASES = [
    # (N, Cin, H, W, Cout, k, pad, dil, Cin2)
    (33, 256, 32, 32, 256, 3, 2, 2, 0),
    (33, 512, 32, 32, 512, 1, 0, 1, 0),
    (32, 128, 32, 32, 256, 3, 1, 1, 384),
    # 256x256 square-tile LDS-DMA kernel (Cout % 256 == 0, >= 256 blocks):
    # padded dilated 3x3 with an M tail, channel-concat 3x3, plain 1x1
    (65, 64, 31, 31, 512, 3, 2, 2, 0),
    (36, 64, 31, 31, 512, 3, 1, 1, 64),
    (34, 512, 32, 32, 1024, 1, 0, 1, 0),
    (34, 2048, 32, 32, 512, 1, 0, 1, 0),
]


@pytest.mark.parametrize("case", WIDE_CASES)
def test_conv_wide_forward_and_bn_stats(case):
    n, ci, h, w, co, k, p, d, ci2 = case
    torch.manual_seed(5)
    conv = nn.Conv2d(ci + ci2, co, k, padding=p, dilation=d, bias=False)
    bn = nn.BatchNorm2d(co)
    a = torch.randn(n, ci, h, w).bfloat16().float()
    b = torch.randn(n, ci2, h, w).bfloat16().float() if ci2 else None
    wq = conv.weight.detach().bfloat16().float()
    xin = torch.cat([a, b], 1) if ci2 else a
    with torch.no_grad():
        raw = F.conv2d(xin, wq, None, 1, p, d)
        ref = F.relu(bn(raw))
    cd, bd = copy.deepcopy(conv).to(DEV), nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        y = O.conv_bn_act(_to_dev(a, torch.bfloat16), cd, (O.WeightCache(), O.WeightCache()), bd, "relu",
                          x2=_to_dev(b, torch.bfloat16) if ci2 else None)
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 3e-2 * ref.abs().max().item(), err
    # batch statistics (running stats after one momentum-0.1 update), tolerance for bf16 outputs
    assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=1e-2, atol=1e-3 * raw.abs().max().item())
    assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=2e-2, atol=1e-3)


# bf16 backward at the encoder's shapes: the weight gradient on the
# transposed-LDS-read kernel (pixel splits, tap-crossing K tiles, M tails,
# the neck's two-source input) and the stride-1 input gradient as a forward
# conv of dY with flipped taps (the LDS-DMA tiles); stride 2 keeps the gather
BWD_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, dil, Cin2)
    (8, 256, 32, 32, 256, 3, 1, 2, 2, 0),
    (9, 512, 32, 32, 512, 1, 1, 0, 1, 0),
    (4, 128, 32, 32, 256, 3, 1, 1, 1, 384),
    (4, 64, 33, 31, 128, 3, 2, 1, 1, 0),
    (3, 64, 20, 20, 64, 3, 1, 4, 4, 0),
    (2, 72, 17, 19, 40, 3, 1, 1, 1, 0),
    (16, 2048, 16, 16, 512, 1, 1, 0, 1, 0),
]


@pytest.mark.parametrize("case", BWD_CASES)
def test_conv_backward_bf16(case):
    n, ci, h, w, co, k, s, p, d, ci2 = case
    torch.manual_seed(6)
    q = lambda t: t.bfloat16().float()
    a = q(torch.randn(n, ci, h, w))
    b = q(torch.randn(n, ci2, h, w)) if ci2 else None
    conv = nn.Conv2d(ci + ci2, co, k, stride=s, padding=p, dilation=d, bias=False)
    wq = q(conv.weight.detach())
    xin = (torch.cat([a, b], 1) if ci2 else a).double().requires_grad_(True)
    wr = wq.double().requires_grad_(True)
    yr = F.conv2d(xin, wr, None, s, p, d)
    gy = q(torch.randn(yr.shape))
    yr.backward(gy.double())
    cd = copy.deepcopy(conv).to(DEV)
    with torch.no_grad():
        cd.weight.copy_(wq)
    g = O.ConvGeom(cd)
    xd = _to_dev(a, torch.bfloat16)
    x2d = _to_dev(b, torch.bfloat16) if ci2 else None
    dx, dw, _ = O._conv_backward(xd, cd.weight, None, g, (O.WeightCache(), O.WeightCache()),
                                 _to_dev(gy, torch.bfloat16), True, True, False, x2=x2d)
    if ci2:
        dx = torch.cat([dx[0].float(), dx[1].float()], 1)
    ref_dx, ref_dw = xin.grad.float(), wr.grad.float()
    err_x = (dx.float().cpu() - ref_dx).abs().max().item()
    assert err_x <= 1e-2 * ref_dx.abs().max().item(), err_x
    err_w = (dw.cpu() - ref_dw).abs().max().item()
    assert err_w <= 1e-3 * ref_dw.abs().max().item(), err_w


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_dual_source(dtype):
    torch.manual_seed(1)
    a = torch.randn(2, 64, 8, 8)
    b = torch.randn(2, 128, 8, 8)
    conv = nn.Conv2d(192, 64, 3, padding=1)
    bn = nn.BatchNorm2d(64)
    ref = F.gelu(bn(F.conv2d(torch.cat([a, b], 1), conv.weight, conv.bias, 1, 1)))
    cd, bd = conv.to(DEV), nn.BatchNorm2d(64).to(DEV)
    y = O.conv_bn_act(_to_dev(a, dtype), cd, (O.WeightCache(), O.WeightCache()), bd, "gelu", x2=_to_dev(b, dtype))
    rtol, atol = _tol(dtype)
    assert torch.allclose(y.float().cpu(), ref.detach(), rtol=rtol, atol=atol * 4)
    assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=1e-3, atol=1e-4 if dtype == torch.float32 else 1e-2)
    assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=1e-3, atol=1e-3 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_conv_bn_act_residual_grads(act):
    torch.manual_seed(2)
    x = torch.randn(2, 32, 10, 10)
    xs = torch.randn(2, 16, 20, 20)
    conv = nn.Conv2d(32, 64, 1)
    bn = nn.BatchNorm2d(64)
    cs = nn.Conv2d(16, 64, 1, stride=2, bias=False)
    bns = nn.BatchNorm2d(64)
    for m in (bn, bns):
        m.weight.data.uniform_(0.5, 1.5)
        m.bias.data.uniform_(-0.5, 0.5)
    xr, xsr = x.clone().requires_grad_(True), xs.clone().requires_grad_(True)
    f = F.relu if act == "relu" else F.gelu
    ref = f(bn(F.conv2d(xr, conv.weight, conv.bias)) + bns(F.conv2d(xsr, cs.weight, None, 2)))
    g = torch.randn_like(ref)
    ref.backward(g)
    mods = [copy.deepcopy(m).to(DEV) for m in (conv, bn, cs, bns)]
    for m in mods:
        m.zero_grad(set_to_none=True)
    xd = _to_dev(x, torch.float32).requires_grad_(True)
    xsd = _to_dev(xs, torch.float32).requires_grad_(True)
    y = O.conv_bn_act(xd, mods[0], (O.WeightCache(), O.WeightCache()), mods[1], act,
                      skip=(xsd, mods[2], (O.WeightCache(), O.WeightCache()), mods[3]))
    y.backward(_to_dev(g, torch.float32))
    assert torch.allclose(y.cpu(), ref.detach(), atol=2e-4, rtol=2e-4)
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=2e-4, rtol=2e-3)
    assert torch.allclose(xsd.grad.cpu(), xsr.grad, atol=2e-4, rtol=2e-3)
    assert torch.allclose(mods[1].weight.grad.cpu(), bn.weight.grad, atol=1e-3, rtol=1e-3)
    assert torch.allclose(mods[3].bias.grad.cpu(), bns.bias.grad, atol=1e-3, rtol=1e-3)
    assert torch.allclose(mods[0].weight.grad.cpu(), conv.weight.grad, atol=1e-3, rtol=1e-3)


def test_dropout_statistics_and_backward():
    torch.manual_seed(3)
    x = torch.randn(4, 64, 16, 16, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    rng = O.RNG.snapshot(DEV)
    site = O.RNG.new_site()
    y = O.act_nhwc(x, "none", dropout_p=0.2, rng=rng, site=site)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.8) < 0.01
    nz = y != 0
    assert torch.allclose(y[nz], x.detach()[nz] / 0.8, rtol=1e-6)
    y.sum().backward()
    assert torch.equal(x.grad != 0, nz)
    # same snapshot + site -> same mask
    y2 = O.act_nhwc(x.detach(), "none", dropout_p=0.2, rng=rng, site=site)
    assert torch.equal(y2 != 0, nz)


@pytest.mark.parametrize("c,dtype", [(32, torch.float32), (36, torch.float32), (64, torch.bfloat16)])
def test_gn_mix_and_grads(c, dtype):
    """GroupNorm(C,C) of the mix, forward + backward: C % 8 == 0 runs the 8-wide apply kernels
    (k_gn_apply8 / k_gn_bwd_apply8), C = 36 the element-wise ones."""
    torch.manual_seed(4)
    a = torch.randn(2, c, 8, 8)
    b = torch.randn(2, c, 8, 8)
    if dtype == torch.bfloat16:
        a, b = a.bfloat16().float(), b.bfloat16().float()
    w = torch.tensor(0.3)
    gn = nn.GroupNorm(c, c)
    gn.weight.data.uniform_(0.5, 1.5)
    gn.bias.data.uniform_(-1, 1)
    ar, br, wr = a.clone().requires_grad_(True), b.clone().requires_grad_(True), w.clone().requires_grad_(True)
    al = torch.sigmoid(wr)
    ref = gn(al * ar + (1 - al) * br)
    g = torch.randn_like(ref)
    ref.backward(g)
    gnd = copy.deepcopy(gn).to(DEV)
    gnd.zero_grad(set_to_none=True)
    ad = _to_dev(a, dtype).requires_grad_(True)
    bd = _to_dev(b, dtype).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = O.gn_mix(ad, bd, wd, gnd)
    y.backward(_to_dev(g, dtype))
    k = 1 if dtype == torch.float32 else 100  # bf16: the mix, y and dy round to 8 bits
    assert torch.allclose(y.float().cpu(), ref.detach(), atol=1e-4 * k, rtol=1e-4 * k)
    assert torch.allclose(ad.grad.float().cpu(), ar.grad, atol=1e-4 * k, rtol=1e-3 * k)
    assert torch.allclose(bd.grad.float().cpu(), br.grad, atol=1e-4 * k, rtol=1e-3 * k)
    assert torch.allclose(wd.grad.cpu(), wr.grad, atol=1e-3 * k, rtol=1e-3 * k)
    # dgamma / dbeta sum 2*8*8 products each; in bf16 the stored mix and dy carry 2^-8 relative errors,
    # so their bound scales with the largest sum, not with each (possibly cancelled) entry
    for got, want in ((gnd.weight.grad.cpu(), gn.weight.grad), (gnd.bias.grad.cpu(), gn.bias.grad)):
        atol = 1e-4 if k == 1 else 2e-2 * want.abs().max().item()
        assert torch.allclose(got, want, atol=atol, rtol=1e-3 * k), (got - want).abs().max().item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_maxpool_recorded_positions_match_rescan(dtype):
    """dmf_maxpool2d_idx + dmf_maxpool2d_bwd_idx (the autograd path for C % 8 == 0)
    against the window re-scan of dmf_maxpool2d / dmf_maxpool2d_bwd: bit-exact,
    with heavy ties (integer-valued input), a NaN, and odd spatial sizes."""
    import dmf_native as N
    torch.manual_seed(6)
    x = torch.randint(-3, 4, (3, 64, 33, 30)).float()
    x[0, 5, 3, 4] = float("nan")
    xd = _to_dev(x, dtype).requires_grad_(True)
    y = O.maxpool2d(xd, 3, 2, 1)
    g = torch.randn(y.shape)
    gd = _to_dev(g, dtype)
    y.backward(gd)
    n, c, h, w = x.shape
    ho, wo = y.shape[2], y.shape[3]
    xs = xd.detach()
    y2 = O.empty_nhwc(n, c, ho, wo, dtype, xs.device)
    N.call("dmf_maxpool2d", O.dt(xs), xs.data_ptr(), n, h, w, c, c, y2.data_ptr(), ho, wo, c, 3, 2, 1, O._stream())
    dx2 = O.empty_nhwc(n, c, h, w, dtype, xs.device)
    N.call("dmf_maxpool2d_bwd", O.dt(xs), xs.data_ptr(), n, h, w, c, c, gd.data_ptr(), ho, wo, c, dx2.data_ptr(), c,
           3, 2, 1, O._stream())
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(y.detach(), nan=1234.0), torch.nan_to_num(y2, nan=1234.0))
    assert torch.equal(xd.grad, dx2)
    ref = F.max_pool2d(x.to(dtype).float().requires_grad_(True), 3, 2, 1)
    assert torch.equal(torch.nan_to_num(y.detach().float().cpu(), nan=9.0), torch.nan_to_num(ref.detach(), nan=9.0))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_maxpool_gradient_routing_matches_torch_on_inf_and_nan_windows(dtype):
    """Window argmax rule of torch's max_pool2d_with_indices: the
    index starts at the window's first valid element and moves on
    ``v > max || isnan(v)``. An all -inf window sends its gradient to that
    first element (not nowhere), two NaNs in a window route to the later one.
    Both the recorded-position path (C % 8 == 0) and the re-scan backward are
    compared with torch's CPU max_pool2d backward, bit for bit."""
    import dmf_native as N
    torch.manual_seed(8)
    x = torch.randn(2, 16, 9, 10)
    x[0, :, 0:4, 0:4] = float("-inf")   # windows of (0,0), (0,1), (1,0), (1,1) entirely -inf
    x[1, 3, 4, 4] = float("nan")
    x[1, 3, 4, 5] = float("nan")        # the later NaN of window (2,2) wins
    x[1, 7, :, :] = float("-inf")       # a whole -inf channel
    xr = x.clone().to(dtype).float().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    g = torch.randn(ref.shape).to(dtype).float()  # representable in dtype: both sides sum the same values
    ref.backward(g)
    xd = _to_dev(x, dtype).requires_grad_(True)
    y = O.maxpool2d(xd, 3, 2, 1)
    y.backward(_to_dev(g, dtype))
    want = xr.grad.to(dtype).float()
    assert torch.equal(xd.grad.float().cpu(), want)
    n, c, h, w = x.shape
    ho, wo = y.shape[2], y.shape[3]
    xs = xd.detach()
    dx2 = O.empty_nhwc(n, c, h, w, dtype, xs.device)
    gd = _to_dev(g, dtype)
    N.call("dmf_maxpool2d_bwd", O.dt(xs), xs.data_ptr(), n, h, w, c, c, gd.data_ptr(), ho, wo, c, dx2.data_ptr(), c,
           3, 2, 1, O._stream())
    torch.cuda.synchronize()
    assert torch.equal(dx2.float().cpu(), want)


def test_maxpool_and_bilinear_and_tokens():
    torch.manual_seed(5)
    x = torch.randn(2, 16, 17, 15)
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    g = torch.randn_like(ref)
    ref.backward(g)
    xd = _to_dev(x, torch.float32).requires_grad_(True)
    y = O.maxpool2d(xd, 3, 2, 1)
    y.backward(_to_dev(g, torch.float32))
    assert torch.allclose(y.cpu(), ref.detach())
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-6)
    # bilinear 4 -> 32 and 32 -> 64
    for (h, H) in [(4, 32), (32, 64), (7, 20)]:
        z = torch.randn(2, 8, h, h)
        zr = z.clone().requires_grad_(True)
        r = F.interpolate(zr, size=(H, H), mode="bilinear", align_corners=False)
        gg = torch.randn_like(r)
        r.backward(gg)
        zd = _to_dev(z, torch.float32).requires_grad_(True)
        o = O.bilinear(zd, H, H)
        o.backward(_to_dev(gg, torch.float32))
        assert torch.allclose(o.cpu(), r.detach(), atol=1e-5)
        assert torch.allclose(zd.grad.cpu(), zr.grad, atol=1e-4, rtol=1e-4)
    # tokens (adaptive avg pool 32 -> 4)
    t = torch.randn(2, 16, 32, 32)
    tr = t.clone().requires_grad_(True)
    ref_t = F.adaptive_avg_pool2d(tr, (4, 4)).flatten(2).transpose(1, 2)
    gt = torch.randn_like(ref_t)
    ref_t.backward(gt)
    td = _to_dev(t, torch.float32).requires_grad_(True)
    tok = O.to_tokens(td, 4, 4)
    tok.backward(gt.to(DEV))
    assert torch.allclose(tok.cpu(), ref_t.detach(), atol=1e-5)
    assert torch.allclose(td.grad.cpu(), tr.grad, atol=1e-6)


def test_se_block_grads():
    torch.manual_seed(6)
    import model_module as MM

    se = MM.SEBlock(32, 2)
    MM.set_compute_dtype(se, torch.float32)
    x = torch.randn(2, 32, 8, 8)
    xr = x.clone().requires_grad_(True)
    fc = se.fc
    w = torch.sigmoid(F.conv2d(F.gelu(F.conv2d(xr.mean((2, 3), keepdim=True), fc[1].weight, fc[1].bias)),
                               fc[3].weight, fc[3].bias))
    ref = xr * w
    g = torch.randn_like(ref)
    ref.backward(g)
    ref_g1 = torch.autograd.grad(
        (xr.detach() * torch.sigmoid(F.conv2d(F.gelu(F.conv2d(xr.detach().mean((2, 3), keepdim=True), fc[1].weight,
                                                              fc[1].bias)), fc[3].weight, fc[3].bias)) * g).sum(),
        fc[1].weight)[0]
    sed = copy.deepcopy(se).to(DEV)
    sed.zero_grad(set_to_none=True)
    xd = _to_dev(x, torch.float32).requires_grad_(True)
    y, wgt = sed(xd)
    y.backward(_to_dev(g, torch.float32))
    assert torch.allclose(y.cpu(), ref.detach(), atol=1e-5)
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(sed.fc[1].weight.grad.cpu(), ref_g1, atol=1e-5, rtol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(32, 512, 32, 32), (5, 128, 16, 16), (3, 14, 9, 7), (2, 6, 4, 4)])
def test_se_excite_one_launch_matches_torch(shape, dtype):
    """dmf_se_mlp (squeeze partials -> fc1 -> GELU -> fc2 -> sigmoid in one launch)
    against torch fp32, with grad off (the frozen-encoder path) and on (its saved
    pooled / hpre / hact feed the SE backward)."""
    import model_module as MM

    n, c, h, w = shape
    torch.manual_seed(11)
    se = MM.SEBlock(c, 2)
    MM.set_compute_dtype(se, dtype)
    x = torch.randn(n, c, h, w)
    xq = x.to(dtype).float()  # the input the kernel sees
    fc = se.fc
    pooled = xq.mean((2, 3))
    hpre = F.linear(pooled, fc[1].weight.flatten(1), fc[1].bias)
    gate = torch.sigmoid(F.linear(F.gelu(hpre), fc[3].weight.flatten(1), fc[3].bias))
    sed = copy.deepcopy(se).to(DEV)
    xd = _to_dev(x, dtype)
    mid = fc[1].weight.shape[0]
    with torch.no_grad():
        p, hp, ha, g = O.se_excite(xd, sed.fc[1].weight.reshape(mid, c), sed.fc[1].bias, sed.fc[3].weight.reshape(c, mid),
                                   sed.fc[3].bias, keep=True)
        y, wg = sed(xd)
    torch.testing.assert_close(p.cpu(), pooled, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(hp.cpu(), hpre, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(ha.cpu(), F.gelu(hpre), atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(g.cpu(), gate, atol=2e-5, rtol=1e-4)
    torch.testing.assert_close(wg.reshape(n, c).cpu(), gate, atol=2e-5, rtol=1e-4)
    rt = 2e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.float().cpu(), (xq * gate[:, :, None, None]), atol=rt, rtol=rt)
    # modality-attention form: a finished pool (S = 1) through the same kernel
    g1 = O.excite_mlp(pooled.to(DEV), 1, 1.0, sed.fc[1].weight.reshape(mid, c), sed.fc[1].bias,
                      sed.fc[3].weight.reshape(c, mid), sed.fc[3].bias, keep=False)[3]
    torch.testing.assert_close(g1.cpu(), gate, atol=2e-5, rtol=1e-4)


def test_mask_attention_fwd_bwd():
    torch.manual_seed(7)
    import model_module as MM
    from oracle.model import MaskGuidedSpatialAttention as RefMSA

    ref = RefMSA(32, 1)
    ref.mask_processor[1].weight.data.uniform_(0.5, 1.5)
    ref.mask_processor[1].bias.data.uniform_(-0.5, 0.5)
    mine = MM.MaskGuidedSpatialAttention(32, 1)
    mine.load_state_dict(ref.state_dict())
    MM.set_compute_dtype(mine, torch.float32)
    mine = mine.to(DEV)
    f = torch.randn(2, 32, 8, 8)
    m = torch.randn(2, 1, 8, 8)
    fr, mr = f.clone().requires_grad_(True), m.clone().requires_grad_(True)
    out_r, a_r = ref(fr, mr)
    g = torch.randn_like(out_r)
    out_r.backward(g)
    fd = _to_dev(f, torch.float32).requires_grad_(True)
    md = _to_dev(m, torch.float32).requires_grad_(True)
    out, a = mine(fd, md)
    out.backward(_to_dev(g, torch.float32))
    assert torch.allclose(out.cpu(), out_r.detach(), atol=1e-5)
    assert torch.allclose(a.cpu(), a_r.detach(), atol=1e-5)
    assert torch.allclose(fd.grad.cpu(), fr.grad, atol=1e-5)
    assert torch.allclose(md.grad.cpu(), mr.grad, atol=1e-4, rtol=1e-3)
    for (n1, p1), (n2, p2) in zip(ref.named_parameters(), mine.named_parameters()):
        assert torch.allclose(p2.grad.cpu().reshape(p1.grad.shape), p1.grad, atol=1e-4, rtol=1e-3), n1


def test_losses_match_oracle():
    torch.manual_seed(8)
    from oracle import losses as L
    import loss as LM

    logits = torch.randn(8, 4)
    labels = torch.randint(0, 4, (8,))
    cw = torch.tensor([0.5, 1.0, 1.5, 2.0])
    lr_ = logits.clone().requires_grad_(True)
    t = L.label_smoothing(lr_, labels, 4, 0.1)
    ref = L.soft_weighted_focal(lr_, t, 1.5, cw)
    ref.backward()
    ld = logits.to(DEV).requires_grad_(True)
    crit = LM.SoftWeightedFocalLoss(1.5, cw.to(DEV))
    sm = LM.LabelSmoothing(4, 0.1)(ld, labels.to(DEV))
    out = crit(ld, sm)
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-5
    assert torch.allclose(ld.grad.cpu(), lr_.grad, atol=1e-6)
    # dice
    x = torch.randn(4, 1, 32, 32)
    m = (torch.rand(4, 1, 32, 32) > 0.5).float()
    xr = x.clone().requires_grad_(True)
    rd = L.soft_dice(xr, m)
    rd.backward()
    xd = _to_dev(x, torch.float32).requires_grad_(True)
    od = LM.SoftDiceLoss()(xd, m.to(DEV))
    od.backward()
    assert abs(od.item() - rd.item()) < 1e-5
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-7)


def test_recon_and_mimic_match_oracle():
    torch.manual_seed(9)
    from oracle import losses as L
    import train_fusion as TF
    import dmf_ops

    img = torch.rand(2, 6, 64, 64)
    r1 = torch.randn(2, 1, 8, 8)
    r2 = torch.randn(2, 1, 8, 8)
    a, b = r1.clone().requires_grad_(True), r2.clone().requires_grad_(True)
    ref = L.recon_list_loss([a, b], img)
    ref.backward()
    ad = _to_dev(r1, torch.float32).requires_grad_(True)
    bd = _to_dev(r2, torch.float32).requires_grad_(True)
    out = TF.compute_recon_list_loss([ad, bd], img.to(DEV))
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-5
    assert torch.allclose(ad.grad.cpu(), a.grad, atol=1e-6, rtol=1e-4)
    # mimic over batch-item pairs (Q5)
    pf = torch.randn(4, 16, 8, 8)
    pr = pf.clone().requires_grad_(True)
    refm = (L.mimic_feat_loss(pr[0], pr[1]) + L.mimic_feat_loss(pr[2], pr[3])) / 2
    refm.backward()
    pd = _to_dev(pf, torch.float32).requires_grad_(True)
    om = dmf_ops.mimic_pairs(pd, 2)
    om.backward()
    assert abs(om.item() - refm.item()) < 1e-5
    assert torch.allclose(pd.grad.cpu(), pr.grad, atol=1e-6)


@pytest.mark.parametrize("hw_out", [(64, 64), (20, 28)])
def test_adaptive_avgpool_any_ratio(hw_out):
    """proj_pool (model_module.py:534) at S=384: AdaptiveAvgPool2d 48 -> 64 (and a shrinking ratio)."""
    torch.manual_seed(12)
    x = torch.randn(2, 16, 48, 48)
    xr = x.clone().requires_grad_(True)
    ref = F.adaptive_avg_pool2d(xr, hw_out)
    g = torch.randn_like(ref)
    ref.backward(g)
    xd = _to_dev(x, torch.float32).requires_grad_(True)
    y = O.adaptive_avgpool(xd, *hw_out)
    assert torch.allclose(y.cpu(), ref.detach(), atol=1e-5, rtol=1e-5)
    y.backward(_to_dev(g, torch.float32))
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("c,dtype", [(256, torch.bfloat16), (72, torch.float32), (12, torch.bfloat16)])
def test_adaptive_avgpool_vector_form(c, dtype):
    """The 8-channel vector form (C % 8 == 0) and the scalar fallback (C = 12), 48 -> 64 as at S=384."""
    torch.manual_seed(15)
    x = torch.randn(3, c, 48, 48).to(dtype).float()
    ref = F.adaptive_avg_pool2d(x.double(), (64, 64))
    y = O.adaptive_avgpool(_to_dev(x, dtype), 64, 64)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.float().cpu().double(), ref, atol=tol * ref.abs().max().item(), rtol=tol)


def test_fused_recon_mixed_map_sizes():
    """config 5: encoder recon maps 8x8 beside a 4x4 fused map (48x48 / 24x24 at
    S=384) -- one launch per size, same value and grads as the oracle's three
    compute_recon_list_loss calls (train_fusion.py:281-285)."""
    torch.manual_seed(13)
    from oracle import losses as L
    import train_fusion as TF

    dimg, cimg = torch.rand(2, 4, 32, 32), torch.rand(2, 3, 32, 32)
    maps = [torch.randn(2, 1, 8, 8) for _ in range(4)] + [torch.randn(2, 1, 4, 4)]
    ref_in = [m.clone().requires_grad_(True) for m in maps]
    ref = (L.recon_list_loss(ref_in[0:2], dimg) + L.recon_list_loss(ref_in[2:4], cimg)
           + L.recon_list_loss([ref_in[4]], torch.cat([dimg, cimg], 1))) / 3
    ref.backward()
    dev_in = [_to_dev(m, torch.float32).requires_grad_(True) for m in maps]
    out = TF.fused_recon_losses(dev_in[0:2], dev_in[2:4], dev_in[4], dimg.to(DEV), cimg.to(DEV))
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-5
    for a, b in zip(dev_in, ref_in):
        assert torch.allclose(a.grad.cpu(), b.grad, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mask_attention_backward_sliced(dtype):
    """MaskGuidedSpatialAttention (model_module.py:49-97) forward + backward at
    the f2 shape (32x32 = 16 slices of 64 pixels per sample) vs the oracle."""
    import oracle.model as OM
    torch.manual_seed(7)
    ref_m = OM.MaskGuidedSpatialAttention(256, 1, 16)
    with torch.no_grad():
        ref_m.gamma.fill_(0.3)
        ref_m.mask_processor[1].weight.uniform_(0.5, 1.5)
        ref_m.mask_processor[1].bias.uniform_(-0.5, 0.5)
    f = torch.randn(3, 256, 32, 32)
    m = torch.randn(3, 1, 32, 32)
    if dtype == torch.bfloat16:
        f, m = f.bfloat16().float(), m.bfloat16().float()
    fr, mr = f.clone().requires_grad_(True), m.clone().requires_grad_(True)
    out_r, a_r = ref_m(fr, mr)
    g = torch.randn_like(out_r)
    if dtype == torch.bfloat16:
        g = g.bfloat16().float()
    out_r.backward(g)
    dev_m = copy.deepcopy(ref_m).to(DEV)
    dev_m.zero_grad(set_to_none=True)
    fd = _to_dev(f, dtype).requires_grad_(True)
    md = _to_dev(m, dtype).requires_grad_(True)
    out, a = O.mask_attention(fd, md, dev_m)
    out.backward(_to_dev(g, dtype))
    tol = 2e-4 if dtype == torch.float32 else 3e-2

    def close(x, y, t):
        return (x.float().cpu() - y).abs().max().item() <= t * max(1.0, y.abs().max().item())
    assert close(out, out_r.detach(), tol)
    assert close(fd.grad, fr.grad, tol)
    assert close(md.grad, mr.grad, 5 * tol)
    for p_dev, p_ref in zip(dev_m.parameters(), ref_m.parameters()):
        assert close(p_dev.grad, p_ref.grad, 5 * tol), (p_dev.grad, p_ref.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(64, 128, 16, 16, 256, "relu"), (8, 64, 32, 32, 64, "gelu"),
                                   (4, 48, 8, 8, 32, "relu")])
def test_conv_fused_input_affine(dtype, shape):
    """Forward-only chain of the frozen encoder (foundation_model.py Bottleneck,
    model_module.py ResNetLite): conv -> BN(batch stats) -> act -> 1x1 conv ->
    BN -> act, with the first BN apply + act run inside the 1x1 conv's operand
    loads (conv_bn_stats + in_ss). Channel counts that are multiples of the
    K-step take the buffer-load kernel; 48 takes the im2col fallback."""
    n, c, h, w, co, act = shape
    torch.manual_seed(5)
    x = torch.randn(n, c, h, w)
    c1, c2 = nn.Conv2d(c, c, 3, padding=1, bias=False), nn.Conv2d(c, co, 1, bias=False)
    b1, b2 = nn.BatchNorm2d(c), nn.BatchNorm2d(co)
    for m in (b1, b2):
        m.weight.data.uniform_(0.5, 1.5)
        m.bias.data.uniform_(-0.5, 0.5)
    f = F.relu if act == "relu" else F.gelu
    with torch.no_grad():
        ref = f(b2(c2(f(b1(c1(x))))))
    mods = [copy.deepcopy(m).to(DEV) for m in (c1, c2)]
    bns = [copy.deepcopy(m).to(DEV) for m in (b1, b2)]
    for m in bns:
        m.running_mean.zero_()
        m.running_var.fill_(1.0)
    with torch.no_grad():
        xd = _to_dev(x, dtype)
        y1, ss = O.conv_bn_stats(xd, mods[0], (O.WeightCache(), O.WeightCache()), bns[0])
        y = O.conv_bn_act(y1, mods[1], (O.WeightCache(), O.WeightCache()), bns[1], act, in_ss=ss, in_act=act)
    rtol, atol = _tol(dtype)
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= atol * 4 + rtol * ref.abs().max().item(), err
    assert torch.allclose(bns[1].running_mean.cpu(), b2.running_mean, rtol=1e-3,
                          atol=1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(32, 64, 32, 32), (3, 24, 7, 9), (2, 520, 5, 6), (1, 3, 4, 4)])
def test_col_stats_partials(shape, dtype):
    """dmf_col_stats (vector and scalar forms): per-256-row-tile column (sum, sum^2)."""
    n, c, h, w = shape
    torch.manual_seed(12)
    x = torch.randn(n, c, h, w)
    xd = _to_dev(x, dtype)
    part = O._col_stats(xd).cpu().double()
    xr = xd.float().cpu().permute(0, 2, 3, 1).reshape(-1, c).double()
    m = xr.shape[0]
    tiles = (m + 255) // 256
    assert part.shape == (tiles, c, 2)
    for t in range(tiles):
        blk = xr[t * 256:(t + 1) * 256]
        torch.testing.assert_close(part[t, :, 0], blk.sum(0), atol=1e-3, rtol=1e-4)
        torch.testing.assert_close(part[t, :, 1], (blk * blk).sum(0), atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(4, 128, 16, 16, 3, 1, 1), (5, 64, 12, 12, 1, 1, 0), (3, 12, 9, 7, 3, 1, 1),
                                  (2, 16, 10, 10, 3, 2, 1)])
def test_conv_cout1_backward(case, dtype):
    """1-output-channel convs (mask / recon heads): the forward, the input gradient (8-channel
    vector form), weight and bias gradients (pixel-lane partials + the 16-lane
    split sum) against torch fp32."""
    n, ci, h, w, k, s, p = case
    torch.manual_seed(13)
    conv = nn.Conv2d(ci, 1, k, stride=s, padding=p, bias=True)
    x = torch.randn(n, ci, h, w).to(dtype).float()
    xr = x.clone().requires_grad_(True)
    yr = F.conv2d(xr, conv.weight, conv.bias, s, p)
    gy = torch.randn_like(yr).to(dtype).float()
    yr.backward(gy)
    cd = copy.deepcopy(conv).to(DEV)
    cd.zero_grad(set_to_none=True)
    xd = _to_dev(x, dtype).requires_grad_(True)
    y = O.conv2d(xd, cd, (O.WeightCache(), O.WeightCache()))
    # forward: the 8-channel vector kernel (Cin % 8 == 0: 16 or 8 lanes per pixel) or the scalar one
    yt = yr.detach().abs().max().item()
    torch.testing.assert_close(y.detach().float().cpu(), yr.detach(), rtol=2e-4 if dtype == torch.float32 else 1e-2,
                               atol=(1e-5 if dtype == torch.float32 else 1e-2) * yt)
    y.backward(_to_dev(gy, dtype))
    rt = 2e-4 if dtype == torch.float32 else 2e-2
    gx = xr.grad.abs().max().item()
    torch.testing.assert_close(xd.grad.float().cpu(), xr.grad, rtol=rt, atol=rt * gx)
    gw = conv.weight.grad.abs().max().item()
    torch.testing.assert_close(cd.weight.grad.cpu(), conv.weight.grad, rtol=1e-3, atol=1e-4 * gw)
    torch.testing.assert_close(cd.bias.grad.cpu(), conv.bias.grad, rtol=1e-4, atol=1e-4)


def test_channel_mean_reuse_never_stale():
    """channel_mean_map reuses input_stage's channel means only for the live tensor they came
    from: an in-place refill (version bump) or a new tensor at a freed input's address recomputes."""
    torch.manual_seed(14)
    x = torch.rand(2, 6, 8, 8, device=DEV)
    _, cm = O.input_stage(x, torch.bfloat16)
    assert O.channel_mean_map(x) is cm
    torch.testing.assert_close(cm, x.mean(1))
    x.copy_(torch.rand_like(x))  # same storage, new contents
    torch.testing.assert_close(O.channel_mean_map(x), x.mean(1))
    ptr = x.data_ptr()
    O.input_stage(x, torch.bfloat16)
    del x
    y = torch.rand(2, 6, 8, 8, device=DEV)  # may land on the freed block
    torch.testing.assert_close(O.channel_mean_map(y), y.mean(1))
    assert ptr is not None


# the persistent 256x256 form's flat K-step stream (k_conv_fwd_ps): one step staged under the current
# step's MFMAs, one more ahead of every tile's epilogue stores. Shapes with 1 (K = 64), 2, 4 and 8 K-steps
# per tile, 2..3 tiles per block, an M tail (the statistics epilogue with row masks) and the bias +
# activation epilogue; the form is asserted from the launch record (dmf_conv_last_form)
PS_CASES = [
    # (N, Cin, H, W, Cout, bias+act epilogue)
    (33, 64, 64, 64, 256, False),
    (33, 128, 32, 32, 512, False),
    (35, 256, 31, 31, 1024, False),
    (34, 512, 32, 32, 1024, False),
    (33, 64, 64, 64, 256, True),
    (35, 256, 31, 31, 512, True),
]


@pytest.mark.parametrize("case", PS_CASES)
def test_conv_ps_stream_forward(case):
    import dmf_native as N

    n, ci, h, w, co, with_bias = case
    torch.manual_seed(9)
    conv = nn.Conv2d(ci, co, 1, bias=with_bias)
    a = torch.randn(n, ci, h, w).bfloat16().float()
    wq = conv.weight.detach().bfloat16().float()
    cd = copy.deepcopy(conv).to(DEV)
    xd = _to_dev(a, torch.bfloat16)
    if with_bias:
        ref = F.relu(F.conv2d(a.double(), wq.double(), conv.bias.detach().double())).float()
        with torch.no_grad():
            y = O.conv2d(xd, cd, (O.WeightCache(), O.WeightCache()), act="relu")
        assert N.FORMS[N.load().dmf_conv_last_form()] == "ps"
        err = (y.float().cpu() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), err
        return
    bn = nn.BatchNorm2d(co)
    with torch.no_grad():
        raw = F.conv2d(a.double(), wq.double()).float()
        ref = F.relu(bn(raw))
    bd = nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        with O.bn_scope(cd, DEV):  # the training forward's statistics arena (dmf_conv2d_fwd_acc)
            y = O.conv_bn_act(xd, cd, (O.WeightCache(), O.WeightCache()), bd, "relu")
    assert N.FORMS[N.load().dmf_conv_last_form()] == "ps"
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 3e-2 * ref.abs().max().item(), err
    assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=1e-2, atol=1e-3 * raw.abs().max().item())
    assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=2e-2, atol=1e-3)


@pytest.mark.parametrize("act", ["relu", "bn"])
def test_conv_ps_nontemporal_stores_bitwise(act):
    """knob conv_nt_store_mb (dmf_conv_tune 16): the persistent form's output stores go out nontemporal
    for outputs of >= that many MiB (default 100: the 512 -> 2048 expansions at B = 32). Threshold 1 here
    (a 32 MiB output) against 0: the same bits, the same BN statistics."""
    import dmf_native as N

    torch.manual_seed(10)
    conv = nn.Conv2d(256, 1024, 1, bias=act == "relu").to(DEV)
    x = _to_dev(torch.randn(16, 256, 32, 32), torch.bfloat16)  # 256 tiles: the persistent form
    outs = []
    for mb in (0, 1):
        O.set_knobs(conv_nt_store_mb=mb)
        try:
            with torch.no_grad():
                if act == "relu":
                    y = O.conv2d(x, conv, (O.WeightCache(), O.WeightCache()), act="relu")
                    rm = None
                else:
                    bd = nn.BatchNorm2d(1024).to(DEV)
                    with O.bn_scope(conv, DEV):
                        y = O.conv_bn_act(x, conv, (O.WeightCache(), O.WeightCache()), bd, "relu")
                    rm = bd.running_mean.clone()
            assert N.FORMS[N.load().dmf_conv_last_form()] == "ps"
            torch.cuda.synchronize()
            outs.append((y.clone(), rm))
        finally:
            O.set_knobs(conv_nt_store_mb=100)
    assert torch.equal(outs[0][0], outs[1][0])
    if act == "bn":
        assert torch.equal(outs[0][1], outs[1][1])


# the 256x256 LDS-DMA weight-gradient tile (dmf_conv_wgrad_tune key 3, knob "wgrad_sq", default 1 = weights
# of >= 2^18 entries) forced on (2) and off (0), so both forms stay covered: Cout and
# KH*KW*Cin multiples of 256, its own pixel split count; a dual-source input (the neck's concat)
SQ_WGRAD_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, dil, Cin2)
    (8, 256, 32, 32, 256, 3, 1, 2, 2, 0),
    (9, 512, 32, 32, 512, 1, 1, 0, 1, 0),
    (16, 2048, 16, 16, 512, 1, 1, 0, 1, 0),
    (4, 256, 32, 32, 256, 3, 1, 1, 1, 256),
    (5, 256, 31, 33, 768, 1, 1, 0, 1, 0),
    # small weights, many pixel splits: the split-lane reducers (k_wgrad_reduce_sl<16> at >= 64 splits,
    # <4> at >= 16)
    (8, 64, 64, 64, 64, 1, 1, 0, 1, 0),
    (8, 128, 32, 32, 256, 1, 1, 0, 1, 0),
    (6, 64, 40, 40, 64, 3, 1, 1, 1, 0),
]


@pytest.mark.parametrize("sq", [0, 2])  # the 128-wide forms / the 256x256 tile wherever legal
@pytest.mark.parametrize("case", SQ_WGRAD_CASES)
def test_conv_wgrad_sq_bf16(case, sq):
    O.set_knobs(wgrad_sq=sq)
    try:
        n, ci, h, w, co, k, s, p, d, ci2 = case
        torch.manual_seed(7)
        q = lambda t: t.bfloat16().float()  # noqa: E731
        a = q(torch.randn(n, ci, h, w))
        b = q(torch.randn(n, ci2, h, w)) if ci2 else None
        conv = nn.Conv2d(ci + ci2, co, k, stride=s, padding=p, dilation=d, bias=False)
        wq = q(conv.weight.detach())
        xin = (torch.cat([a, b], 1) if ci2 else a).double()
        yr = F.conv2d(xin, wq.double(), None, s, p, d)
        gy = q(torch.randn(yr.shape))
        ref_dw = torch.nn.grad.conv2d_weight(xin, wq.shape, gy.double(), s, p, d).float()
        cd = copy.deepcopy(conv).to(DEV)
        with torch.no_grad():
            cd.weight.copy_(wq)
        _, dw, _ = O._conv_backward(_to_dev(a, torch.bfloat16), cd.weight, None, O.ConvGeom(cd),
                                    (O.WeightCache(), O.WeightCache()), _to_dev(gy, torch.bfloat16), False, True, False,
                                    x2=_to_dev(b, torch.bfloat16) if ci2 else None)
        err = (dw.cpu() - ref_dw).abs().max().item()
        assert err <= 1e-3 * ref_dw.abs().max().item(), err
    finally:
        O.set_knobs(wgrad_sq=1)


# the fp16 compute dtype ("16-mixed" = IEEE half activations / MFMA operands, fp32 accumulation): every
# forward body on its own shape (form asserted from the launch record), BN statistics into the arena,
# against fp32 on the same half-rounded operands; plus the weight gradient and the stride-1 dgrad
F16_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad, dil, form)
    (33, 64, 64, 64, 256, 1, 1, 0, 1, "ps"),
    (34, 2048, 32, 32, 512, 1, 1, 0, 1, "pp"),
    (64, 256, 32, 32, 256, 3, 1, 2, 2, "pp"),
    (33, 256, 32, 32, 256, 3, 1, 1, 1, "wide"),
    (4, 64, 16, 16, 128, 3, 1, 1, 1, "buf"),
    (4, 16, 256, 256, 64, 7, 2, 3, 1, "stem"),
    (3, 24, 17, 19, 40, 3, 2, 1, 1, "igemm"),
]


@pytest.mark.parametrize("case", F16_CASES)
def test_conv_f16_forms_forward_and_bn_stats(case):
    import dmf_native as N

    n, ci, h, w, co, k, s, p, d, form = case
    torch.manual_seed(13)
    conv = nn.Conv2d(ci, co, k, stride=s, padding=p, dilation=d, bias=False)
    a = torch.rand(n, ci, h, w).half().float() if form == "stem" else torch.randn(n, ci, h, w).half().float()
    wq = conv.weight.detach().half().float()
    bn = nn.BatchNorm2d(co)
    with torch.no_grad():
        raw = F.conv2d(a, wq, None, s, p, d)  # fp32 accumulation: far inside the half tolerance
        ref = F.relu(bn(raw))
    cd, bd = copy.deepcopy(conv).to(DEV), nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        cd.weight.copy_(wq)
        with O.bn_scope(cd, DEV):
            y = O.conv_bn_act(_to_dev(a, torch.float16), cd, (O.WeightCache(), O.WeightCache()), bd, "relu")
    assert y.dtype == torch.float16
    assert N.FORMS[N.load().dmf_conv_last_form()] == form
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    assert torch.allclose(bd.running_mean.cpu(), bn.running_mean, rtol=2e-3, atol=2e-4 * raw.abs().max().item())
    assert torch.allclose(bd.running_var.cpu(), bn.running_var, rtol=4e-3, atol=1e-4)


@pytest.mark.parametrize("case", BWD_CASES[:5])
def test_conv_backward_f16(case):
    n, ci, h, w, co, k, s, p, d, ci2 = case
    torch.manual_seed(6)
    q = lambda t: t.half().float()  # noqa: E731
    a = q(torch.randn(n, ci, h, w))
    b = q(torch.randn(n, ci2, h, w)) if ci2 else None
    conv = nn.Conv2d(ci + ci2, co, k, stride=s, padding=p, dilation=d, bias=False)
    wq = q(conv.weight.detach())
    xin = (torch.cat([a, b], 1) if ci2 else a).double().requires_grad_(True)
    wr = wq.double().requires_grad_(True)
    yr = F.conv2d(xin, wr, None, s, p, d)
    gy = q(torch.randn(yr.shape))
    yr.backward(gy.double())
    cd = copy.deepcopy(conv).to(DEV)
    with torch.no_grad():
        cd.weight.copy_(wq)
    dx, dw, _ = O._conv_backward(_to_dev(a, torch.float16), cd.weight, None, O.ConvGeom(cd),
                                 (O.WeightCache(), O.WeightCache()), _to_dev(gy, torch.float16), True, True, False,
                                 x2=_to_dev(b, torch.float16) if ci2 else None)
    if ci2:
        dx = torch.cat([dx[0].float(), dx[1].float()], 1)
    ref_dx, ref_dw = xin.grad.float(), wr.grad.float()
    assert dx.dtype in (torch.float16, torch.float32)
    err_x = (dx.float().cpu() - ref_dx).abs().max().item()
    assert err_x <= 2e-3 * ref_dx.abs().max().item(), err_x
    err_w = (dw.cpu() - ref_dw).abs().max().item()
    assert err_w <= 1e-3 * ref_dw.abs().max().item(), err_w


# fp32 GEMM (dmf_sgemm, 64x64 tiles with the ordered split-K reduce where the workspace is given): every
# transpose, alpha, an accumulating beta, bias and activation, against float64 torch on the same operands
SGEMM_CASES = [
    # (tA, tB, M, N, K, beta, bias, act)
    (0, 1, 512, 128, 128, 0.0, True, "none"),
    (0, 0, 512, 128, 384, 0.0, False, "relu"),
    (1, 0, 384, 128, 512, 1.0, False, "none"),
    (1, 1, 70, 45, 600, 0.5, True, "gelu"),
    (0, 1, 32, 4, 512, 0.0, True, "none"),
    (0, 0, 33, 129, 1100, 0.0, False, "sigmoid"),
    (0, 1, 2048, 512, 256, 0.0, True, "none"),
]


@pytest.mark.parametrize("case", SGEMM_CASES)
def test_sgemm_forms(case):
    tA, tB, M, N_, K, beta, with_bias, act = case
    g = torch.Generator().manual_seed(5)
    A = torch.randn((K, M) if tA else (M, K), generator=g)
    B = torch.randn((N_, K) if tB else (K, N_), generator=g)
    C0 = torch.randn(M, N_, generator=g)
    bias = torch.randn(N_, generator=g) if with_bias else None
    ref = 0.75 * ((A.t() if tA else A).double() @ (B.t() if tB else B).double()) + beta * C0.double()
    if bias is not None:
        ref = ref + bias.double()
    ref = {"none": ref, "relu": torch.relu(ref), "gelu": F.gelu(ref), "sigmoid": torch.sigmoid(ref)}[act]
    Ad, Bd, Cd = A.to(DEV), B.to(DEV), C0.clone().to(DEV)
    bd = bias.to(DEV) if bias is not None else None
    O._sgemm(tA, tB, M, N_, K, 0.75, Ad.data_ptr(), Ad.shape[1], Bd.data_ptr(), Bd.shape[1], beta, Cd.data_ptr(),
             N_, O._p(bd), O.ACT[act], O._stream())
    torch.cuda.synchronize()
    err = (Cd.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()) * (K / 128) ** 0.5, err
