"""GPU: the fused attention forward (dmf_flash_attn_fwd, csrc/attn.hip) of a
block that builds no autograd graph (transformer_model.py:100-116): against a
float64 restatement of softmax(q k^T / sqrt(d)) v with key padding, against the
unfused path it replaces (QK^T GEMM -> k_softmax_drop -> PV GEMM) with the same
Philox dropout masks, and the whole forward-only TransformerBlock
(dmf_tokens._block_fwd_nograd: the conv-engine qkv linear, the fused attention,
no backward copies) against the autograd block's forward."""
import copy

import pytest
import torch

import dmf_native as N
import dmf_ops as O
import dmf_tokens as D

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _qkv(b, n, e, seed=0):
    torch.manual_seed(seed)
    return (torch.randn(b * n, 3 * e, device=DEV) * 1.5).bfloat16()


def _ref64(qkv, b, n, nv, e, heads):
    d = e // heads
    x = qkv.double().view(b, n, 3, heads, d)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = q @ k.transpose(-1, -2) * d ** -0.5
    s[..., nv:] = float("-inf")
    return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(b * n, e)


@pytest.mark.parametrize("b,n,nv,heads", [(2, 576, 576, 4), (3, 264, 257, 4), (1, 100, 100, 2), (2, 64, 40, 6)])
def test_flash_attention_vs_float64(b, n, nv, heads):
    e = 128 * heads
    qkv = _qkv(b, n, e)
    o = D.flash_attention(qkv, b, n, nv, e, heads, 0.0, None, 0)
    torch.cuda.synchronize()
    ref = _ref64(qkv, b, n, nv, e, heads)
    err = (o.double() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


def _unfused(qkv, b, n, nv, e, heads, p, rng, site):
    d = e // heads
    S = torch.empty((b, heads, n, n), dtype=torch.float32, device=DEV)
    D.gemm(S, qkv, qkv, n, n, d, lda=3 * e, ldb=3 * e, ldc=n, batch=(b, heads), sa=(n * 3 * e, d),
           sb=(n * 3 * e, d), sc=(heads * n * n, n * n), b_off=e)
    P = torch.empty((b, heads, n, n), dtype=torch.bfloat16, device=DEV)
    Pd = torch.empty_like(P)
    N.call("dmf_softmax_dropout", S.data_ptr(), n, b * heads * n, n, nv, float(d ** -0.5), float(p), O._p(rng),
           site, P.data_ptr(), Pd.data_ptr(), n, O._stream())
    o = torch.empty((b * n, e), dtype=torch.bfloat16, device=DEV)
    D.gemm(o, Pd, qkv, n, d, n, tb=1, lda=n, ldb=3 * e, ldc=e, batch=(b, heads), sa=(heads * n * n, n * n),
           sb=(n * 3 * e, d), sc=(n * e, d), b_off=2 * e)
    return o


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention_matches_unfused_with_dropout(p):
    """Same Philox masks (element ((b*h + head)*n + query)*n + key) as k_softmax_drop: the outputs
    agree to the bf16 rounding of the probabilities."""
    b, n, nv, heads, e = 4, 576, 570, 4, 512
    qkv = _qkv(b, n, e, seed=1)
    rng = torch.tensor([0x1234_5678_9ABC, 77], dtype=torch.int64, device=DEV)
    o1 = D.flash_attention(qkv, b, n, nv, e, heads, p, rng, 5)
    o2 = _unfused(qkv, b, n, nv, e, heads, p, rng, 5)
    torch.cuda.synchronize()
    scale = o2.float().abs().max().item()
    err = (o1.float() - o2.float()).abs().max().item()
    assert err <= 1.5e-2 * scale, (err, scale)
    if p > 0:
        # a different site draws different masks: the outputs must move well past that bound
        o3 = D.flash_attention(qkv, b, n, nv, e, heads, p, rng, 6)
        assert (o3.float() - o2.float()).abs().max().item() > 5e-2 * scale


def test_flash_attention_refuses_dropout_at_unaligned_n():
    """the dropout masks are drawn 4 elements per Philox block, so the launcher refuses
    p > 0 when n % 4 != 0 (a loud error, not correlated masks); p = 0 at the same n still runs."""
    b, n, heads = 1, 102, 2
    e = 128 * heads
    qkv = _qkv(b, n, e, seed=3)
    rng = torch.tensor([0x1234_5678_9ABC, 77], dtype=torch.int64, device=DEV)
    with pytest.raises(RuntimeError, match="n % 4"):
        D.flash_attention(qkv, b, n, n, e, heads, 0.1, rng, 0)
    o = D.flash_attention(qkv, b, n, n, e, heads, 0.0, None, 0)
    torch.cuda.synchronize()
    ref = _ref64(qkv, b, n, n, e, heads)
    assert (o.double() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


def test_forward_only_block_matches_autograd_forward():
    """dmf_tokens.transformer_block with no grad (the conv-engine qkv, the fused attention, no backward
    copies) against the same block's autograd forward (train mode: dropout on, same rng snapshot)."""
    import transformer_model as TM

    torch.manual_seed(3)
    blk = TM.TransformerBlock(512, heads=4).to(DEV).train()
    with torch.no_grad():
        blk.gamma1.fill_(0.5)
        blk.gamma2.fill_(0.7)
    x = torch.randn(4, 576, 512, device=DEV)
    rng = O.RNG.snapshot(torch.device(DEV))
    with torch.no_grad():
        y_fused = D.transformer_block(x, blk, rng, blk._sites, torch.bfloat16)
    prev = D.FWD_FUSED
    D.FWD_FUSED = False
    try:
        with torch.no_grad():
            y_ref = D.transformer_block(x, blk, rng, blk._sites, torch.bfloat16)
    finally:
        D.FWD_FUSED = prev
    torch.cuda.synchronize()
    d = (y_fused - y_ref).abs().max().item()
    assert d <= 2e-2 * y_ref.abs().max().item(), d
    # and the path really is the fused one
    recs = []
    O.PROBE["tok_gemm"] = recs
    try:
        with torch.no_grad():
            D.transformer_block(x, blk, rng, blk._sites, torch.bfloat16)
    finally:
        O.PROBE["tok_gemm"] = None
    names = [r["fn"] for r in recs]
    assert "dmf_flash_attn_fwd" in names and any(n.startswith("dmf_conv2d") for n in names), names


def test_fc1_dropout_on_conv_engine_matches_token_gemm():
    """fc1 -> GELU -> dropout of a forward-only block on the conv engine (dmf_conv2d_fwd_drop, persistent
    1x1 form, packed GELU) against the token GEMM's epilogue (k_gemm_bf16) with the same rng and site:
    identical keep masks (element row * Nout + col), values within bf16 rounding."""
    torch.manual_seed(4)
    b, n, e, hid, p, site = 32, 576, 512, 2048, 0.1, 5  # config 5's B = 32: the persistent plan's tile count
    lin = torch.nn.Linear(e, hid).to(DEV)
    x = torch.randn(b * n, e, device=DEV).bfloat16()
    rng = O.RNG.snapshot(torch.device(DEV))
    assert D._linear_conv_drop_ok(x, lin, n)
    with torch.no_grad():
        yc = D._linear_conv_drop(x, lin, b, n, p, rng, site)
        (w1,) = D._wcast(torch.bfloat16, lin.weight)
        yg = D.gemm(torch.empty((b * n, hid), dtype=torch.bfloat16, device=DEV), x, w1, b * n, hid, e, lda=e, ldb=e,
                    ldc=hid, bias=lin.bias, act="gelu", dropout_p=p, rng=rng, site=site)
    torch.cuda.synchronize()
    dropped_c, dropped_g = yc == 0, yg == 0
    frac = dropped_g.float().mean().item()
    assert 0.08 < frac < 0.12, frac
    assert (dropped_c != dropped_g).float().mean().item() < 1e-4  # (a GELU output that is exactly 0 aside)
    d = (yc.float() - yg.float()).abs().max().item()
    assert d <= 2e-2 * yg.float().abs().max().item(), d


@pytest.mark.parametrize("hid,p", [(512, 0.0), (512, 0.1), (2048, 0.1)])
def test_proj_fc2_residual_on_conv_engine_matches_token_gemm(hid, p):
    """proj (K = E) / fc2 (K = 4E) of a forward-only block on the conv engine (dmf_conv2d_fwd_tokres: + bias,
    dropout, x LayerScale, + the f32 residual stream, f32 out) against k_gemm_bf16's epilogue with the same rng
    and site: identical keep masks (a dropped element equals its residual exactly), values within the bf16
    operands' accumulation-order differences. Config 5's B = 32 inside the two-encoder fork's tile threshold
    (O.concurrent_tiles), where the production forward takes this form."""
    torch.manual_seed(6 + hid)
    b, n, e, site = 32, 576, 512, 9
    lin = torch.nn.Linear(hid, e).to(DEV)
    x = torch.randn(b * n, hid, device=DEV).bfloat16()
    res = torch.randn(b * n, e, device=DEV)
    gamma = torch.rand(e, device=DEV) + 0.5
    rng = O.RNG.snapshot(torch.device(DEV))
    O.concurrent_tiles(True)
    try:
        assert D._linear_conv_tokres_ok(x, lin, n, res)
        with torch.no_grad():
            yc = D._linear_conv_tokres(x, lin, b, n, gamma, res, p, rng, site)
    finally:
        O.concurrent_tiles(False)
    with torch.no_grad():
        (w,) = D._wcast(torch.bfloat16, lin.weight)
        yg = D.gemm(torch.empty((b * n, e), dtype=torch.float32, device=DEV), x, w, b * n, e, hid, lda=hid, ldb=hid,
                    ldc=e, bias=lin.bias, colscale=gamma, res=res, dropout_p=p, rng=rng, site=site)
    torch.cuda.synchronize()
    assert not D._linear_conv_tokres_ok(x, lin, n, res)  # single-stream threshold: the GEMM path
    if p > 0:
        dc, dg = yc == res, yg == res
        frac = dg.float().mean().item()
        assert 0.08 < frac < 0.12, frac
        assert torch.equal(dc, dg)
    scale = (yg - res).abs().max().item()
    d = (yc - yg).abs().max().item()
    assert d <= 2e-3 * scale, (d, scale)


def test_token_probe_replays_the_fork_sizing():
    """bench.py's token-GEMM probe replays the recorded launches through the C-ABI: a proj / fc2 launch
    recorded inside the two-encoder fork (half-chip tile sizing, the only sizing at which its persistent
    form applies at B = 32) must be replayed at that sizing (probe_replay as_recorded) -- replayed at the
    single-stream sizing the launcher refuses it."""
    torch.manual_seed(7)
    b, n, e, hid = 32, 576, 512, 2048
    lin = torch.nn.Linear(hid, e).to(DEV)
    x = torch.randn(b * n, hid, device=DEV).bfloat16()
    res = torch.randn(b * n, e, device=DEV)
    gamma = torch.rand(e, device=DEV) + 0.5
    rng = O.RNG.snapshot(torch.device(DEV))
    recs = []
    O.PROBE["tok_gemm"] = recs
    O.concurrent_tiles(True)
    try:
        with torch.no_grad():
            D._linear_conv_tokres(x, lin, b, n, gamma, res, 0.1, rng, 9)
    finally:
        O.concurrent_tiles(False)
        O.PROBE["tok_gemm"] = None
    assert [r["fn"] for r in recs] == ["dmf_conv2d_fwd_tokres"] and recs[0]["tiles"] == O.CONC_MIN_TILES
    ms, per = O.probe_replay(recs, as_recorded=True)
    assert ms > 0 and len(per) == 1
    with pytest.raises(RuntimeError, match="persistent 1x1"):
        O.probe_replay(recs)
