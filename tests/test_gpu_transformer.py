"""Configuration 5 (hybrid TransformerStage, transformer_model.py:7-175):
the bf16 MFMA GEMM with its fused epilogues, softmax+dropout, the token
LayerNorm / LayerScale-dropout kernels, one TransformerBlock forward+backward
(eval mode against the CPU oracle; train mode with dropout against a torch
fp32 restatement that uses the library's own Philox keep-masks), and the
hybrid encoder end to end.

Tolerances, as max|ours - ref| <= tol * max(1, max|ref|): bf16 operands
(fp32 accumulation) 2e-2 for single GEMMs and 3e-2 for a whole block /
gradient; the f32 parity mode (dmf_gemm_f32 on the 16x16x4 f32 MFMA, f32
probabilities and saved activations) 1e-5 for a GEMM and 1e-4 for a block,
its gradients and the standalone attention / MLP modules."""
import copy

import pytest
import torch
import torch.nn.functional as F

import dmf_native as N
import dmf_ops as O
import dmf_tokens as D
import model_module as MM
import parameters as PR
import transformer_model as TM
from oracle import model as OM

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(x):
    return x.to(torch.bfloat16).float()


def _close(a, b, tol, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), f"{what}: max err {err:.3e} (ref max {b.abs().max():.3e})"


GEMM_CASES = [
    # (ta, tb, M, N, K, out dtype)
    (0, 0, 200, 136, 72, torch.float32),
    (0, 1, 256, 128, 96, torch.bfloat16),
    (1, 0, 136, 264, 48, torch.float32),
    (1, 1, 64, 72, 520, torch.float32),
    (0, 0, 1030, 512, 512, torch.bfloat16),
]


@pytest.mark.parametrize("case", GEMM_CASES)
def test_gemm_bf16_plain(case):
    ta, tb, M, Nn, K, odt = case
    g = torch.Generator().manual_seed(M + Nn + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((K, Nn) if tb else (Nn, K), generator=g)
    bias = torch.randn(Nn, generator=g)
    ref = (_bf(A).t() if ta else _bf(A)) @ (_bf(B) if tb else _bf(B).t()) + bias
    Ad, Bd = A.to(DEV, torch.bfloat16), B.to(DEV, torch.bfloat16)
    C = torch.empty((M, Nn), dtype=odt, device=DEV)
    D.gemm(C, Ad, Bd, M, Nn, K, ta=ta, tb=tb, lda=A.shape[1], ldb=B.shape[1], ldc=Nn, bias=bias.to(DEV))
    _close(C, ref, 1e-2, "gemm")


@pytest.mark.parametrize("case", GEMM_CASES)
def test_gemm_f32_plain(case):
    ta, tb, M, Nn, K, odt = case
    g = torch.Generator().manual_seed(M + Nn + K + 1)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((K, Nn) if tb else (Nn, K), generator=g)
    bias = torch.randn(Nn, generator=g)
    ref = (A.double().t() if ta else A.double()) @ (B.double() if tb else B.double().t()) + bias.double()
    C = torch.empty((M, Nn), dtype=odt, device=DEV)
    D.gemm(C, A.to(DEV), B.to(DEV), M, Nn, K, ta=ta, tb=tb, lda=A.shape[1], ldb=B.shape[1], ldc=Nn,
           bias=bias.to(DEV))
    _close(C, ref, 1e-5 if odt == torch.float32 else 1e-2, "gemm f32")


def test_gemm_f32_epilogues_and_attention_layout():
    """f32 operands through the aux / gelu / gradient epilogues and the
    head-sliced batched layout (Q K^T and P V) against float64."""
    M, Nn, K, p = 96, 256, 64, 0.25
    g = torch.Generator().manual_seed(12)
    A, W, bias = torch.randn(M, K, generator=g), torch.randn(Nn, K, generator=g) * 0.2, torch.randn(Nn, generator=g)
    rng = O.RNG.snapshot(DEV)
    site = O.RNG.new_site()
    keep = torch.empty(M * Nn, dtype=torch.uint8, device=DEV)
    N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, M * Nn, p, keep.data_ptr(), N.stream_ptr())
    mk = keep.cpu().double().view(M, Nn) / (1 - p)
    aux = torch.empty((M, Nn), device=DEV)
    out = torch.empty((M, Nn), device=DEV)
    D.gemm(out, A.to(DEV), W.to(DEV), M, Nn, K, lda=K, ldb=K, ldc=Nn, bias=bias.to(DEV), act="gelu", aux=aux,
           dropout_p=p, rng=rng, site=site)
    pre = A.double() @ W.double().t() + bias.double()
    _close(aux, pre, 1e-5, "aux f32")
    _close(out, F.gelu(pre) * mk, 1e-5, "gelu+dropout f32")
    dh, W2 = torch.randn(M, 128, generator=g), torch.randn(128, Nn, generator=g) * 0.1
    dpre = torch.empty((M, Nn), device=DEV)
    dbias = torch.zeros(Nn, device=DEV)
    D.gemm(dpre, dh.to(DEV), W2.to(DEV), M, Nn, 128, tb=1, lda=128, ldb=Nn, ldc=Nn, act="gelu", pre=aux,
           dropout_p=p, rng=rng, site=site, dbias=dbias)
    x_ = pre.clone().requires_grad_(True)
    F.gelu(x_).backward(torch.ones_like(x_))
    ref = (dh.double() @ W2.double()) * mk * x_.grad
    _close(dpre, ref, 1e-5, "grad epilogue f32")
    _close(dbias, ref.sum(0), 1e-5, "dbias f32")
    b, h, n, d = 2, 4, 40, 64
    e = h * d
    qkv = torch.randn(b, n, 3 * e, generator=g)
    qd = qkv.to(DEV)
    S = torch.empty((b, h, n, n), device=DEV)
    D.gemm(S, qd, qd, n, n, d, lda=3 * e, ldb=3 * e, ldc=n, batch=(b, h), sa=(n * 3 * e, d), sb=(n * 3 * e, d),
           sc=(h * n * n, n * n), b_off=e)
    q = qkv[..., :e].double().view(b, n, h, d).transpose(1, 2)
    k = qkv[..., e:2 * e].double().view(b, n, h, d).transpose(1, 2)
    _close(S, q @ k.transpose(-1, -2), 1e-5, "QK^T f32")
    P = torch.softmax(torch.randn(b, h, n, n, generator=g), -1)
    o = torch.zeros((b * n, e), device=DEV)
    D.gemm(o, P.to(DEV), qd, n, d, n, tb=1, lda=n, ldb=3 * e, ldc=e, batch=(b, h), sa=(h * n * n, n * n),
           sb=(n * 3 * e, d), sc=(n * e, d), b_off=2 * e)
    v = qkv[..., 2 * e:].double().view(b, n, h, d).transpose(1, 2)
    _close(o, (P.double() @ v).transpose(1, 2).reshape(b * n, e), 1e-5, "PV f32")


def test_gemm_bf16_batched_offsets():
    """attention-style operands: heads are column slices of packed rows"""
    b, h, n, d = 2, 3, 40, 16
    g = torch.Generator().manual_seed(1)
    qkv = torch.randn(b, n, 3 * h * d, generator=g)
    e = h * d
    S = torch.empty((b, h, n, n), device=DEV)
    qd = qkv.to(DEV, torch.bfloat16)
    D.gemm(S, qd, qd, n, n, d, lda=3 * e, ldb=3 * e, ldc=n, batch=(b, h), sa=(n * 3 * e, d), sb=(n * 3 * e, d),
           sc=(h * n * n, n * n), b_off=e)
    q = _bf(qkv[..., :e]).view(b, n, h, d).transpose(1, 2)
    k = _bf(qkv[..., e:2 * e]).view(b, n, h, d).transpose(1, 2)
    _close(S, q @ k.transpose(-1, -2), 1e-2, "QK^T")
    # P V with V^T-free layout (tb=1) into a column slice
    P = torch.softmax(torch.randn(b, h, n, n, generator=g), -1)
    o = torch.zeros((b * n, e), dtype=torch.bfloat16, device=DEV)
    D.gemm(o, P.to(DEV, torch.bfloat16), qd, n, d, n, tb=1, lda=n, ldb=3 * e, ldc=e, batch=(b, h),
           sa=(h * n * n, n * n), sb=(n * 3 * e, d), sc=(n * e, d), b_off=2 * e)
    v = _bf(qkv[..., 2 * e:]).view(b, n, h, d).transpose(1, 2)
    ref = (_bf(P) @ v).transpose(1, 2).reshape(b * n, e)
    _close(o, ref, 1e-2, "PV")


def test_gemm_epilogues():
    """aux + gelu + dropout forward, its gradient epilogue with dbias, and
    LayerScale + residual (f32) -- masks from dmf_dropout_keep_mask"""
    M, Nn, K, p = 96, 256, 64, 0.25
    g = torch.Generator().manual_seed(2)
    A, W, bias = torch.randn(M, K, generator=g), torch.randn(Nn, K, generator=g) * 0.2, torch.randn(Nn, generator=g)
    rng = O.RNG.snapshot(DEV)
    site = O.RNG.new_site()
    keep = torch.empty(M * Nn, dtype=torch.uint8, device=DEV)
    N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, M * Nn, p, keep.data_ptr(), N.stream_ptr())
    mk = keep.cpu().float().view(M, Nn) / (1 - p)
    Ad, Wd = A.to(DEV, torch.bfloat16), W.to(DEV, torch.bfloat16)
    aux = torch.empty((M, Nn), dtype=torch.bfloat16, device=DEV)
    out = torch.empty((M, Nn), dtype=torch.bfloat16, device=DEV)
    D.gemm(out, Ad, Wd, M, Nn, K, lda=K, ldb=K, ldc=Nn, bias=bias.to(DEV), act="gelu", aux=aux, dropout_p=p,
           rng=rng, site=site)
    pre = _bf(A) @ _bf(W).t() + bias
    _close(aux, pre, 1e-2, "aux")
    _close(out, F.gelu(pre) * mk, 2e-2, "gelu+dropout")
    # gradient epilogue: dpre = mask(dh) * gelu'(pre), dbias = colsum(dpre)
    dh = torch.randn(M, 128, generator=g)
    W2 = torch.randn(128, Nn, generator=g) * 0.1   # dh @ W2 -> [M, Nn]  (tb=1 on W2 [128][Nn])
    dpre = torch.empty((M, Nn), dtype=torch.bfloat16, device=DEV)
    dbias = torch.zeros(Nn, device=DEV)
    D.gemm(dpre, dh.to(DEV, torch.bfloat16), W2.to(DEV, torch.bfloat16), M, Nn, 128, tb=1, lda=128, ldb=Nn, ldc=Nn,
           act="gelu", pre=aux, dropout_p=p, rng=rng, site=site, dbias=dbias)
    pre_b = _bf(pre)
    x_ = pre_b.clone().requires_grad_(True)
    F.gelu(x_).backward(torch.ones_like(x_))
    ref = (_bf(dh) @ _bf(W2)) * mk * x_.grad
    _close(dpre, ref, 2e-2, "grad epilogue")
    _close(dbias, ref.sum(0), 2e-2, "dbias")
    # LayerScale + residual into f32
    res = torch.randn(M, Nn, generator=g)
    gam = torch.rand(Nn, generator=g)
    out32 = torch.empty((M, Nn), device=DEV)
    D.gemm(out32, Ad, Wd, M, Nn, K, lda=K, ldb=K, ldc=Nn, bias=bias.to(DEV), colscale=gam.to(DEV), res=res.to(DEV))
    _close(out32, res + pre * gam, 1e-2, "layerscale residual")


def test_softmax_dropout_fwd_bwd():
    rows, L, p, scale = 300, 72, 0.2, 0.125
    g = torch.Generator().manual_seed(3)
    S = torch.randn(rows, L, generator=g) * 4
    rng = O.RNG.snapshot(DEV)
    site = O.RNG.new_site()
    Sd = S.to(DEV)
    P = torch.empty((rows, L), dtype=torch.bfloat16, device=DEV)
    Pd = torch.empty_like(P)
    N.call("dmf_softmax_dropout", Sd.data_ptr(), L, rows, L, L, scale, p, rng.data_ptr(), site, P.data_ptr(),
           Pd.data_ptr(), L, N.stream_ptr())
    keep = torch.empty(rows * L, dtype=torch.uint8, device=DEV)
    N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, rows * L, p, keep.data_ptr(), N.stream_ptr())
    mk = keep.cpu().float().view(rows, L) / (1 - p)
    ref = torch.softmax(S * scale, -1)
    _close(P, ref, 1e-2, "probs")
    _close(Pd, ref * mk, 1e-2, "dropped probs")
    G = torch.randn(rows, L, generator=g)
    dS = torch.empty((rows, L), dtype=torch.bfloat16, device=DEV)
    N.call("dmf_softmax_dropout_bwd", P.data_ptr(), L, G.to(DEV).data_ptr(), L, rows, L, scale, p, rng.data_ptr(),
           site, dS.data_ptr(), L, N.stream_ptr())
    s_ = S.clone().requires_grad_(True)
    (torch.softmax(s_ * scale, -1) * mk).backward(G)
    _close(dS, s_.grad, 2e-2, "dscores")


def test_token_layernorm_and_scale_dropout():
    R, E, p = 70, 512, 0.3
    g = torch.Generator().manual_seed(4)
    x = torch.randn(R, E, generator=g) * 2 + 0.5
    gam, bet = 1 + 0.1 * torch.randn(E, generator=g), 0.1 * torch.randn(E, generator=g)
    y, save = D.ln_fwd(x.to(DEV), gam.to(DEV), bet.to(DEV), 1e-5, torch.bfloat16)
    xr = x.clone().requires_grad_(True)
    gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (E,), gr, br, 1e-5)
    _close(y, yr, 1e-2, "ln fwd")
    dy = torch.randn(R, E, generator=g)
    dres = torch.randn(R, E, generator=g)
    yr.backward(dy)
    dg, db = torch.zeros(E, device=DEV), torch.zeros(E, device=DEV)
    dx = D.ln_bwd(dy.to(DEV), x.to(DEV), save, gam.to(DEV), dres.to(DEV).clone(), dg, db)
    _close(dx, xr.grad + dres, 1e-3, "ln dx")
    _close(dg, gr.grad, 1e-3, "ln dgamma")
    _close(db, br.grad, 1e-3, "ln dbeta")
    # out = res + drop(y) * gamma  backward
    yb = torch.randn(R, E, generator=g)
    rng = O.RNG.snapshot(DEV)
    site = O.RNG.new_site()
    keep = torch.empty(R * E, dtype=torch.uint8, device=DEV)
    N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, R * E, p, keep.data_ptr(), N.stream_ptr())
    mk = keep.cpu().float().view(R, E) / (1 - p)
    ydev = yb.to(DEV, torch.bfloat16)
    dyo = torch.empty((R, E), dtype=torch.bfloat16, device=DEV)
    dgam, dbias = torch.zeros(E, device=DEV), torch.zeros(E, device=DEV)
    ws = torch.empty(N.load().dmf_tok_bwd_ws_floats(R, E), dtype=torch.float32, device=DEV)
    N.call("dmf_tok_scale_dropout_bwd", dy.to(DEV).data_ptr(), ydev.data_ptr(), R, E, gam.to(DEV).data_ptr(), p,
           rng.data_ptr(), site, dyo.data_ptr(), dgam.data_ptr(), dbias.data_ptr(), ws.data_ptr(), N.stream_ptr())
    _close(dyo, dy * mk * gam, 1e-2, "branch dy")
    _close(dgam, (dy * mk * _bf(yb)).sum(0), 1e-3, "dgamma")
    _close(dbias, (dy * mk * gam).sum(0), 1e-3, "dbias")


def _masked_block_ref(blk, x, masks, p):
    """transformer_model.py:78-134 in fp32 with explicit keep masks (1/(1-p) scaled)."""
    b, n, e = x.shape
    at, ml = blk.attn, blk.mlp
    hh, d = at.num_heads, at.head_dim
    h1 = blk.norm1(x)
    q, k, v = at.qkv(h1).reshape(b, n, 3, hh, d).permute(2, 0, 3, 1, 4)
    a = torch.softmax((q @ k.transpose(-2, -1)) * at.scale, dim=-1) * masks[0]
    y = at.proj((a @ v).transpose(1, 2).reshape(b, n, e)) * masks[1]
    x = x + y * blk.gamma1
    hm = F.gelu(ml.fc1(blk.norm2(x))) * masks[2]
    return x + ml.fc2(hm) * masks[3] * blk.gamma2


def _block_pair(e, heads, seed):
    torch.manual_seed(seed)
    ref = OM.TransformerBlock(e, heads)
    for m in ref.modules():
        if isinstance(m, torch.nn.LayerNorm):
            m.weight.data = 1 + 0.1 * torch.randn(e)
            m.bias.data = 0.1 * torch.randn(e)
    ref.gamma1.data = 0.5 + torch.rand(e)
    ref.gamma2.data = 0.5 + torch.rand(e)
    ours = TM.TransformerBlock(e, heads)
    ours.load_state_dict(ref.state_dict())
    return ours.to(DEV), ref


def _grads(mod):
    return {n: p.grad for n, p in mod.named_parameters()}


def test_block_eval_parity_vs_oracle():
    b, n, e, heads = 2, 64, 256, 4
    ours, ref = _block_pair(e, heads, 5)
    ours.eval()
    ref.eval()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(b, n, e, generator=g)
    gy = torch.randn(b, n, e, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(gy)
    xd = x.to(DEV).requires_grad_(True)
    y = ours(xd)
    y.backward(gy.to(DEV))
    _close(y, yr, 3e-2, "block out")
    _close(xd.grad, xr.grad, 3e-2, "dx")
    gr = _grads(ref)
    for name, gd in _grads(ours).items():
        _close(gd, gr[name], 3e-2, name)


def test_block_train_dropout_vs_masked_restatement():
    b, n, e, heads, p = 2, 48, 256, 4, 0.1
    ours, ref = _block_pair(e, heads, 7)
    ours.train()
    ref.train()
    g = torch.Generator().manual_seed(8)
    x = torch.randn(b, n, e, generator=g)
    gy = torch.randn(b, n, e, generator=g)
    rng = O.RNG.snapshot(DEV)
    hid = ours.mlp.fc1.out_features
    shapes = [(b * heads * n * n, (b, heads, n, n)), (b * n * e, (b, n, e)), (b * n * hid, (b, n, hid)),
              (b * n * e, (b, n, e))]
    masks = []
    for site, (cnt, shp) in zip(ours._sites, shapes):
        keep = torch.empty(cnt, dtype=torch.uint8, device=DEV)
        N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, cnt, p, keep.data_ptr(), N.stream_ptr())
        masks.append(keep.cpu().float().view(shp) / (1 - p))
    xr = x.clone().requires_grad_(True)
    yr = _masked_block_ref(ref, xr, masks, p)
    yr.backward(gy)
    xd = x.to(DEV).requires_grad_(True)
    y = D.transformer_block(xd, ours, rng, ours._sites)
    y.backward(gy.to(DEV))
    _close(y, yr, 3e-2, "block out (dropout)")
    _close(xd.grad, xr.grad, 3e-2, "dx (dropout)")
    gr = _grads(ref)
    for name, gd in _grads(ours).items():
        _close(gd, gr[name], 3e-2, name)
    # same snapshot -> same masks -> same output
    with torch.no_grad():
        y2 = D.transformer_block(x.to(DEV), ours, rng, ours._sites)
    assert torch.equal(y2, y.detach())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [False, True])
def test_block_parity_dtype(dtype, train):
    """The whole block in each compute dtype, eval (vs the oracle) and train
    with dropout (vs the masked restatement on the library's keep-masks)."""
    b, n, e, heads, p = 2, 48, 256, 4, 0.1
    ours, ref = _block_pair(e, heads, 13)
    MM.set_compute_dtype(ours, dtype)
    ours.train(train)
    ref.train(train)
    g = torch.Generator().manual_seed(14)
    x = torch.randn(b, n, e, generator=g)
    gy = torch.randn(b, n, e, generator=g)
    xr = x.clone().requires_grad_(True)
    rng = None
    if train:
        rng = O.RNG.snapshot(DEV)
        hid = ours.mlp.fc1.out_features
        shapes = [(b * heads * n * n, (b, heads, n, n)), (b * n * e, (b, n, e)), (b * n * hid, (b, n, hid)),
                  (b * n * e, (b, n, e))]
        masks = []
        for site, (cnt, shp) in zip(ours._sites, shapes):
            keep = torch.empty(cnt, dtype=torch.uint8, device=DEV)
            N.call("dmf_dropout_keep_mask", rng.data_ptr(), site, cnt, p, keep.data_ptr(), N.stream_ptr())
            masks.append(keep.cpu().float().view(shp) / (1 - p))
        yr = _masked_block_ref(ref, xr, masks, p)
    else:
        yr = ref(xr)
    yr.backward(gy)
    xd = x.to(DEV).requires_grad_(True)
    y = D.transformer_block(xd, ours, rng, ours._sites, dtype) if train else ours(xd)
    y.backward(gy.to(DEV))
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    _close(y, yr, tol, "block out")
    _close(xd.grad, xr.grad, tol, "dx")
    gr = _grads(ref)
    for name, gd in _grads(ours).items():
        _close(gd, gr[name], tol, name)


def _masked_mhsa_ref(at, x, masks):
    b, n, e = x.shape
    q, k, v = at.qkv(x).reshape(b, n, 3, at.num_heads, at.head_dim).permute(2, 0, 3, 1, 4)
    a = torch.softmax((q @ k.transpose(-2, -1)) * at.scale, dim=-1) * masks[0]
    return at.proj((a @ v).transpose(1, 2).reshape(b, n, e)) * masks[1]


def _masked_mlp_ref(ml, x, masks):
    return ml.fc2(F.gelu(ml.fc1(x)) * masks[0]) * masks[1]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_standalone_attention_and_mlp_train_mode(dtype):
    """MultiHeadSelfAttention and MLP used as modules (transformer_model.py
    :83-134) in train mode with their dropouts -- the reference's own
    forwards -- against the masked fp32 restatement; eval against the oracle."""
    b, n, e, heads, p = 2, 56, 256, 4, 0.1
    torch.manual_seed(15)
    ref_at, ref_ml = OM.TransformerBlock(e, heads).attn, OM.TransformerBlock(e, heads).mlp
    at, ml = TM.MultiHeadSelfAttention(e, heads), TM.MLP(e)
    at.load_state_dict(ref_at.state_dict())
    ml.load_state_dict(ref_ml.state_dict())
    at, ml = at.to(DEV), ml.to(DEV)
    for m in (at, ml):
        MM.set_compute_dtype(m, dtype)
    g = torch.Generator().manual_seed(16)
    x = torch.randn(b, n, e, generator=g)
    gy = torch.randn(b, n, e, generator=g)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    for mod, ref, kind in ((at, ref_at, "attn"), (ml, ref_ml, "mlp")):
        hid = e if kind == "attn" else ml.fc1.out_features
        shapes = [(b * heads * n * n, (b, heads, n, n)), (b * n * e, (b, n, e))] if kind == "attn" else \
            [(b * n * hid, (b, n, hid)), (b * n * e, (b, n, e))]
        for train in (False, True):
            mod.train(train)
            ref.train(train)
            for q in mod.parameters():
                q.grad = None
            for q in ref.parameters():
                q.grad = None
            snap = O.RNG.snapshot(DEV) if train else None
            O.RNG_CURRENT[0] = snap
            try:
                xd = x.to(DEV).requires_grad_(True)
                y = mod(xd)
            finally:
                O.RNG_CURRENT[0] = None
            xr = x.clone().requires_grad_(True)
            if train:
                masks = []
                for site, (cnt, shp) in zip(mod._sites, shapes):
                    keep = torch.empty(cnt, dtype=torch.uint8, device=DEV)
                    N.call("dmf_dropout_keep_mask", snap.data_ptr(), site, cnt, p, keep.data_ptr(),
                           N.stream_ptr())
                    masks.append(keep.cpu().float().view(shp) / (1 - p))
                yr = _masked_mhsa_ref(ref, xr, masks) if kind == "attn" else _masked_mlp_ref(ref, xr, masks)
            else:
                yr = ref(xr)
            y.backward(gy.to(DEV))
            yr.backward(gy)
            _close(y, yr, tol, f"{kind} out (train={train})")
            _close(xd.grad, xr.grad, tol, f"{kind} dx (train={train})")
            gr = _grads(ref)
            for name, gd in _grads(mod).items():
                _close(gd, gr[name], tol, f"{kind} {name} (train={train})")


def test_hybrid_encoder_forward_backward():
    """ModelMaskHeadBackbone with use_hybrid_transformer (model_module.py:564-579,
    :701-703) against the oracle, eval mode, all in the f32 parity mode
    (f32 convs + f32 transformer GEMMs): logits within 1e-3."""
    P = PR.small_parameters(channels=(16, 32, 64), input_size=64, dropout=0.0, use_backbone=False)
    mp = P["dwi_model_parameters"]
    mp["use_hybrid_transformer"] = True
    mp["transformer_embed_dim"] = 256
    mp["transformer_depth"] = 2
    mp["transformer_heads"] = 4
    mp["mask_stage"] = "f2"
    torch.manual_seed(9)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", copy.deepcopy(P), None), True)
    ref = OM.ModelMaskHeadBackbone("dwi", copy.deepcopy(P), None)
    ref.load_state_dict(enc.state_dict())
    MM.set_compute_dtype(enc, torch.float32)
    enc = enc.to(DEV).eval()
    ref.eval()
    g = torch.Generator().manual_seed(10)
    x = (0.5 + torch.randn(2, 14, 64, 64, generator=g) / 6).clamp(0, 1)
    lo, aux, mp_ = enc(x.to(DEV))
    lr_, auxr, mpr = ref(x)
    _close(lo, lr_, 1e-3, "logits")
    _close(aux["raw_feats"][2], auxr["raw_feats"][2], 1e-3, "f3")
    (aux["raw_feats"][2].float().square().mean()).backward()
    (auxr["raw_feats"][2].square().mean()).backward()
    gr = dict(ref.named_parameters())
    for name, prm in enc.named_parameters():
        if name.startswith("transformer.") and prm.grad is not None:
            _close(prm.grad, gr[name].grad, 1e-3, name)


def test_hybrid_encoder_under_16_mixed():
    """precision "16-mixed" (fp16 compute): the CNN encoder runs fp16 and the hybrid
    TransformerStage bf16 (dmf_tokens.token_dtype), casting at its boundaries -- the forward and backward
    run (they used to raise) and the logits stay within the 16-bit tolerance of the f32 parity run."""
    P = PR.small_parameters(channels=(16, 32, 64), input_size=64, dropout=0.0, use_backbone=False)
    mp = P["dwi_model_parameters"]
    mp["use_hybrid_transformer"] = True
    mp["transformer_embed_dim"] = 256
    mp["transformer_depth"] = 2
    mp["transformer_heads"] = 4
    mp["mask_stage"] = "f2"
    torch.manual_seed(9)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", copy.deepcopy(P), None), True)
    e32 = copy.deepcopy(enc)
    MM.set_compute_dtype(enc, torch.float16)
    MM.set_compute_dtype(e32, torch.float32)
    enc, e32 = enc.to(DEV).eval(), e32.to(DEV).eval()
    g = torch.Generator().manual_seed(10)
    x = (0.5 + torch.randn(2, 14, 64, 64, generator=g) / 6).clamp(0, 1).to(DEV)
    lo, aux, _ = enc(x)
    l32, aux32, _ = e32(x)
    assert aux["raw_feats"][2].dtype == torch.float16
    _close(lo, l32, 3e-2, "logits fp16 vs f32")
    # the token stage itself runs bf16 (8-bit mantissa) where the reference's fp16 autocast
    # runs fp16 (11-bit); its error against the f32 parity mode is pinned here, as a relative L2 of the
    # stage output (bf16 rounding of a 2-block, 256-wide stage: a few 2^-9 per op).
    f16, f32 = aux["raw_feats"][2].float(), aux32["raw_feats"][2].float()
    rel = ((f16 - f32).norm() / f32.norm()).item()
    assert rel <= 1.5e-2, f"TransformerStage under 16-mixed (bf16 tokens) vs f32: rel L2 {rel:.3e}"
    (aux["raw_feats"][2].float().square().mean()).backward()
    grads = [p.grad for n, p in enc.named_parameters() if n.startswith("transformer.") and p.grad is not None]
    assert grads and all(torch.isfinite(g_).all() for g_ in grads)


def test_patch_embed_fp8_matches_quantised_reference():
    """Config 5's fp8 patch-embed (PatchEmbed.proj, transformer_model.py:17-22,
    on e4m3 MFMA): the quantiser must produce OCP e4m3fn bytes identical to
    torch.float8_e4m3fn's cast of the scaled rows, and the GEMM must match the
    fp32 product of the dequantised operands (fp32 accumulation order only);
    the bf16 backward is the conv engine's."""
    import dmf_native as N
    import dmf_tokens as D
    torch.manual_seed(11)
    n, c, h, w, e, p = 3, 256, 12, 10, 512, 2
    conv = torch.nn.Conv2d(c, e, p, stride=p).to(DEV)
    x = torch.randn(n, c, h, w, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    # reference quantisation (per token row / per output channel, amax -> 448)
    xr = x.float().permute(0, 2, 3, 1).reshape(n, h // p, p, w // p, p, c).permute(0, 1, 3, 2, 4, 5)
    xr = xr.reshape(n * (h // p) * (w // p), p * p * c).cpu()
    rs = xr.abs().amax(1).clamp_min(1e-30) / 448.0
    xq = (xr / rs[:, None]).to(torch.float8_e4m3fn)
    wr = conv.weight.detach().float().permute(0, 2, 3, 1).reshape(e, -1).cpu()
    cs = wr.abs().amax(1) / 448.0
    wq = (wr / cs[:, None]).to(torch.float8_e4m3fn)
    # the kernel's bytes
    m, k = xr.shape
    q = torch.empty((m, k), dtype=torch.uint8, device=DEV)
    rsd = torch.empty(m, dtype=torch.float32, device=DEV)
    N.call("dmf_patch_quant_fp8", x.data_ptr(), n, h, w, c, c, p, q.data_ptr(), k, rsd.data_ptr(),
           N.stream_ptr())
    torch.cuda.synchronize()
    mism = (q.cpu() != xq.view(torch.uint8)).float().mean().item()
    assert mism < 1e-3, mism  # ties may round differently; the format and the scaling must agree
    assert torch.allclose(rsd.cpu(), rs, rtol=1e-6)
    ref = (xq.float() * rs[:, None]) @ (wq.float() * cs[:, None]).t() + conv.bias.detach().float().cpu()
    xd = x.clone().requires_grad_(True)
    y = D.patch_embed_fp8(xd, conv, (O.WeightCache(), O.WeightCache()))
    got = y.float().permute(0, 2, 3, 1).reshape(m, e).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    # and the fp8 projection stays close to the exact conv
    exact = torch.nn.functional.conv2d(x.float(), conv.weight, conv.bias, stride=p)
    rel = (y.float() - exact).abs().max().item() / exact.abs().max().item()
    assert rel < 0.08, rel
    # backward: bf16 conv engine
    g = torch.randn_like(y)
    y.backward(g)
    xr2 = x.float().detach().requires_grad_(True)
    torch.nn.functional.conv2d(xr2, conv.weight.detach(), None, stride=p).backward(g.float())
    assert (xd.grad.float() - xr2.grad).abs().max().item() <= 3e-2 * xr2.grad.abs().max().item()


# token-linear shapes through the bf16 GEMM (128x128 tiles) with every forward epilogue -- bias, gelu +
# aux, LayerScale + f32 residual -- M tails, against float64 on the bf16-rounded operands
NT_CASES = [
    # (M, N, K, out dtype, epilogue)
    (1030, 512, 512, torch.bfloat16, "bias"),
    (4608, 1536, 512, torch.bfloat16, "bias"),
    (700, 384, 2048, torch.float32, "scale_res"),
    (520, 256, 128, torch.bfloat16, "gelu_aux"),
]


@pytest.mark.parametrize("case", NT_CASES)
def test_gemm_token_linear_epilogues(case):
    M, Nn, K, odt, epi = case
    g = torch.Generator().manual_seed(M + K)
    A, W, bias = torch.randn(M, K, generator=g), torch.randn(Nn, K, generator=g) * 0.1, torch.randn(Nn, generator=g)
    res, gam = torch.randn(M, Nn, generator=g), torch.rand(Nn, generator=g)
    Ad, Wd = A.to(DEV, torch.bfloat16), W.to(DEV, torch.bfloat16)
    pre = _bf(A).double() @ _bf(W).double().t() + bias.double()
    C = torch.empty((M, Nn), dtype=odt, device=DEV)
    aux = torch.empty((M, Nn), dtype=torch.bfloat16, device=DEV) if epi == "gelu_aux" else None
    kw = dict(bias=bias.to(DEV))
    if epi == "scale_res":
        kw.update(colscale=gam.to(DEV), res=res.to(DEV))
    if epi == "gelu_aux":
        kw.update(act="gelu", aux=aux)
    D.gemm(C, Ad, Wd, M, Nn, K, lda=K, ldb=K, ldc=Nn, **kw)
    ref = {"bias": pre, "scale_res": res.double() + pre * gam.double(), "gelu_aux": F.gelu(pre)}[epi]
    _close(C, ref, 1e-2, "token linear")
    if epi == "gelu_aux":
        _close(aux, pre, 1e-2, "aux")


def test_gemm_attention_scores_head_slices():
    """Q K^T over head slices of packed qkv rows (batch strides, b_off), n = 200 (tails in both tiles)"""
    b, h, n, d = 2, 4, 200, 128
    e = h * d
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(b, n, 3 * e, generator=g)
    qd = qkv.to(DEV, torch.bfloat16)
    S = torch.empty((b, h, n, n), device=DEV)
    D.gemm(S, qd, qd, n, n, d, lda=3 * e, ldb=3 * e, ldc=n, batch=(b, h), sa=(n * 3 * e, d), sb=(n * 3 * e, d),
           sc=(h * n * n, n * n), b_off=e, alpha=0.125)
    q = _bf(qkv[..., :e]).double().view(b, n, h, d).transpose(1, 2)
    k = _bf(qkv[..., e:2 * e]).double().view(b, n, h, d).transpose(1, 2)
    _close(S, 0.125 * (q @ k.transpose(-1, -2)), 1e-3, "QK^T")
