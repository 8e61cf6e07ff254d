"""Hybrid CNN -> Transformer stage -- MI355X build of the reference's
``code/transformer_model.py`` (used when ``use_hybrid_transformer`` replaces
block3, model_module.py:564-579, :701-703; configuration 5).

Module and parameter names match the reference (PatchEmbed :7-32,
TokensToFeatureMap :34-52, TransformerEncoder :54-66, TransformerBlock
:68-81, MultiHeadSelfAttention :83-116, MLP :118-134, TransformerStage
:137-175). Patch embedding runs on the conv engine; LayerNorm, the linear
layers and attention on the MFMA GEMM + token kernels (dmf_tokens), in the
module's compute dtype (bf16, or f32 for the parity mode).
"""
from __future__ import annotations

import torch
import torch.nn as nn

import dmf_ops as O
import dmf_tokens as D


def _caches(conv):
    c = getattr(conv, "_dmf_caches", None)
    if c is None:
        c = (O.WeightCache(), O.WeightCache())
        conv._dmf_caches = c
    return c


def _rng_if(x, *drops):
    """The Philox snapshot when any of the nn.Dropout modules draws (their own
    train flags: MC dropout turns on only them) -- the enclosing encoder's
    snapshot if there is one, else a fresh one."""
    if not any(d.training and d.p > 0 for d in drops):
        return None
    cur = O.RNG_CURRENT[0]
    return cur if cur is not None else O.RNG.snapshot(x.device)


class PatchEmbed(nn.Module):
    def __init__(self, in_ch, embed_dim, patch_size=2, dim=2):
        super().__init__()
        assert dim in (2, 3)
        self.dim = dim
        self.norm = nn.LayerNorm(embed_dim)
        self.proj = nn.Conv2d(in_ch, embed_dim, kernel_size=patch_size, stride=patch_size)

    # config 5 (BASELINE.json configs[4]): the projection on e4m3 MFMA; set by
    # TransformerStage from parameters "patch_embed_fp8" (bf16 compute only)
    use_fp8 = False

    def forward(self, x):
        dt = D.token_dtype(getattr(self, "compute_dtype", torch.bfloat16))
        x = O.as_nhwc(x.to(dt))
        if self.use_fp8 and dt == torch.bfloat16:
            y = D.patch_embed_fp8(x, self.proj, _caches(self.proj))
        else:
            y = O.conv2d(x, self.proj, _caches(self.proj))       # [B, E, h, w] NHWC
        h, w = y.shape[-2:]
        return D.patch_tokens_layernorm(y, self.norm), (h, w)    # NHWC storage == token order


class TokensToFeatureMap(nn.Module):
    def __init__(self, dim=2):
        super().__init__()
        assert dim in (2, 3)
        self.dim = dim

    def forward(self, tokens, spatial_shape):
        b, n, c = tokens.shape
        h, w = spatial_shape
        return tokens.reshape(b, h, w, c).permute(0, 3, 1, 2)   # NCHW logical, NHWC storage


class MultiHeadSelfAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, qkv_bias=True, attn_drop=0.1, proj_drop=0.1):
        super().__init__()
        assert embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(embed_dim, embed_dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(embed_dim, embed_dim)
        self.proj_drop = nn.Dropout(proj_drop)
        self._sites = (O.RNG.new_site(), O.RNG.new_site())   # Philox: attn_drop, proj_drop

    def forward(self, x):
        rng = _rng_if(x, self.attn_drop, self.proj_drop)
        return D.multihead_self_attention(x, self, rng, D.token_dtype(getattr(self, "compute_dtype", torch.bfloat16)))


class MLP(nn.Module):
    def __init__(self, embed_dim, mlp_ratio=4.0, drop=0.1):
        super().__init__()
        hidden_dim = int(embed_dim * mlp_ratio)
        self.fc1 = nn.Linear(embed_dim, hidden_dim)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden_dim, embed_dim)
        self.drop = nn.Dropout(drop)
        self._sites = (O.RNG.new_site(), O.RNG.new_site())   # Philox: drop after GELU, drop after fc2

    def forward(self, x):
        rng = _rng_if(x, self.drop)
        return D.mlp(x, self, rng, D.token_dtype(getattr(self, "compute_dtype", torch.bfloat16)))


class TransformerBlock(nn.Module):
    def __init__(self, embed_dim, heads, init_scale=0.1):
        super().__init__()
        self.norm1 = nn.LayerNorm(embed_dim)
        self.attn = MultiHeadSelfAttention(embed_dim, heads)
        self.norm2 = nn.LayerNorm(embed_dim)
        self.mlp = MLP(embed_dim)
        self.gamma1 = nn.Parameter(init_scale * torch.ones(embed_dim))
        self.gamma2 = nn.Parameter(init_scale * torch.ones(embed_dim))
        # Philox sites: attn_drop, proj_drop, MLP drop after GELU, MLP drop after fc2
        self._sites = self.attn._sites + self.mlp._sites

    def forward(self, x):
        rng = _rng_if(x, self.attn.attn_drop, self.attn.proj_drop, self.mlp.drop)
        return D.transformer_block(x.float(), self, rng, self._sites,
                                   D.token_dtype(getattr(self, "compute_dtype", torch.bfloat16)))


class TransformerEncoder(nn.Module):
    def __init__(self, embed_dim, depth=4, heads=8):
        super().__init__()
        self.layers = nn.ModuleList([TransformerBlock(embed_dim, heads=heads) for _ in range(depth)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class TransformerStage(nn.Module):
    def __init__(self, in_ch, embed_dim, depth=2, heads=8, patch_size=2, dim=2):
        super().__init__()
        assert dim in (2, 3)
        self.dim = dim
        self.patch_embed = PatchEmbed(in_ch=in_ch, embed_dim=embed_dim, patch_size=patch_size, dim=dim)
        self.transformer = TransformerEncoder(embed_dim=embed_dim, depth=depth, heads=heads)
        self.tokens_to_map = TokensToFeatureMap(dim=dim)

    def forward(self, x):
        # under "16-mixed" the CNN around the stage runs fp16 and the stage bf16 (D.token_dtype): the map
        # leaves in the dtype it came in
        dt = getattr(self, "compute_dtype", torch.bfloat16)
        tokens, hw = self.patch_embed(x)
        tokens = self.transformer(tokens)
        return D.tokens_to_map(tokens, hw[0], hw[1], dt)
