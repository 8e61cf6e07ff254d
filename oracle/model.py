"""fp32 CPU restatement of the reference encoder / backbone / fusion modules.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). PARITY UNPINNED.

Attribute names follow the reference so that ``state_dict`` keys interchange
with the HIP-backed modules in the product package (SURVEY.md 8(b),
"Ownership"); the code itself is written from the source text, not copied.
Every ``forward`` is spelled out functionally (F.conv2d / F.batch_norm ...)
so the op order is visible next to the citation.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def _bn(x, bn: nn.BatchNorm2d):
    # torch BatchNorm2d semantics (train: batch stats + running-stat update,
    # num_batches_tracked += 1 as nn.BatchNorm2d.forward does)
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    return F.batch_norm(
        x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
        bn.training, bn.momentum, bn.eps,
    )


def _conv(x, conv: nn.Conv2d):
    return F.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation)


# --------------------------------------------------------------------- SE
class SEBlock(nn.Module):
    """model_module.py:25-43 -- squeeze/excite returning (x*w, w)."""

    def __init__(self, channels, reduction=2):
        super().__init__()
        hidden = max(channels // reduction, 1)
        self.fc = nn.Sequential(
            nn.AdaptiveAvgPool2d(1), nn.Conv2d(channels, hidden, 1, bias=True), nn.GELU(),
            nn.Conv2d(hidden, channels, 1, bias=True), nn.Sigmoid(),
        )

    def forward(self, x):
        s = x.mean(dim=(2, 3), keepdim=True)
        w = torch.sigmoid(_conv(F.gelu(_conv(s, self.fc[1])), self.fc[3]))
        return x * w, w


class MaskGuidedSpatialAttention(nn.Module):
    """model_module.py:49-97."""

    def __init__(self, in_channels_img, in_channels_mask, hidden_channels=16):
        super().__init__()
        self.gamma = nn.Parameter(torch.tensor(0.1))
        self.mask_processor = nn.Sequential(
            nn.Conv2d(in_channels_mask, hidden_channels, 1, bias=False),
            nn.GroupNorm(1, hidden_channels), nn.GELU(),
            nn.Conv2d(hidden_channels, 1, 1), nn.Sigmoid(),
        )

    def forward(self, img, mask):
        if mask.shape[-2:] != img.shape[-2:]:
            mask = F.interpolate(mask, size=img.shape[-2:], mode="bilinear", align_corners=False)
        mp = self.mask_processor
        h = F.group_norm(_conv(mask, mp[0]), 1, mp[1].weight, mp[1].bias, mp[1].eps)
        a = torch.sigmoid(_conv(F.gelu(h), mp[3])).clamp(1e-4, 1.0 - 1e-4)
        return img * (1 + self.gamma * a), a


class ReconHead(nn.Module):
    """model_module.py:100-125 (upsample=False on every call site)."""

    def __init__(self, in_ch, recon_ch=1):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(in_ch, in_ch, 3, padding=1, bias=False), nn.BatchNorm2d(in_ch), nn.GELU(),
            nn.Conv2d(in_ch, recon_ch, 3, padding=1),
        )

    def forward(self, x):
        c = self.conv
        return _conv(F.gelu(_bn(_conv(x, c[0]), c[1])), c[3])


class MaskHeadResize(nn.Module):
    """model_module.py:131-215: 1x1 pre -> size-dispatched stride-2 3x3 chain
    (or bilinear fallback) -> 1x1 out."""

    def __init__(self, in_ch, mid_ch=64, out_ch=1, out_size=32):
        super().__init__()
        self.out_size = out_size
        self.pre = nn.Conv2d(in_ch, mid_ch, 1)

        def chain(n):
            mods = []
            for _ in range(n):
                mods += [nn.Conv2d(mid_ch, mid_ch, 3, stride=2, padding=1), nn.GELU()]
            return nn.Sequential(*mods)

        self.down_64_to_32 = chain(1)
        self.down_128_to_32 = chain(2)
        self.down_256_to_32 = chain(3)
        self.down_512_to_32 = chain(4)
        self.out = nn.Conv2d(mid_ch, out_ch, 1)
        self._ndown = {32: 0, 64: 1, 128: 2, 256: 3, 512: 4}

    def forward(self, x):
        x = _conv(x, self.pre)
        n = self._ndown.get(x.shape[-1], None)
        if n is None:
            x = F.interpolate(x, size=(self.out_size, self.out_size), mode="bilinear", align_corners=False)
        elif n > 0:
            seq = {1: self.down_64_to_32, 2: self.down_128_to_32, 3: self.down_256_to_32,
                   4: self.down_512_to_32}[n]
            for i in range(0, len(seq), 2):
                x = F.gelu(_conv(x, seq[i]))
        return _conv(x, self.out)


# Test hook: when a list, ResNetLiteBlock_withRecon's dropouts take their
# (1/(1-p)-scaled) masks from it in call order instead of drawing -- the MC
# "shared-mask" parity check feeds the build's Philox masks through here.
DROPOUT_MASKS = None


def _dropout(x, p, on):
    if not on or p <= 0:
        return x
    if DROPOUT_MASKS is not None:
        return x * DROPOUT_MASKS.pop(0).to(x.dtype)
    return F.dropout(x, p, True)


class ResNetLiteBlock_withRecon(nn.Module):
    """model_module.py:220-316 (2-D)."""

    def __init__(self, in_ch, out_ch, downsample=False, recon_ch=1, use_se=False, se_reduction=2,
                 dropout=0.4, num_repeats=1, downsample_each_repeat=False, mid_squeeze=2):
        super().__init__()
        stride = 2 if downsample else 1
        mid = max(out_ch // mid_squeeze, 1)
        self.p = dropout
        self.bottlenecks = nn.ModuleList()
        for i in range(num_repeats):
            s = stride if (downsample_each_repeat or i == 0) else 1
            self.bottlenecks.append(nn.Sequential(
                nn.Conv2d(in_ch if i == 0 else out_ch, mid, 1, stride=s, bias=False), nn.BatchNorm2d(mid),
                nn.GELU(), nn.Dropout(dropout),
                nn.Conv2d(mid, mid, 3, padding=1, bias=False), nn.BatchNorm2d(mid), nn.GELU(),
                nn.Conv2d(mid, out_ch, 1, bias=False), nn.BatchNorm2d(out_ch),
            ))
        self.act = nn.GELU()
        self.dropout = nn.Dropout(dropout)
        self.skip = None
        if stride > 1 or in_ch != out_ch:
            self.skip = nn.Sequential(nn.Conv2d(in_ch, out_ch, 1, stride=stride, bias=False),
                                      nn.BatchNorm2d(out_ch))
        self.use_se = use_se
        self.se = SEBlock(out_ch, se_reduction) if use_se else None
        self.recon_ch = int(recon_ch)
        self.reconstruct = ReconHead(out_ch, recon_ch) if self.recon_ch > 0 else None

    def forward(self, x):
        ident = x if self.skip is None else _bn(_conv(x, self.skip[0]), self.skip[1])
        h = x
        for b in self.bottlenecks:
            # the nn.Dropout modules' own flags, as the reference's
            # nn.Sequential / self.dropout calls (MC dropout turns on only them)
            h = _dropout(F.gelu(_bn(_conv(h, b[0]), b[1])), self.p, b[3].training)
            h = F.gelu(_bn(_conv(h, b[4]), b[5]))
            h = _bn(_conv(h, b[7]), b[8])
        h = _dropout(F.gelu(h + ident), self.p, self.dropout.training)
        if self.se is not None:
            h, _ = self.se(h)
        r = self.reconstruct(h) if self.reconstruct is not None else None
        return h, r


class Projector(nn.Module):
    """model_module.py:323-348."""

    def __init__(self, in_ch, proj_dim=64):
        super().__init__()
        self.proj = nn.Sequential(
            nn.Conv2d(in_ch, proj_dim, 1, bias=False), nn.BatchNorm2d(proj_dim), nn.GELU(),
            nn.Conv2d(proj_dim, proj_dim, 1, bias=False), nn.BatchNorm2d(proj_dim), nn.GELU(),
        )

    def forward(self, x):
        p = self.proj
        return F.gelu(_bn(_conv(F.gelu(_bn(_conv(x, p[0]), p[1])), p[3]), p[4]))


class ClassificationHead(nn.Module):
    """model_module.py:355-369."""

    def __init__(self, in_ch, num_classes, normalize=True):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2d((1, 1))
        self.flatten = nn.Flatten()
        self.fc = nn.Linear(in_ch, num_classes)
        self.normalize = normalize

    def forward(self, x):
        v = x.mean(dim=(2, 3))
        if self.normalize:
            v = F.normalize(v, dim=1)
        return F.linear(v, self.fc.weight, self.fc.bias)


class FeatureDownAlign(nn.Module):
    """model_module.py:371-396."""

    def __init__(self, in_ch, out_ch, downsample=True):
        super().__init__()
        if in_ch != out_ch or downsample:
            k, s, p = (3, 2, 1) if downsample else (1, 1, 0)
            self.proj = nn.Sequential(nn.Conv2d(in_ch, out_ch, k, stride=s, padding=p, bias=False),
                                      nn.BatchNorm2d(out_ch), nn.GELU())
        else:
            self.proj = nn.Identity()

    def forward(self, x):
        if isinstance(self.proj, nn.Identity):
            return x
        return F.gelu(_bn(_conv(x, self.proj[0]), self.proj[1]))


class _FeatInfo:
    def __init__(self, chans, reds):
        self._c, self._r = list(chans), list(reds)

    def channels(self):
        return list(self._c)

    def reduction(self):
        return list(self._r)


# ---------------------------------------------- timm ResNet-50 at stride 8
class Bottleneck(nn.Module):
    """timm resnet Bottleneck (expansion 4, stride on conv2, ReLU);
    SURVEY.md Appendix B. Built at foundation_model.py:260-267."""

    def __init__(self, cin, planes, stride, dilation, first_dilation, downsample):
        super().__init__()
        out = planes * 4
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=first_dilation,
                               dilation=first_dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, out, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out)
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:
            sc = x
        elif len(self.downsample) == 3:  # ResNet-D: pool -> 1x1 -> BN
            sc = _bn(_conv(self.downsample[0](x), self.downsample[1]), self.downsample[2])
        else:
            sc = _bn(_conv(x, self.downsample[0]), self.downsample[1])
        h = F.relu(_bn(_conv(x, self.conv1), self.bn1))
        h = F.relu(_bn(_conv(h, self.conv2), self.bn2))
        h = _bn(_conv(h, self.conv3), self.bn3)
        return F.relu(h + sc)


class AvgDown(nn.Module):
    """timm resnet.py downsample_avg's pool (ResNet-D, reference foundation_model.py:15-68 with
    name='resnet50d'): AvgPool2d(2, stride, ceil_mode=True, count_include_pad=False), or in a
    dilated stage AvgPool2dSame(2, 1) -- pad_same's zero row / column at the end, then the same
    avg_pool2d (the padded zeros are input to it, so they count)."""

    def __init__(self, stride, same):
        super().__init__()
        self.stride, self.same = stride, same

    def forward(self, x):
        if self.same:
            return F.avg_pool2d(F.pad(x, (0, 1, 0, 1)), 2, 1, 0, ceil_mode=True, count_include_pad=False)
        return F.avg_pool2d(x, 2, self.stride, 0, ceil_mode=True, count_include_pad=False)


class ResNet50OS8(nn.Module):
    """timm.create_model('resnet50', features_only=True, output_stride=8,
    out_indices=(1,2,3,4)) -- returns [layer1, layer2, layer3, layer4].
    variant='resnet50d': timm's ResNet-D (stem_type='deep', stem_width=32,
    avg_down=True): conv1 = Sequential(3x3/2 -> 32, BN, ReLU, 3x3 -> 32, BN,
    ReLU, 3x3 -> 64) then bn1; shortcuts AvgDown -> stride-1 1x1 -> BN."""

    LAYOUT = ((64, 3), (128, 4), (256, 6), (512, 3))

    def __init__(self, in_chans=3, variant="resnet50"):
        super().__init__()
        self.variant = variant
        deep = variant == "resnet50d"
        if deep:
            self.conv1 = nn.Sequential(
                nn.Conv2d(in_chans, 32, 3, stride=2, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                nn.Conv2d(32, 32, 3, stride=1, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(),
                nn.Conv2d(32, 64, 3, stride=1, padding=1, bias=False))
        else:
            self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        cin, net_stride, dil, prev_dil = 64, 4, 1, 1
        for si, (planes, n) in enumerate(self.LAYOUT):
            stride = 1 if si == 0 else 2
            if net_stride >= 8:
                dil *= stride
                stride = 1
            else:
                net_stride *= stride
            blocks = []
            for bi in range(n):
                ds = None
                if bi == 0 and (stride != 1 or cin != planes * 4):
                    if deep:
                        pool = nn.Identity() if stride == 1 and dil == 1 else AvgDown(stride, dil > 1)
                        ds = nn.Sequential(pool, nn.Conv2d(cin, planes * 4, 1, stride=1, bias=False),
                                           nn.BatchNorm2d(planes * 4))
                    else:
                        ds = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride=stride, bias=False),
                                           nn.BatchNorm2d(planes * 4))
                blocks.append(Bottleneck(cin, planes, stride if bi == 0 else 1, dil, prev_dil, ds))
                prev_dil = dil
                cin = planes * 4
            setattr(self, f"layer{si + 1}", nn.Sequential(*blocks))
        self.feature_info = _FeatInfo([256, 512, 1024, 2048], [4, 8, 8, 8])
        self.output_dims = self.feature_info.channels()
        self.expected_input = "B, C, H, W"
        self.is_3d = False

    def forward(self, x):
        if self.variant == "resnet50d":
            c = self.conv1
            x = F.relu(_bn(_conv(x, c[0]), c[1]))
            x = F.relu(_bn(_conv(x, c[3]), c[4]))
            x = F.relu(_bn(_conv(x, c[6]), self.bn1))
        else:
            x = F.relu(_bn(_conv(x, self.conv1), self.bn1))
        x = F.max_pool2d(x, 3, 2, 1)
        feats = []
        for i in range(1, 5):
            x = getattr(self, f"layer{i}")(x)
            feats.append(x)
        return feats


class _Wrapped(nn.Module):
    """Stands in for the OptimizedModule that torch._dynamo.disable(backbone)
    yields at model_module.py:539 (state_dict prefix ``_orig_mod``)."""

    def __init__(self, mod):
        super().__init__()
        self._orig_mod = mod
        self.feature_info = getattr(mod, "feature_info", None)

    def forward(self, x):
        return self._orig_mod(x)


class BackboneAdapter(nn.Module):
    """model_module.py:401-476 (CNN feature maps; token reshape for ViT)."""

    def __init__(self, backbone, selected_indices_chains, out_channels=(64, 128, 256), is_transformer=False):
        super().__init__()
        self.backbone = backbone
        self.selected_indices_chains = selected_indices_chains
        self.is_transformer = is_transformer
        chans = backbone.feature_info.channels()
        self.necks = nn.ModuleDict()
        for i, chain in enumerate(selected_indices_chains):
            cin = sum(chans[j] for j in chain)
            co = out_channels[i]
            self.necks[f"f{i + 1}"] = nn.Sequential(
                nn.Conv2d(cin, co, 3, padding=1), nn.BatchNorm2d(co), nn.GELU(),
                nn.Conv2d(co, co, 3, padding=1), nn.BatchNorm2d(co), nn.GELU(),
            )

    def forward(self, x):
        feats = self.backbone(x)
        outs = []
        for i, chain in enumerate(self.selected_indices_chains):
            parts = []
            for j in chain:
                f = feats[j]
                if self.is_transformer and f.ndim == 3:
                    b, n, c = f.shape
                    s = int(n ** 0.5)
                    f = f.permute(0, 2, 1).reshape(b, c, s, s)
                parts.append(f)
            h = torch.cat(parts, dim=1)
            nk = self.necks[f"f{i + 1}"]
            h = F.gelu(_bn(_conv(h, nk[0]), nk[1]))
            outs.append(F.gelu(_bn(_conv(h, nk[3]), nk[4])))
        return outs[0], outs[1], outs[2]


# ------------------------------------------------------------- ViT-B/16
class _VitAttention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.num_heads, self.head_dim = heads, dim // heads
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        b, n, c = x.shape
        q, k, v = self.qkv(x).reshape(b, n, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        a = torch.softmax((q @ k.transpose(-2, -1)) * self.head_dim ** -0.5, dim=-1)
        return self.proj((a @ v).transpose(1, 2).reshape(b, n, c))


class _VitMlp(nn.Module):
    def __init__(self, dim, hid):
        super().__init__()
        self.fc1 = nn.Linear(dim, hid)
        self.fc2 = nn.Linear(hid, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class _VitBlock(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _VitAttention(dim, heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _VitMlp(dim, 4 * dim)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class _PatchProj(nn.Module):
    def __init__(self, cin, dim, p):
        super().__init__()
        self.proj = nn.Conv2d(cin, dim, p, stride=p)


class _Vit(nn.Module):
    def __init__(self, cin, img, p, dim, depth, heads):
        super().__init__()
        self.patch = p
        self.patch_embed = _PatchProj(cin, dim, p)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, (img // p) ** 2 + 1, dim))
        self.blocks = nn.ModuleList([_VitBlock(dim, heads) for _ in range(depth)])


class VisionTransformerFeatures(nn.Module):
    """timm vit_base_patch16_224(features_only=True, out_indices=range(12),
    img_size=S) as foundation_model.py:371-431 builds it: FeatureGetterNet
    ('model' = the VisionTransformer, norm / head pruned) ->
    forward_intermediates(norm=False, output_fmt='NCHW'): patch_embed (conv
    k = s = 16, flatten), class token prepended, + pos_embed, then every
    block's output with the class token dropped, reshaped [B, 768, S/16, S/16]."""

    def __init__(self, in_chans=6, img_size=256, patch=16, dim=768, depth=12, heads=12):
        super().__init__()
        self.model = _Vit(in_chans, img_size, patch, dim, depth, heads)
        self.feature_info = _FeatInfo([dim] * depth, [patch] * depth)
        self.output_dims = self.feature_info.channels()

    def forward(self, x):
        m = self.model
        b = x.shape[0]
        y = _conv(x, m.patch_embed.proj)
        gh, gw = y.shape[-2:]
        t = y.flatten(2).transpose(1, 2)
        t = torch.cat([m.cls_token.expand(b, -1, -1), t], 1) + m.pos_embed
        feats = []
        for blk in m.blocks:
            t = blk(t)
            feats.append(t[:, 1:].reshape(b, gh, gw, -1).permute(0, 3, 1, 2).contiguous())
        return feats


# ------------------------------------------------- hybrid transformer stage
class PatchEmbed(nn.Module):
    """transformer_model.py:7-32."""

    def __init__(self, in_ch, embed_dim, patch_size=2):
        super().__init__()
        self.norm = nn.LayerNorm(embed_dim)
        self.proj = nn.Conv2d(in_ch, embed_dim, patch_size, stride=patch_size)

    def forward(self, x):
        x = _conv(x, self.proj)
        hw = x.shape[-2:]
        t = x.flatten(2).transpose(1, 2)
        return F.layer_norm(t, t.shape[-1:], self.norm.weight, self.norm.bias, self.norm.eps), hw


class MultiHeadSelfAttention(nn.Module):
    """transformer_model.py:83-116 (dropouts are identity for p=0 / eval)."""

    def __init__(self, embed_dim, num_heads, qkv_bias=True, attn_drop=0.1, proj_drop=0.1):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(embed_dim, embed_dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(embed_dim, embed_dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        b, n, c = x.shape
        q, k, v = self.qkv(x).reshape(b, n, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        a = self.attn_drop(torch.softmax((q @ k.transpose(-2, -1)) * self.scale, dim=-1))
        y = (a @ v).transpose(1, 2).reshape(b, n, c)
        return self.proj_drop(self.proj(y))


class MLP(nn.Module):
    """transformer_model.py:118-134."""

    def __init__(self, embed_dim, mlp_ratio=4.0, drop=0.1):
        super().__init__()
        hid = int(embed_dim * mlp_ratio)
        self.fc1 = nn.Linear(embed_dim, hid)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hid, embed_dim)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.drop(self.fc2(self.drop(F.gelu(self.fc1(x)))))


class TransformerBlock(nn.Module):
    """transformer_model.py:68-81 (pre-LN, LayerScale)."""

    def __init__(self, embed_dim, heads, init_scale=0.1):
        super().__init__()
        self.norm1 = nn.LayerNorm(embed_dim)
        self.attn = MultiHeadSelfAttention(embed_dim, heads)
        self.norm2 = nn.LayerNorm(embed_dim)
        self.mlp = MLP(embed_dim)
        self.gamma1 = nn.Parameter(init_scale * torch.ones(embed_dim))
        self.gamma2 = nn.Parameter(init_scale * torch.ones(embed_dim))

    def forward(self, x):
        x = x + self.attn(self.norm1(x)) * self.gamma1
        return x + self.mlp(self.norm2(x)) * self.gamma2


class TransformerEncoder(nn.Module):
    def __init__(self, embed_dim, depth=4, heads=8):
        super().__init__()
        self.layers = nn.ModuleList([TransformerBlock(embed_dim, heads) for _ in range(depth)])

    def forward(self, x):
        for blk in self.layers:
            x = blk(x)
        return x


class TransformerStage(nn.Module):
    """transformer_model.py:137-175."""

    def __init__(self, in_ch, embed_dim, depth=2, heads=8, patch_size=2):
        super().__init__()
        self.patch_embed = PatchEmbed(in_ch, embed_dim, patch_size)
        self.transformer = TransformerEncoder(embed_dim, depth, heads)

    def forward(self, x):
        t, (h, w) = self.patch_embed(x)
        t = self.transformer(t)
        return t.transpose(1, 2).reshape(t.shape[0], t.shape[2], h, w)


# ---------------------------------------------------------------- encoder
class ModelMaskHeadBackbone(nn.Module):
    """model_module.py:481-733 (2-D)."""

    def __init__(self, method, parameters_dict, backbone=None):
        super().__init__()
        P = parameters_dict
        mp = P[f"{method}_model_parameters"]
        self.channel_num = P[f"{method}_channel_num"]
        self.num_classes = P["class_num"]
        c1, c2, c3 = mp["channels"]
        self.use_backbone = mp["use_backbone"]
        self.use_hybrid_transformer = mp["use_hybrid_transformer"]
        mk = mp["mask_parameters"]
        self.mask_enabled = mk["mask"]
        self.mask_stage = mk["mask_stage"].lower()
        self.mask_size = mk["mask_target_size"][0]
        self.proj_dim = mp["proj_dim"]
        ds, rep, drop = mp["downsample"], mp["repeat_blocks"], mp["dropout"]
        dser, msq, use_se = mp["downsample_each_repeat"], mp["mid_squeeze"], mp["use_se"]

        self.backbone = _Wrapped(backbone) if backbone is not None else None
        if self.use_backbone:
            self.backbone_adapter = BackboneAdapter(self.backbone, mp["backbone_index_lists"], (c1, c1, c2),
                                                    is_transformer=mp["transformer_backbone"])
            b1_in = c1
        else:
            b1_in = self.channel_num
        kw = dict(use_se=use_se, dropout=drop, downsample_each_repeat=dser, mid_squeeze=msq)
        self.block1 = ResNetLiteBlock_withRecon(b1_in, c1, ds[0], recon_ch=1, num_repeats=rep[0], **kw)
        self.block2 = ResNetLiteBlock_withRecon(c1, c2, ds[1], recon_ch=1, num_repeats=rep[1], **kw)
        if not self.use_hybrid_transformer:
            self.block3 = ResNetLiteBlock_withRecon(c2, c3, ds[2], recon_ch=0, num_repeats=rep[2], **kw)
        else:
            self.transformer = TransformerStage(c2, mp["transformer_embed_dim"], mp["transformer_depth"],
                                                mp["transformer_heads"], mp["transformer_patch_size"])
            self.trans_out_proj = nn.Conv2d(mp["transformer_embed_dim"], c3, 1)
        self.modality_attention = None
        if mp["enable_modality_attention"]:
            if method not in ("dwi", "dce"):
                raise ValueError("Unknown method for modality attention.")
            self.modality_attention = SEBlock(self.channel_num, 2)
        self.f2_weight = nn.Parameter(torch.tensor(0.5))
        self.f3_weight = nn.Parameter(torch.tensor(0.5))
        self.norm_f2 = nn.GroupNorm(c1, c1)
        self.norm_f3 = nn.GroupNorm(c2, c2)
        if self.mask_enabled:
            self.f1_to_f2 = FeatureDownAlign(c1, c2, downsample=False)
            self.f2_to_f3 = FeatureDownAlign(c2, c3, downsample=False)
            m_in = {"f1": c1, "f2": c2, "f3": c3}[self.mask_stage]
            self.mask_head = MaskHeadResize(m_in, out_size=self.mask_size)
            self.mask_spatial_attention = MaskGuidedSpatialAttention(c3, 1)
        self.classification_head = ClassificationHead(c3, self.num_classes)
        self.proj_f1 = Projector(c1, self.proj_dim)
        self.proj_f2 = Projector(c2, self.proj_dim)
        self.proj_r1 = Projector(1, self.proj_dim)
        self.proj_r2 = Projector(1, self.proj_dim)

    @staticmethod
    def _gn(x, gn):
        return F.group_norm(x, gn.num_groups, gn.weight, gn.bias, gn.eps)

    def forward(self, x, masks=None):
        mask_pred = attn_map = None
        if self.modality_attention is not None:
            x, mod_map = self.modality_attention(x)
        else:
            mod_map = None
        if self.use_backbone:
            f1_b, f2_b, f3_b = self.backbone_adapter(x)
            f1, r1 = self.block1(f1_b)
        else:
            f1, r1 = self.block1(x)
        if self.mask_enabled and self.mask_stage == "f1":
            mask_pred = self.mask_head(f1)
            f1, attn_map = self.mask_spatial_attention(f1, mask_pred)
        if self.use_backbone:
            a = torch.sigmoid(self.f2_weight)
            f2, r2 = self.block2(self._gn(a * f2_b + (1 - a) * f1, self.norm_f2))
        else:
            f2, r2 = self.block2(f1)
        if self.mask_enabled and self.mask_stage == "f2":
            mask_pred = self.mask_head(f2 + self.f1_to_f2(f1))
            f2, attn_map = self.mask_spatial_attention(f2, mask_pred)
        if not self.use_hybrid_transformer:
            if self.use_backbone:
                a = torch.sigmoid(self.f3_weight)
                f3, _ = self.block3(self._gn(a * f3_b + (1 - a) * f2, self.norm_f3))
            else:
                f3, _ = self.block3(f2)
            if self.mask_enabled and self.mask_stage == "f3":
                mask_pred = self.mask_head(f3 + self.f2_to_f3(f2))
                f3, attn_map = self.mask_spatial_attention(f3, mask_pred)
        else:
            f3 = _conv(self.transformer(f2), self.trans_out_proj)
        pool = (self.proj_dim, self.proj_dim)
        p1 = self.proj_f1(F.adaptive_avg_pool2d(f1, pool))
        p2 = self.proj_f2(F.adaptive_avg_pool2d(f2, pool))
        p1_r = self.proj_r1(F.adaptive_avg_pool2d(r1, pool))
        p2_r = self.proj_r2(F.adaptive_avg_pool2d(r2, pool))
        logits = self.classification_head(f3)
        aux = {"raw_feats": [f1, f2, f3], "recon_feats": [r1, r2], "proj_pairs": [p1, p1_r, p2, p2_r],
               "mask_attn_map": attn_map, "mod_attn_map": mod_map}
        return logits, aux, mask_pred


# ----------------------------------------------------------------- fusion
class GatingAttention(nn.Module):
    """model_module.py:745-780 (mask confidence = mean of mask LOGITS)."""

    def __init__(self, feat_dim, use_mask_attention=True):
        super().__init__()
        self.use_mask_attention = use_mask_attention
        self.fc = nn.Linear(feat_dim * 2 + (2 if use_mask_attention else 0), 2)

    def forward(self, pv_dwi, pv_dce, dwi_mask=None, dce_mask=None):
        parts = [pv_dwi, pv_dce]
        if self.use_mask_attention and dwi_mask is not None and dce_mask is not None:
            parts += [dwi_mask.mean(dim=(2, 3)).reshape(len(pv_dwi), -1),
                      dce_mask.mean(dim=(2, 3)).reshape(len(pv_dce), -1)]
        return torch.softmax(F.linear(torch.cat(parts, 1), self.fc.weight, self.fc.bias), dim=1)


class FusionReduce(nn.Module):
    """model_module.py:782-794."""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.reduce = nn.Sequential(nn.Conv2d(in_ch, out_ch, 1, bias=False), nn.BatchNorm2d(out_ch), nn.GELU())

    def forward(self, x):
        return F.gelu(_bn(_conv(x, self.reduce[0]), self.reduce[1]))


class CrossAttentionBlock(nn.Module):
    """model_module.py:799-818."""

    def __init__(self, channels, num_heads=4):
        super().__init__()
        self.cross_attn = nn.MultiheadAttention(channels, num_heads, batch_first=True)
        self.attn_ffn = nn.Sequential(nn.LayerNorm(channels), nn.Linear(channels, channels), nn.GELU(),
                                      nn.Linear(channels, channels))

    def forward(self, q, kv):
        out, w = self.cross_attn(q, kv, kv, need_weights=True)
        f = self.attn_ffn
        h = F.layer_norm(out, out.shape[-1:], f[0].weight, f[0].bias, f[0].eps)
        h = F.linear(F.gelu(F.linear(h, f[1].weight, f[1].bias)), f[3].weight, f[3].bias)
        return out + h, w


class FusionModel(nn.Module):
    """model_module.py:821-1000 (2-D)."""

    def __init__(self, parameters_dict):
        super().__init__()
        fc = parameters_dict["fusion_model_parameters"]
        fs = fc["fusion_specific_parameters"]
        C = self.fusion_channels = fs["fusion_channels"]
        self.token_pool = fs["token_pool"]
        self.use_cross_attention = fs["use_cross_attention"]
        self.num_classes = parameters_dict["class_num"]
        self.proj_in_dwi = nn.Conv2d(fs["dwi_out_channels"], C, 1, bias=False) \
            if fs["dwi_out_channels"] != C else nn.Identity()
        self.proj_in_dce = nn.Conv2d(fs["dce_out_channels"], C, 1, bias=False) \
            if fs["dce_out_channels"] != C else nn.Identity()
        self.fusion_conv_reduce = FusionReduce(2 * C, C)
        self.refine_act = nn.GELU()
        self.fusion_se = SEBlock(C, 2) if fc["use_se"] else None
        self.gating = GatingAttention(C, fs["use_mask_attention"])
        self.refine = ResNetLiteBlock_withRecon(C, C, dropout=fc["dropout"], mid_squeeze=2)
        if self.use_cross_attention:
            self.cross_attn_block = CrossAttentionBlock(C, fs["mha_heads"])
        self.mask_head = MaskHeadResize(C, out_size=fc["mask_parameters"]["mask_target_size"][0])
        self.fusion_reconstruct = ReconHead(C, fs["fusion_recon_ch"])
        self.classifier = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)), nn.Flatten(), nn.Linear(C, self.num_classes))
        self.projF = Projector(C, fc["proj_dim"])

    def _proj(self, mod, x):
        return x if isinstance(mod, nn.Identity) else _conv(x, mod)

    def forward(self, raw_feats_dwi, raw_feats_dce, dwi_mask_pred=None, dce_mask_pred=None):
        p_dwi = self._proj(self.proj_in_dwi, raw_feats_dwi[-1])
        p_dce = self._proj(self.proj_in_dce, raw_feats_dce[-1])
        reduced = self.fusion_conv_reduce(torch.cat([p_dwi, p_dce], 1))
        residual, _ = self.refine(reduced)
        _refined = F.gelu(reduced + residual)  # Q4: computed, never consumed
        g = self.gating(p_dwi.mean(dim=(2, 3)), p_dce.mean(dim=(2, 3)), dwi_mask_pred, dce_mask_pred)
        fused = g[:, 0].view(-1, 1, 1, 1) * p_dwi + g[:, 1].view(-1, 1, 1, 1) * p_dce
        attn_w = None
        if self.use_cross_attention:
            hp, wp = self.token_pool
            tok = lambda f: F.adaptive_avg_pool2d(f, (hp, wp)).flatten(2).transpose(1, 2)
            out, attn_w = self.cross_attn_block(tok(p_dwi), tok(p_dce))
            b, n, c = out.shape
            low = out.transpose(1, 2).reshape(b, c, hp, wp)
            fused = fused + F.interpolate(low, size=fused.shape[-2:], mode="bilinear", align_corners=False)
        if self.fusion_se is not None:
            fused, _ = self.fusion_se(fused)
        mask_logits = self.mask_head(fused)
        cl = self.classifier[2]
        logits = F.linear(fused.mean(dim=(2, 3)), cl.weight, cl.bias)
        recon = self.fusion_reconstruct(fused)
        proj = self.projF(fused)
        aux = {"proj_fused": proj, "recon_fused": recon, "gating_weights": g, "attn_weights": attn_w,
               "p_dwi": p_dwi, "p_dce": p_dce}
        return logits, mask_logits, aux


def init_parameter(m):
    """model_module.py:1002-1015."""
    if isinstance(m, nn.Linear):
        nn.init.kaiming_uniform_(m.weight.data)
        if m.bias is not None:
            nn.init.zeros_(m.bias.data)
    elif isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d)):
        if m.weight is not None:
            nn.init.normal_(m.weight.data, 1.0, 0.02)
        if m.bias is not None:
            nn.init.zeros_(m.bias.data)


def initialize_model(model, requires_grad):
    """model_module.py:1018-1023."""
    for p in model.parameters():
        p.requires_grad = requires_grad
    model.apply(init_parameter)
    return model
