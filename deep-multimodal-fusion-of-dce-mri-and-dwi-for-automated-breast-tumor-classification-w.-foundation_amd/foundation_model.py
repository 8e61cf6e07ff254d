"""Foundation backbones for the DCE / DWI encoders -- MI355X build.

Drop-in for the reference's ``code/foundation_model.py``: same builder names
and signatures (``build_medical_backbone(parameters, device, method,
in_channels)`` :490, ``adapt_first_conv`` :99-124,
``advanced_adapt_first_conv`` :128-176, ``map_rasool_to_timm_keys``
:180-218) and the same side effects on ``parameters`` (:515-523, :559-567).

The reference builds timm's ``resnet50(features_only=True,
output_stride=8, out_indices=(1,2,3,4))`` (:260-267). timm is not a
dependency here: ``ResNet50OS8`` restates that network (module names, stride
/ dilation schedule, feature_info) and runs it on the gfx950 conv engine
(``dmf_ops.conv_bn_act``). Pretrained RadImageNet weights are fetched by the
reference from the HF hub (:74-97); with no network, a local checkpoint can be
given as ``pretrained_path`` (loaded with ``weights_only=True``), otherwise
the backbone keeps timm's random init (documented deviation).
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn as nn

import dmf_ops as O


class _FeatureInfo:
    """timm FeatureInfo subset used by BackboneAdapter (model_module.py:430-433)."""

    def __init__(self, chs, reds):
        self._chs, self._reds = list(chs), list(reds)

    def channels(self, idx=None):
        return list(self._chs) if idx is None else self._chs[idx]

    def reduction(self, idx=None):
        return list(self._reds) if idx is None else self._reds[idx]


def _caches(conv):
    c = getattr(conv, "_dmf_caches", None)
    if c is None:
        c = (O.WeightCache(), O.WeightCache())
        conv._dmf_caches = c
    return c


class Bottleneck(nn.Module):
    """timm Bottleneck (expansion 4): 1x1 -> 3x3 (stride, first_dilation) ->
    1x1, BN after each, ReLU, projection shortcut on the first block."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1, first_dilation=None):
        super().__init__()
        first_dilation = first_dilation or dilation
        outplanes = planes * self.expansion
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=first_dilation, dilation=first_dilation,
                               bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(planes, outplanes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(outplanes)
        self.act3 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def zero_init_last(self):
        nn.init.zeros_(self.bn3.weight)

    def forward(self, x):
        h = O.conv_bn_act(x, self.conv1, _caches(self.conv1), self.bn1, "relu")
        kw = {}
        if O.fuse_input_affine(h, self.conv2, self.conv3, x, *self.parameters()):
            # no autograd (frozen encoder, mode A): conv2's BN apply + ReLU run
            # inside conv3's operand loads -- act2's output is never written
            h, ss2 = O.conv_bn_stats(h, self.conv2, _caches(self.conv2), self.bn2)
            kw = dict(in_ss=ss2, in_act="relu")
        else:
            h = O.conv_bn_act(h, self.conv2, _caches(self.conv2), self.bn2, "relu")
        if self.downsample is not None:
            if len(self.downsample) == 3:
                # ResNet-D (avg_down): the pool, then a stride-1 1x1 projection + BN
                pool, ds_conv, ds_bn = self.downsample
                xs = pool(x)
            else:
                (ds_conv, ds_bn), xs = self.downsample, x
            return O.conv_bn_act(h, self.conv3, _caches(self.conv3), self.bn3, "relu",
                                 skip=(xs, ds_conv, _caches(ds_conv), ds_bn), **kw)
        return O.conv_bn_act(h, self.conv3, _caches(self.conv3), self.bn3, "relu", res=x, **kw)


class AvgDown(nn.Module):
    """The pool of timm's ``downsample_avg`` (resnet.py, ResNet-D): AvgPool2d(2, 2, ceil_mode=True,
    count_include_pad=False) where the stage strides, AvgPool2dSame(2, 1) where output_stride turned the
    stride into dilation. No parameters (the projection stays ``downsample.1`` / ``downsample.2``)."""

    def __init__(self, stride, same):
        super().__init__()
        self.stride, self.same = stride, same

    def forward(self, x):
        return O.avgpool2(x, self.stride, self.same)


class ResNet50OS8(nn.Module):
    """timm ``resnet50`` as built with ``features_only=True, output_stride=8,
    out_indices=(1,2,3,4)``: stem 7x7/2 + maxpool, layer1 (s1), layer2 (s2),
    layer3 (dilation 2), layer4 (dilation 4). forward(x) -> [C2, C3, C4, C5]
    (NCHW logical / NHWC physical, compute dtype).

    variant "resnet50d" (the reference's other ImageNet option,
    foundation_model.py:15-68, dispatch :503): timm's ResNet-D -- the deep
    stem (3x3/2 32 -> 3x3 32 -> 3x3 64, BN + ReLU between, ``conv1.0/1/3/4/6``
    then ``bn1``) and avg_down shortcuts (``AvgDown`` -> stride-1 1x1 -> BN)."""

    def __init__(self, in_chans=3, output_stride=8, layers=(3, 4, 6, 3), compute_dtype=torch.bfloat16,
                 variant="resnet50"):
        super().__init__()
        if variant not in ("resnet50", "resnet50d"):
            raise ValueError(f"ResNet50OS8: unknown variant {variant!r}")
        self.variant = variant
        deep = variant == "resnet50d"
        self.compute_dtype = compute_dtype
        self.in_chans = in_chans
        if deep:
            self.conv1 = nn.Sequential(
                nn.Conv2d(in_chans, 32, 3, stride=2, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
                nn.Conv2d(32, 32, 3, stride=1, padding=1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
                nn.Conv2d(32, 64, 3, stride=1, padding=1, bias=False))
        else:
            self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.act1 = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        inplanes, net_stride, dilation, prev_dilation = 64, 4, 1, 1
        chs, reds = [], []
        for idx, (planes, nblocks) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if idx == 0 else 2
            if net_stride >= output_stride:
                dilation *= stride
                stride = 1
            else:
                net_stride *= stride
            downsample = None
            if stride != 1 or inplanes != planes * Bottleneck.expansion:
                if deep:
                    # timm downsample_avg: no pool at stride 1 / dilation 1; AvgPool2dSame(2, 1) when dilated
                    pool = nn.Identity() if stride == 1 and dilation == 1 else AvgDown(stride, dilation > 1)
                    downsample = nn.Sequential(
                        pool, nn.Conv2d(inplanes, planes * Bottleneck.expansion, 1, stride=1, bias=False),
                        nn.BatchNorm2d(planes * Bottleneck.expansion))
                else:
                    downsample = nn.Sequential(
                        nn.Conv2d(inplanes, planes * Bottleneck.expansion, 1, stride=stride, bias=False),
                        nn.BatchNorm2d(planes * Bottleneck.expansion))
            blocks = []
            for b in range(nblocks):
                blocks.append(Bottleneck(inplanes, planes, stride if b == 0 else 1, downsample if b == 0 else None,
                                         dilation=dilation, first_dilation=prev_dilation))
                prev_dilation = dilation
                inplanes = planes * Bottleneck.expansion
            self.add_module(f"layer{idx + 1}", nn.Sequential(*blocks))
            chs.append(inplanes)
            reds.append(net_stride)
        self.feature_info = _FeatureInfo(chs, reds)
        self._init_timm()

    def _init_timm(self):
        # timm ResNet.init_weights: kaiming_normal_(fan_out, relu) convs, BN (1, 0), zero_init_last
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        for m in self.modules():
            if isinstance(m, Bottleneck):
                m.zero_init_last()

    def stage_input(self, x):
        """NCHW fp32 volume stack -> padded NHWC compute-dtype tensor."""
        dt = self.compute_dtype
        cp = O.channel_pad(self.in_chans, dt)
        if x.dtype == dt and x.shape[1] == cp:
            return O.as_nhwc(x)
        y, _ = O.input_stage(x, dt, None)
        return y

    supports_feature_callback = True

    def forward(self, x, on_feature=None):
        """on_feature(i, feats): called as soon as out_indices map i is
        produced (lets a consumer start on C2 while layer2..4 still run)."""
        with O.bn_scope(self, x.device):
            return self._forward(x, on_feature)

    def _forward(self, x, on_feature):
        if x.shape[1] == self.in_chans or x.dtype != self.compute_dtype:
            x = self.stage_input(x)
        if self.variant == "resnet50d":
            c = self.conv1
            x = O.conv_bn_act(x, c[0], _caches(c[0]), c[1], "relu")
            x = O.conv_bn_act(x, c[3], _caches(c[3]), c[4], "relu")
            x = O.conv_bn_act(x, c[6], _caches(c[6]), self.bn1, "relu")
        else:
            x = O.conv_bn_act(x, self.conv1, _caches(self.conv1), self.bn1, "relu")
        x = O.maxpool2d(x, 3, 2, 1)
        feats = []
        for i in range(1, 5):
            for blk in getattr(self, f"layer{i}"):
                x = blk(x)
            feats.append(x)
            if on_feature is not None:
                on_feature(i - 1, feats)
        return feats


class _DisabledWrapper(nn.Module):
    """Stand-in for the OptimizedModule that ``torch._dynamo.disable(backbone)``
    yields at model_module.py:539 -- keeps the ``_orig_mod`` state_dict prefix."""

    def __init__(self, mod):
        super().__init__()
        self._orig_mod = mod

    @property
    def feature_info(self):
        return self._orig_mod.feature_info

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._modules["_orig_mod"], name)

    @property
    def supports_feature_callback(self):
        return getattr(self._orig_mod, "supports_feature_callback", False)

    def forward(self, x, **kw):
        return self._orig_mod(x, **kw)


# ------------------------------------------------------------- ViT-B/16
# The reference's alternate backbone (foundation_model.py:371-431, dispatch
# :526-545): timm ``vit_base_patch16_224(features_only=True,
# out_indices=range(12), img_size=input_size)`` -- a FeatureGetterNet whose
# ``model`` is the VisionTransformer with norm / head pruned, returning every
# block's output tokens without the class token, reshaped to NCHW maps
# (forward_intermediates, norm=False). Restated with timm's module and
# parameter names (state_dict ``model.blocks.{i}.attn.qkv.weight`` ...); each
# block runs as ONE fused node of the transformer engine (dmf_tokens: pre-LN
# attention + MLP with bias / GELU / residual in the GEMM epilogues;
# LayerScale = ones as timm's init_values=None). The token count 1 + (S/16)^2
# is padded to the GEMM granule of 8 and the padded keys are masked out of
# every softmax row.
class _ViTAttention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.embed_dim = dim
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.attn_drop = nn.Dropout(0.0)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(0.0)
        self._sites = (O.RNG.new_site(), O.RNG.new_site())


class _ViTMlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.drop = nn.Dropout(0.0)
        self.fc2 = nn.Linear(hidden, dim)
        self._sites = (O.RNG.new_site(), O.RNG.new_site())


class ViTBlock(nn.Module):
    """timm Block (pre-LN, no LayerScale, drop_path 0), LayerNorm eps 1e-6."""

    def __init__(self, dim=768, num_heads=12, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _ViTAttention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _ViTMlp(dim, int(dim * mlp_ratio))
        self._sites = self.attn._sites + self.mlp._sites


class _ViTPatchEmbed(nn.Module):
    def __init__(self, in_chans, dim, patch):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, dim, kernel_size=patch, stride=patch)


class _VisionTransformer(nn.Module):
    def __init__(self, in_chans, img_size, patch, dim, depth, num_heads):
        super().__init__()
        self.patch = patch
        self.grid = img_size // patch
        self.patch_embed = _ViTPatchEmbed(in_chans, dim, patch)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, self.grid * self.grid + 1, dim))
        self.blocks = nn.ModuleList([ViTBlock(dim, num_heads) for _ in range(depth)])
        # timm init: pos_embed trunc_normal(0.02), cls_token normal(1e-6), Linear trunc_normal(0.02) / bias 0
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)


class VisionTransformerFeatures(nn.Module):
    """timm FeatureGetterNet(vit_base_patch16_224, out_indices=0..11): forward(x)
    -> 12 maps [B, 768, S/16, S/16] (NCHW logical, NHWC storage, compute dtype)."""

    def __init__(self, in_chans=6, img_size=256, patch=16, dim=768, depth=12, num_heads=12):
        super().__init__()
        self.model = _VisionTransformer(in_chans, img_size, patch, dim, depth, num_heads)
        self.feature_info = _FeatureInfo([dim] * depth, [patch] * depth)
        self.register_buffer("_ones", torch.ones(dim), persistent=False)

    def forward(self, x, on_feature=None):
        import dmf_tokens as D

        m = self.model
        dt = getattr(self, "compute_dtype", torch.bfloat16)
        b, c, h, w = x.shape
        if h % m.patch or w % m.patch or (h // m.patch) * (w // m.patch) + 1 != m.pos_embed.shape[1]:
            raise ValueError(f"ViT-B/16: input {h}x{w} does not match the {m.grid}x{m.grid} patch grid of pos_embed")
        cin = m.patch_embed.proj.in_channels
        if x.dtype != dt or c != O.channel_pad(cin, dt):  # a raw NCHW stack (the encoder stages it already)
            x, _ = O.input_stage(x, dt, None)
        y = O.conv2d(O.as_nhwc(x), m.patch_embed.proj, _caches(m.patch_embed.proj))  # [B, E, h', w'] NHWC
        gh, gw = y.shape[-2:]
        e = y.shape[1]
        tok = y.permute(0, 2, 3, 1).reshape(b, gh * gw, e).float()       # NHWC storage == token order
        n = gh * gw + 1
        t = torch.cat([m.cls_token.expand(b, 1, e), tok], 1) + m.pos_embed   # _pos_embed (class token first)
        npad = (n + 7) // 8 * 8
        if npad != n:
            t = torch.nn.functional.pad(t, (0, 0, 0, npad - n))
        feats = []
        for i, blk in enumerate(m.blocks):
            # (the token kernels run bf16 under "16-mixed": D.token_dtype; the maps leave in dt)
            t = D.transformer_block(t, blk, None, blk._sites, D.token_dtype(dt), n_valid=n,
                                    gammas=(self._ones, self._ones))
            f = t[:, 1:n].reshape(b, gh, gw, e).to(dt)                        # prefix token dropped
            feats.append(O.as_nhwc(f.permute(0, 3, 1, 2)))
            if on_feature is not None:
                on_feature(i, feats)
        return feats


def build_vit_dino_backbone(name="vit_base_patch16_224", pretrained=True, device="cuda", in_channels=6,
                            out_indices=None, img_size=256, use_advanced_adapt=False, compute_dtype=torch.bfloat16):
    """foundation_model.py:371-431. No hub access here: pretrained weights
    are unavailable and the backbone keeps timm's random init (documented)."""
    if out_indices is not None and list(out_indices) != list(range(12)):
        raise NotImplementedError("ViT-B/16 features: out_indices must be all 12 blocks (the reference's call)")
    if pretrained:
        warnings.warn("ViT-B/16 pretrained weights unavailable offline: backbone keeps timm random init")
    vit = VisionTransformerFeatures(in_chans=in_channels, img_size=img_size)
    vit.compute_dtype = compute_dtype
    vit = vit.to(device)  # ModelMaskHeadBackbone adds the _orig_mod wrapper (model_module.py:539)
    vit.output_dims = vit.feature_info.channels()
    vit.expected_input = "B, C, H, W"
    vit.is_3d = False
    return vit


# --------------------------------------------------------- weight plumbing
def adapt_first_conv(state_dict, in_channels):
    """foundation_model.py:99-124: RGB conv1 -> mean over input channels,
    repeated ``in_channels`` times."""
    for k in ("conv1.weight", "encoder.conv1.weight", "module.conv1.weight"):
        if k in state_dict:
            w = state_dict[k]
            if w.shape[1] != in_channels:
                state_dict[k] = w.mean(dim=1, keepdim=True).repeat(1, in_channels, 1, 1)
            return state_dict
    return state_dict


def advanced_adapt_first_conv(state_dict, in_channels, eps=0.05):
    """foundation_model.py:128-176: BT.601 luminance filter replicated with a
    linspace(1-eps, 1+eps) per-channel scale."""
    convs = [k for k, v in state_dict.items() if k.endswith(".weight") and v.dim() == 4]
    if not convs:
        return state_dict
    key = min(convs, key=lambda k: state_dict[k].shape[1])
    w = state_dict[key]
    if w.shape[1] == in_channels:
        return state_dict
    with torch.no_grad():
        if w.shape[1] >= 3:
            lum = 0.2989 * w[:, 0:1] + 0.5870 * w[:, 1:2] + 0.1140 * w[:, 2:3]
        else:
            lum = w.mean(dim=1, keepdim=True)
        scales = torch.linspace(1.0 - eps, 1.0 + eps, in_channels, dtype=w.dtype, device=w.device)
        state_dict[key] = lum.repeat(1, in_channels, 1, 1) * scales.view(1, in_channels, 1, 1)
    return state_dict


def map_rasool_to_timm_keys(rasool_state_dict):
    """foundation_model.py:180-218: torchvision-Sequential RadImageNet keys
    ('0.weight', '1.*', '4.'..'7.') -> timm names; drops 'fc.*'."""
    stage = {"4": "layer1", "5": "layer2", "6": "layer3", "7": "layer4"}
    out = {}
    for k, v in rasool_state_dict.items():
        nk = k[len("backbone."):] if k.startswith("backbone.") else k
        if nk == "0.weight":
            nk = "conv1.weight"
        elif nk.startswith("1."):
            nk = "bn1." + nk[2:]
        elif len(nk) > 1 and nk[0] in stage and nk[1] == ".":
            nk = f"{stage[nk[0]]}.{nk[2:]}"
        if nk.startswith("fc."):
            continue
        out[nk] = v
    return out


def _load_local_checkpoint(backbone, path, in_channels, use_advanced_adapt):
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(ckpt, dict):
        for key in ("state_dict", "model_state_dict", "model", "encoder"):
            if key in ckpt and isinstance(ckpt[key], dict):
                ckpt = ckpt[key]
                break
    if not isinstance(ckpt, dict):
        raise RuntimeError("[RadImageNet] Invalid checkpoint format")
    ckpt = map_rasool_to_timm_keys(ckpt)
    ckpt = advanced_adapt_first_conv(ckpt, in_channels) if use_advanced_adapt else adapt_first_conv(ckpt, in_channels)
    model_state = backbone.state_dict()
    cleaned = {k: v for k, v in ckpt.items() if k in model_state and model_state[k].shape == v.shape}
    backbone.load_state_dict(cleaned, strict=False)
    if len(cleaned) < 100:
        raise RuntimeError("[RadImageNet] Too few weights loaded -- "
                           "likely wrong architecture or incompatible checkpoint")
    return len(cleaned)


def build_radimagenet_backbone(name="resnet50", device="cuda", in_channels=6, output_stride=8,
                               out_indices=(1, 2, 3, 4), use_advanced_adapt=True, pretrained_path=None,
                               compute_dtype=torch.bfloat16):
    """foundation_model.py:220-312 (ResNet-50 only; RadImageNet weights from a
    local ``pretrained_path`` or $DMF_RADIMAGENET_CKPT when present)."""
    if name != "resnet50":
        raise ValueError("RadImageNet build supports resnet50 on this path")
    if tuple(out_indices) != (1, 2, 3, 4):
        raise ValueError("out_indices must be (1, 2, 3, 4)")
    bb = ResNet50OS8(in_chans=in_channels, output_stride=output_stride, compute_dtype=compute_dtype)
    path = pretrained_path or os.environ.get("DMF_RADIMAGENET_CKPT")
    if path:
        _load_local_checkpoint(bb, path, in_channels, use_advanced_adapt)
    else:
        warnings.warn("RadImageNet checkpoint unavailable offline: backbone keeps timm random init")
    bb = bb.to(device)
    bb.output_dims = bb.feature_info.channels()
    bb.expected_input = "B, C, H, W"
    bb.is_3d = False
    bb.foundation_model = True
    bb.transformer_backbone = False
    return bb


def build_imagenet_backbone(name="resnet50d", pretrained=True, device="cuda", in_channels=6, output_stride=8,
                            use_advanced_adapt=False, skip_adapt=True, compute_dtype=torch.bfloat16):
    """foundation_model.py:15-68: timm ``resnet50`` or ``resnet50d`` (ResNet-D: deep stem, avg_down
    shortcuts) at output stride 8; ImageNet weights are network-only, so the backbone keeps timm's
    random init."""
    if name not in ("resnet50", "resnet50d"):
        raise NotImplementedError(f"backbone {name!r} is not an ImageNet ResNet of the reference (resnet50 / resnet50d)")
    bb = ResNet50OS8(in_chans=in_channels, output_stride=output_stride, compute_dtype=compute_dtype,
                     variant=name).to(device)
    bb.output_dims = bb.feature_info.channels()
    bb.expected_input = "B, C, H, W"
    bb.is_3d = False
    return bb


def build_medical_backbone(parameters, device, method, in_channels):
    """foundation_model.py:490-573 -- same dispatch and side effects on
    ``parameters[f'{method}_model_parameters']``."""
    mp = parameters[f"{method}_model_parameters"]
    name = mp["backbone_str"].lower()
    output_stride = 8
    import parameters as _PR

    dtype = _PR.compute_dtype_of(parameters, mp)
    if name in ("resnet50d", "resnet50"):
        bb = build_imagenet_backbone(name=name, device=device, in_channels=in_channels, output_stride=output_stride,
                                     use_advanced_adapt=mp["use_advanced_adapt"], skip_adapt=mp["use_input_adapt"],
                                     compute_dtype=dtype)
        mp["backbone_index_lists"] = [[0], [1], [2, 3]]
        mp["downsample"] = (True, False, False)
        mp["downsample_each_repeat"] = False
        return bb
    if name in ("radimagenet", "radimagenet_resnet50"):
        bb = build_radimagenet_backbone(name="resnet50", device=device, in_channels=in_channels,
                                        output_stride=output_stride, out_indices=(1, 2, 3, 4),
                                        use_advanced_adapt=mp["use_advanced_adapt"],
                                        pretrained_path=mp.get("pretrained_path"), compute_dtype=dtype)
        mp["backbone_index_lists"] = [[0], [1], [2, 3]]
        mp["downsample"] = (True, False, False)
        mp["downsample_each_repeat"] = False
        return bb
    if name in ("vit_base_patch16_224", "dino_vitbase16_pretrain"):
        # :526-545: all 12 block maps at stride 16, chains 3 / 4 / 5 blocks
        mp["backbone_index_lists"] = [[0, 1, 2], [3, 4, 5, 6], [7, 8, 9, 10, 11]]
        mp["downsample"] = (False, False, False)
        mp["channels"] = (768, 768, 768)
        mp["transformer_backbone"] = True
        return build_vit_dino_backbone(in_channels=in_channels, device=device, out_indices=list(range(12)),
                                       img_size=mp["input_size"], use_advanced_adapt=mp["use_advanced_adapt"],
                                       compute_dtype=dtype)
    raise ValueError(f"Unknown backbone_str {name!r}")
