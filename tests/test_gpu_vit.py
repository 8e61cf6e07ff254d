"""a22: the ViT-B/16 backbone alternate (foundation_model.py:371-431,
dispatch :526-545) against the oracle's restatement of timm's
vit_base_patch16_224 features_only forward (oracle.model.VisionTransformerFeatures):

* all 12 block maps and the encoder's logits / mask in the f32 parity mode,
  eval: 17 tokens at S=64 (padded to 24 on the device, the padded keys
  masked out of every softmax row);
* train mode forward + backward: every ViT parameter's gradient;
* bf16 at the config shape (S=256: 257 tokens padded to 264), finite, with
  the relative error against the oracle reported."""
import copy

import pytest
import torch

import foundation_model as FM
import model_module as MM
import parameters as PR
from oracle import model as OM

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(size, seed=0, dtype=torch.float32):
    P = copy.deepcopy(PR.small_parameters(dropout=0.0, input_size=size))
    P["dwi_model_parameters"]["backbone_str"] = "vit_base_patch16_224"
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", "dwi", 14)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, bb), True)
    with torch.no_grad():  # non-trivial pos / cls / LayerNorm parameters
        for n, p in enc.named_parameters():
            if "norm" in n and n.endswith("weight"):
                p.copy_(1 + 0.1 * torch.randn_like(p))
            elif "norm" in n and n.endswith("bias"):
                p.copy_(0.1 * torch.randn_like(p))
            elif n.endswith("cls_token"):
                p.copy_(0.02 * torch.randn_like(p))
    ref = OM.ModelMaskHeadBackbone("dwi", P, OM.VisionTransformerFeatures(14, size))
    ref.load_state_dict(enc.state_dict())
    MM.set_compute_dtype(enc, dtype)
    return enc.to(DEV), ref


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_vit_features_and_encoder_eval_f32():
    enc, ref = _pair(64)
    enc.eval()
    ref.eval()
    x = torch.rand(2, 14, 64, 64)
    with torch.no_grad():
        feats = enc.backbone_adapter.backbone(x.to(DEV))
        rfeats = ref.backbone_adapter.backbone(x)
        lo, aux, mp = enc(x.to(DEV))
        rlo, raux, rmp = ref(x)
    assert len(feats) == 12
    for i, (a, b) in enumerate(zip(feats, rfeats)):
        assert a.shape == b.shape, (i, a.shape, b.shape)
        assert _rel(a, b) < 1e-4, (i, _rel(a, b))
    assert (lo.cpu() - rlo).abs().max().item() < 1e-3
    assert (mp.cpu() - rmp).abs().max().item() < 1e-3 * max(1.0, rmp.abs().max().item())
    for a, b in zip(aux["raw_feats"], raux["raw_feats"]):
        assert _rel(a, b) < 1e-3


def test_vit_train_backward_f32():
    enc, ref = _pair(64, seed=1)
    enc.train()
    ref.train()
    x = torch.rand(2, 14, 64, 64)
    lo, aux, _ = enc(x.to(DEV))
    rlo, raux, _ = ref(x)
    (lo.float().square().mean() + aux["raw_feats"][2].float().square().mean()).backward()
    (rlo.square().mean() + raux["raw_feats"][2].square().mean()).backward()
    assert (lo.detach().cpu() - rlo.detach()).abs().max().item() < 1e-3
    named = dict(ref.named_parameters())
    checked = 0
    for n, p in enc.named_parameters():
        if ".model." in n and named[n].grad is not None and p.grad is not None:
            g = named[n].grad
            assert _rel(p.grad.reshape(g.shape), g) < 2e-3, (n, _rel(p.grad.reshape(g.shape), g))
            checked += 1
    assert checked > 100, checked


def test_vit_bf16_config_shape():
    enc, ref = _pair(256, seed=2, dtype=torch.bfloat16)
    enc.eval()
    ref.eval()
    x = torch.rand(2, 14, 256, 256)
    with torch.no_grad():
        lo, aux, _ = enc(x.to(DEV))
        rlo, raux, _ = ref(x)
        feats = enc.backbone_adapter.backbone(x.to(DEV))
        rfeats = ref.backbone_adapter.backbone(x)
    assert feats[0].shape == (2, 768, 16, 16)
    assert torch.isfinite(lo).all()
    errs = [_rel(a, b) for a, b in zip(feats, rfeats)]
    print(f"ViT bf16 S=256: block-map rel L2 {max(errs):.2e} (max over 12), logits max abs "
          f"{(lo.float().cpu() - rlo).abs().max().item():.2e}")
    assert max(errs) < 3e-2


def test_vit_under_16_mixed():
    """precision "16-mixed" (fp16 compute): the ViT's patch conv and feature maps run fp16,
    its transformer blocks bf16 (dmf_tokens.token_dtype); forward + backward run (they used to raise in
    the token kernels' dtype check) and the block maps stay within the 16-bit tolerance of the oracle."""
    enc, ref = _pair(64, seed=3, dtype=torch.float16)
    enc.train()
    ref.train()
    x = torch.rand(2, 14, 64, 64)
    feats = enc.backbone_adapter.backbone(x.to(DEV))
    with torch.no_grad():
        rfeats = ref.backbone_adapter.backbone(x)
    assert all(f.dtype == torch.float16 for f in feats)
    errs = [_rel(a, b) for a, b in zip(feats, rfeats)]
    assert max(errs) < 3e-2, errs
    lo, aux, _ = enc(x.to(DEV))
    (lo.float().square().mean() + aux["raw_feats"][2].float().square().mean()).backward()
    grads = [p.grad for n, p in enc.named_parameters() if ".model." in n and p.grad is not None]
    assert len(grads) > 100 and all(torch.isfinite(g).all() for g in grads)
