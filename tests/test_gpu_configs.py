"""BASELINE.json configs 1 and 2 on the HIP path, against the CPU oracle.

* Config 2 -- the DCE-only foundation feature extractor: the timm-equivalent
  ResNet-50 OS8 built by ``build_medical_backbone(P, device, 'dce',
  in_channels=5)`` (reference foundation_model.py:260-267 via :546-556; five
  DCE phases, parameters_generate.py:242/:251), forward only. The 5-channel
  stem runs on the channel-padded staging path (5 -> 8), which is exactly what
  this test pins. fp32 parity mode: C2..C5 within 2e-3 of the oracle (relative
  to each map's max); bf16 throughput mode: relative L2 error per map reported
  and bounded at 3e-2.
* Config 1 -- the single-modality DWI CNN with ``use_backbone=False`` (reference
  model_module.py:550-552, :663-666; train.py:294-428; synthetic recipe of
  debug_suite.py:16-24): C=16, S=128, B=4, default channel widths. One train
  step (loss terms, logits, every parameter gradient) plus one val step.
  Tolerances: logits 1e-3 absolute, loss terms 1e-4 relative; gradients judged
  against a float64 evaluation of the oracle (the fp32 oracle's own error sets
  the bar, as in test_gpu_parity).
"""
import copy

import pytest
import torch

import foundation_model as FM
import model_module as MM
import parameters as PR
import train as TR
from oracle import losses as OL
from oracle import model as OM
from selector_helpers import get_classification_loss
from test_gpu_parity import _randomize_bn

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _config2_pair(dtype, seed=1):
    P = PR.default_parameters()
    P["dce_channel_num"] = 5
    P["dwi_model_parameters"]["compute_dtype"] = dtype
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", "dce", 5)
    _randomize_bn(bb, seed)  # timm zero-inits every bn3 gamma: randomise so each residual branch counts
    ref = OM.ResNet50OS8(5)
    ref.load_state_dict(bb.state_dict())
    return bb.to(DEV), ref


def _dce_volumes(B, C, S, seed):
    """U[0,1) (Nyul output range), 5 phases."""
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, C, S, S, generator=g)


@pytest.mark.parametrize("train", [False, True])
def test_config2_dce_backbone_f32_parity(train):
    bb, ref = _config2_pair(torch.float32)
    bb.train(train)
    ref.train(train)
    x = _dce_volumes(2, 5, 256, 1)
    with torch.no_grad():
        got = bb(x.to(DEV))
        want = ref(x)
    assert [tuple(f.shape) for f in got] == [(2, 256, 64, 64), (2, 512, 32, 32), (2, 1024, 32, 32), (2, 2048, 32, 32)]
    for i, (a, b) in enumerate(zip(got, want)):
        err = (a.float().cpu() - b).abs().max().item()
        assert err < 2e-3 * max(1.0, b.abs().max().item()), (f"C{i + 2}", err)
    if train:  # running statistics moved exactly as nn.BatchNorm2d's
        for (n, b1), (_, b2) in zip(bb.named_buffers(), ref.named_buffers()):
            if b1.dtype.is_floating_point:
                assert (b1.cpu() - b2).abs().max() < 1e-3 * max(1.0, b2.abs().max().item()), n
            else:
                assert torch.equal(b1.cpu(), b2), n


def test_config2_dce_backbone_bf16_close():
    """The throughput dtype (what bench.py --config 2 runs) at the config's
    batch 16: relative L2 error of every feature map vs the fp32 oracle."""
    bb, ref = _config2_pair(torch.bfloat16)
    bb.eval()
    ref.eval()
    x = _dce_volumes(16, 5, 256, 2)
    with torch.no_grad():
        got = bb(x.to(DEV))
        want = ref(x)
    errs = []
    for a, b in zip(got, want):
        errs.append(((a.float().cpu() - b).norm() / b.norm().clamp_min(1e-12)).item())
    print("config 2 bf16 relative L2 error C2..C5:", [round(e, 5) for e in errs])
    assert max(errs) < 3e-2, errs


def _config1_params():
    P = PR.default_parameters()
    mp = P["dwi_model_parameters"]
    mp["use_backbone"] = False
    mp["input_size"] = 128
    mp["dropout"] = 0.0  # parity: deterministic path (the Philox masks are not torch's)
    P["dwi_channel_num"] = 16
    return P


def _config1_batch(B=4, C=16, S=128, seed=0):
    """debug_suite.py:16-24 recipe on SURVEY 8(d) config-1 inputs."""
    g = torch.Generator().manual_seed(seed)
    x = (0.5 + torch.randn(B, C, S, S, generator=g) / 6).clamp(0, 1)
    masks = (torch.rand(B, 1, 32, 32, generator=g) > 0.5).float()
    labels = torch.tensor([0, 1, 2, 3])[:B]
    return x, masks, labels


def _config1_pair(seed=5):
    P = _config1_params()
    torch.manual_seed(seed)
    enc = MM.initialize_model(MM.ModelMaskHeadBackbone("dwi", P, None), True)
    _randomize_bn(enc, seed)
    ref = OM.ModelMaskHeadBackbone("dwi", P, None)
    ref.load_state_dict(enc.state_dict())
    MM.set_compute_dtype(enc, torch.float32)
    return enc.to(DEV), ref, P


def test_config1_no_backbone_train_and_val_step():
    enc, ref, P = _config1_pair()
    assert not hasattr(enc, "backbone_adapter") and enc.block1.bottlenecks[0][0].in_channels == 16
    ref64 = copy.deepcopy(ref).double()
    train_labels = torch.arange(4) % 4
    crit = get_classification_loss(P, train_labels, "dwi", DEV)
    lm = TR.LightningSingleModel(model=enc, method="dwi", criterion_clf=crit, parameters_dict=P)
    cw = OL.class_weights_from_labels(train_labels)
    x, masks, labels = _config1_batch()
    # ---- one train step (train.py:294-428)
    for m in (lm, ref, ref64):
        m.train()
    loss = lm.training_step((x.to(DEV), masks.to(DEV), labels.to(DEV)))
    loss.backward()
    r = OL.single_shared_step(ref, (x, masks, labels), P, cw, "dwi", epoch=0)
    r["total"].backward()
    r64 = OL.single_shared_step(ref64, (x.double(), masks.double(), labels), P, cw.double(), "dwi", epoch=0)
    r64["total"].backward()
    assert abs(loss.item() - r["total"].item()) < 1e-4 * max(1, abs(r["total"].item())), (loss.item(), r["total"])
    for k in ("cls", "mask", "recon", "mimic", "feat_norm"):
        got, want = lm.last_metrics[k].item(), r[k].item()
        assert abs(got - want) < 1e-4 * max(1e-2, abs(want)), (k, got, want)
    bad = {}
    # a gradient that is analytically ~0 (a norm's bias feeding another normalisation) has no
    # meaningful relative error: scale by at least 1e-4 of the largest parameter gradient
    floor = 1e-4 * max(p3.grad.float().norm().item() for p3 in ref64.parameters() if p3.grad is not None)
    for (n, p1), (_, p2), (_, p3) in zip(enc.named_parameters(), ref.named_parameters(), ref64.named_parameters()):
        if p3.grad is None:
            continue
        assert p1.grad is not None, n
        truth = p3.grad.float()
        scale = max(1e-12, floor, truth.norm().item())
        e_mine = (p1.grad.float().cpu().reshape(truth.shape) - truth).norm().item() / scale
        e_ref = (p2.grad - truth).norm().item() / scale
        if e_mine > 3 * e_ref + 5e-3:
            bad[n] = (round(e_mine, 5), round(e_ref, 5))
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:10]
    # ---- one val step (eval BN with the running stats the train step left)
    lm.eval()
    ref.eval()
    with torch.no_grad():
        vloss, logits, _, _ = lm._shared_step((x.to(DEV), masks.to(DEV), labels.to(DEV)), 0, "val",
                                              return_preds=True)
        rv = OL.single_shared_step(ref, (x, masks, labels), P, cw, "dwi", epoch=0, phase="val")
    assert (logits.float().cpu() - rv["logits"]).abs().max().item() < 1e-3
    assert abs(vloss.item() - rv["total"].item()) < 1e-4 * max(1, abs(rv["total"].item()))
