"""Single-modality training step (reference
train.py:294-466): LightningSingleModel._shared_step on the HIP path (f32
parity mode) against the oracle restatement oracle/losses.py
single_shared_step, sharing one state_dict and one seeded batch.

Tolerances: loss terms within 1e-4 relative (as the fusion step); parameter
gradients judged against a float64 evaluation of the oracle, as in
test_gpu_parity.test_encoder_backward_parity_all_trainable (at B=4, 8x8
backbone maps under a dozen training-mode BNs the fp32 oracle itself is
percent-level away from float64)."""
import copy

import pytest
import torch
import torch.nn.functional as F

import dmf_ops as O
import parameters as PR
import train as TR
from oracle import losses as OL
from selector_helpers import get_classification_loss
from test_gpu_parity import batch, build_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mimic_items_matches_torch(layout, dtype):
    torch.manual_seed(0)
    s = torch.randn(6, 64, 16, 16)
    t = torch.randn(6, 64, 16, 16)
    t[2] = s[2] * 3.0  # cos == 1 -> clamp branch (zero grad for that item)
    sr = s.clone().requires_grad_(True)
    ref = OL.mimic_feat_loss(sr, t)
    ref.backward()
    mf = torch.channels_last if layout == "nhwc" else torch.contiguous_format
    sd = s.to(DEV, dtype).contiguous(memory_format=mf).requires_grad_(True)
    td = t.to(DEV, dtype).contiguous(memory_format=mf)
    out = O.mimic_items(sd, td)
    out.backward()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert abs(out.item() - ref.item()) < tol * max(1.0, abs(ref.item())), (out.item(), ref.item())
    g = sd.grad.float().cpu()
    assert (g - sr.grad).abs().max().item() <= (1e-6 if dtype == torch.float32 else 1e-4) + \
        (1e-4 if dtype == torch.float32 else 2e-2) * sr.grad.abs().max().item()


@pytest.mark.parametrize("phase", ["train", "val"])
def test_single_step_parity(phase):
    P = PR.small_parameters(dropout=0.0)
    enc, ref, P = build_pair(P, "dwi", 14, 61)
    ref64 = copy.deepcopy(ref).double()
    train_labels = torch.arange(64) % 4
    crit = get_classification_loss(P, train_labels, "dwi", DEV)
    lm = TR.LightningSingleModel(model=enc, method="dwi", criterion_clf=crit, optimizer_fn=None,
                                 scheduler_fn=None, parameters_dict=P)
    lm.current_epoch = 3
    for m in (lm, ref, ref64):
        m.train()
    dwi, _, masks, labels = batch(4, 64, 13)
    cw = OL.class_weights_from_labels(train_labels)
    if phase == "val":
        lm.eval()
        ref.eval()
        with torch.no_grad():
            loss, logits, _, _ = lm._shared_step((dwi.to(DEV), masks.to(DEV), labels.to(DEV)), 0, "val",
                                                 return_preds=True)
            r = OL.single_shared_step(ref, (dwi, masks, labels), P, cw, "dwi", epoch=3, phase="val")
        assert (logits.float().cpu() - r["logits"]).abs().max().item() < 1e-3
        assert abs(loss.item() - r["total"].item()) < 1e-4 * max(1, abs(r["total"].item()))
        return
    loss = lm.training_step((dwi.to(DEV), masks.to(DEV), labels.to(DEV)))
    loss.backward()
    r = OL.single_shared_step(ref, (dwi, masks, labels), P, cw, "dwi", epoch=3)
    r["total"].backward()
    r64 = OL.single_shared_step(ref64, (dwi.double(), masks.double(), labels), P, cw.double(), "dwi", epoch=3)
    r64["total"].backward()
    assert abs(loss.item() - r["total"].item()) < 1e-4 * max(1, abs(r["total"].item()))
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


def test_checkpoint_reload_reproduces_logits(tmp_path):
    """run_training.py:123-131 on the device: a Lightning-layout .ckpt written
    from a GPU module and loaded into a differently initialised one gives the
    same eval logits (frozen-weight caches re-prepare on the new versions)."""
    import run_training as RT

    P = PR.small_parameters(dropout=0.0)
    enc, _, P = build_pair(P, "dce", 6, 71)
    lm = TR.LightningSingleModel(model=enc, method="dce", parameters_dict=P)
    for p in lm.parameters():
        p.requires_grad = False
    lm.eval()
    _, dce, _, _ = batch(2, 64, 17)
    with torch.no_grad():
        want, _, _ = lm(dce.to(DEV))
    path = RT.save_checkpoint(lm, str(tmp_path / "best.ckpt"))
    other, _, _ = build_pair(P, "dce", 6, 72)
    for p in other.parameters():
        p.requires_grad = False
    with torch.no_grad():
        before, _, _ = other.eval()(dce.to(DEV))  # warms the weight caches on the old weights
    got_m = TR.LightningSingleModel.load_from_checkpoint(path, map_location=DEV, model=other, method="dce",
                                                         parameters_dict=P).eval()
    with torch.no_grad():
        got, _, _ = got_m(dce.to(DEV))
    assert (before - want).abs().max().item() > 1e-3
    assert torch.equal(got, want)
