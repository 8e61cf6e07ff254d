"""Test-time prediction (train_fusion.py:445-632): TTA
flips and MC dropout run as ONE batched forward over the replicas.

* predict_tta (eval mode, deterministic): equal to the reference's sequential
  loop -- one forward_from_inputs per flip, softmax, mean / std -- run on the
  same kernels (batch composition must not change a volume's result).
* predict_mc_dropout: the encoders' Dropout modules on and BN in eval
  (mc_enable), module states restored afterwards; with p = 0 it equals the
  plain eval forward (std 0); with p > 0 the replicas draw distinct masks.
* predict_tta_mc: mean over flips of the per-flip MC means.
MC results are random by construction: parity is on these properties, not on
mask bits."""
import pytest
import torch

import bench
import parameters as PR
from train import tta_flip_lr, tta_flip_lrud, tta_flip_ud, tta_id

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lm(dtype=torch.float32, size=64):
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = size
    lm = bench.build(P, torch.device(DEV), dtype, "B", seed=3)
    lm.eval()
    return lm


def test_tta_batched_equals_sequential_loop():
    lm = _lm()
    dwi, dce, _, _ = bench.synthetic_batch(3, 64, DEV, 5)
    mean, std, aux = lm.predict_tta(dwi, dce)
    probs, gates = [], []
    with torch.no_grad():
        for t in (tta_id, tta_flip_lr, tta_flip_ud, tta_flip_lrud):
            logits, _, a = lm.forward_from_inputs(t(dwi), t(dce))
            probs.append(torch.softmax(logits.float(), 1))
            gates.append(a["gating_weights"].float().cpu())
    ps = torch.stack(probs)
    assert torch.allclose(mean, ps.mean(0), atol=1e-5), (mean - ps.mean(0)).abs().max()
    assert torch.allclose(std, ps.std(0), atol=1e-5)
    assert torch.allclose(aux["gating_weights"], torch.stack(gates).mean(0), atol=1e-5)
    assert aux["dwi_aux"] is None and aux["dce_aux"] is None
    # flips matter (the views are not all identical)
    assert std.abs().max().item() > 0


def test_mc_dropout_states_masks_and_p0_identity():
    lm = _lm()
    dwi, dce, _, _ = bench.synthetic_batch(2, 64, DEV, 6)
    with torch.no_grad():
        ref_logits, _, _ = lm.forward_from_inputs(dwi, dce)
    ref = torch.softmax(ref_logits.float(), 1)
    states = {m: m.training for m in lm.modules()}
    mean, std, aux = lm.predict_mc_dropout(dwi, dce, passes=6)
    assert {m: m.training for m in lm.modules()} == states, "module train states not restored"
    assert std.max().item() > 1e-4, "MC passes drew identical dropout masks"
    assert aux["gating_weights"].shape == (2, 2)
    # p = 0: MC collapses to the eval forward
    for m in lm.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    for m in lm.modules():
        if hasattr(m, "p") and isinstance(getattr(m, "p"), float) and not isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    mean0, std0, _ = lm.predict_mc_dropout(dwi, dce, passes=4)
    assert torch.allclose(mean0, ref, atol=1e-5), (mean0 - ref).abs().max()
    assert std0.abs().max().item() < 1e-6


def test_tta_mc_and_predict_custom_modes():
    lm = _lm(torch.bfloat16)
    b = bench.synthetic_batch(2, 64, DEV, 7)
    mean, std, aux = lm.predict_tta_mc(b[0], b[1], passes=3)
    assert mean.shape == (2, 4) and std.shape == (2, 4)
    assert torch.allclose(mean.sum(1), torch.ones(2, device=DEV), atol=1e-4)
    for mode in ("normal", "tta", "mc", "tta_mc"):
        out = lm.predict_custom(b, mode=mode, mc_passes=2)
        assert out is not None
    with pytest.raises(ValueError):
        lm.predict_custom(b, mode="bogus")
