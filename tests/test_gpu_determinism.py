"""GPU: the captured training step is bitwise reproducible.

The production plan at configuration 3's own shape (B=32, S=256, default
widths, bf16, dropout on): one FusionTrainer captures the step, a snapshot of
everything a step mutates is taken (parameters, BN running statistics and
num_batches_tracked, AdamW moments and step counters, the Philox states), and
the same two batches are replayed twice from that snapshot. Losses, every
parameter gradient of the second step, every parameter and every buffer after
it must be BIT-identical between the two replays, in mode A (encoders frozen,
train-mode BN: the fusion backward) and mode B (everything trainable: the
encoders' backward too).

What makes this hold (DESIGN.md "Determinism"): every parameter-gradient
reduction of the step is a fixed-order one -- the fusion LayerNorm / gating
column sums by one owner per column, mask-attention, gated-mix, mimic, token
LayerNorm / LayerScale / bias sums through per-block slab rows summed in row
order (dmf_colsum_f32), the weight gradient through k_wgrad_reduce's slab
order. The BN statistics stay float64 atomic sums of fp32 tile partials: those
are order-free only in practice, not by construction -- a float64 sum of fp32
values is exact while the partials' magnitudes span fewer than ~29 bits (53 - 24),
and rounds (so depends on the atomics' order) beyond that. This test is the
empirical check that the production shapes stay inside that range. The reference's torch CPU LayerNorm / Linear backward
is deterministic in the same sense (model_module.py:745-780, :799-818)."""
import copy

import pytest
import torch

import make_golden as MG
import model_module as MM
import parameters as PR
import train_fusion as TF
from selector_helpers import get_classification_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, S = 32, 256


def _lm(mode):
    P = copy.deepcopy(PR.default_parameters())
    P["backbone_freeze_on_start"] = mode == "A"
    dwi, _ = MG.seeded_encoder(P, "dwi", 14, 91)
    dce, _ = MG.seeded_encoder(P, "dce", 6, 92)
    fm, _ = MG.seeded_fusion(P, 93)
    for m in (dwi, dce, fm):
        MM.set_compute_dtype(m, torch.bfloat16)
    crit = get_classification_loss(P, torch.arange(1024) % 4, "fusion", DEV)
    lm = TF.LightningFusionModel(dwi.to(DEV), dce.to(DEV), fm.to(DEV), P, crit)
    lm.train()
    return lm


def _record(tr, lm, batches):
    losses = [tr.step(b).clone() for b in batches]
    torch.cuda.synchronize()
    return {"loss": torch.stack(losses).cpu(),
            "grads": {n: p.grad.detach().clone() for n, p in lm.named_parameters() if p.grad is not None},
            "params": {n: p.detach().clone() for n, p in lm.named_parameters()},
            "buffers": {n: b.clone() for n, b in lm.named_buffers()}}


def _diff(a, b):
    """names whose tensors are not bit-identical (NaN-aware: compared as raw bytes)."""
    bad = []
    for n in a:
        x, y = a[n], b[n]
        if x.shape != y.shape or not torch.equal(x.reshape(-1).view(torch.uint8), y.reshape(-1).view(torch.uint8)):
            bad.append(n)
    return bad


@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["A", "B"])
def test_captured_step_replays_bitwise(mode):
    from dmf_dp import FusionTrainer

    lm = _lm(mode)
    tr = FusionTrainer(lm, world=1, use_graph=True)
    batches = [tuple(t.to(DEV) for t in MG.volume_batch(B, S, 200 + i)) for i in range(2)]
    tr.capture(batches[0])
    assert tr.captures == 1
    snap = tr._snapshot()
    runs = []
    moved = []
    for _ in range(2):
        tr._restore(snap)
        torch.cuda.synchronize()
        runs.append(_record(tr, lm, batches))
        moved.append(sum(not torch.equal(p.detach(), v) for p, v in snap["params"]))
    assert tr.captures == 1 and tr.eager_steps == 0
    r0, r1 = runs
    assert torch.isfinite(r0["loss"]).all(), r0["loss"]
    # the two steps really trained: parameters moved, and in mode B the encoders got gradients
    assert moved[0] > 0 and moved[0] == moved[1], moved
    enc_grads = [n for n in r0["grads"] if n.startswith(("dwi_model.", "dce_model."))]
    assert (len(enc_grads) > 100) == (mode == "B"), len(enc_grads)
    assert torch.equal(r0["loss"].view(torch.int32), r1["loss"].view(torch.int32)), (r0["loss"], r1["loss"])
    for key in ("grads", "params", "buffers"):
        bad = _diff(r0[key], r1[key])
        assert not bad, (key, len(bad), bad[:10])
    print(f"mode {mode}: losses {r0['loss'].tolist()} bit-identical over two replays; "
          f"{len(r0['grads'])} gradients, {len(r0['params'])} parameters, {len(r0['buffers'])} buffers equal")
