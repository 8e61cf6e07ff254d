"""GPU: pipelined mode-A steps (dmf_dp.FusionTrainer.run_pipelined) train
exactly as the sequential captured steps do.

With the encoders frozen (mode A, the reference's state before the unfreeze:
selector_helpers.py:541-584) step k+1's encoder forward depends on nothing step
k computes, so the trainer runs it on its own stream while step k's fusion
forward / backward / AdamW runs. Every step still does all of its work on its
own batch, with the sequential step's dropout masks: from one snapshot, five
different batches through `run_pipelined` and through `for b: trainer.step(b)`
must leave bit-identical parameters, buffers (BN running statistics of the
frozen encoders included), AdamW moments, last loss and Philox state -- the
same bar as tests/test_gpu_determinism.py's replay check.
"""
import pytest
import torch

import make_golden as MG
from test_gpu_determinism import B, S, _diff, _lm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _state(tr, lm):
    import dmf_ops as O

    torch.cuda.synchronize()
    return {"params": {n: p.detach().clone() for n, p in lm.named_parameters()},
            "buffers": {n: b.clone() for n, b in lm.named_buffers()},
            "opt": {f"{i}.{k}": t.clone() for i, st in enumerate(tr.opt.state.values()) for k, t in st.items()
                    if torch.is_tensor(t) and t.is_cuda},
            "rng": {str(k): v.clone() for k, v in O.RNG.states.items()},
            "loss": {"loss": tr.loss.detach().clone().view(1)}}


@pytest.mark.timeout(900)
def test_pipelined_steps_equal_sequential_steps():
    from dmf_dp import FusionTrainer

    lm = _lm("A")
    tr = FusionTrainer(lm, world=1, use_graph=True)
    batches = [tuple(t.to(DEV) for t in MG.volume_batch(B, S, 300 + i)) for i in range(5)]
    tr.capture(batches[0])
    assert tr.pipeline_ok(batches)
    snap = tr._snapshot()

    for b in batches:
        tr.step(b)
    seq = _state(tr, lm)
    steps_seq = lm.global_step

    tr._restore(snap)
    torch.cuda.synchronize()
    tr.run_pipelined(batches)
    pip = _state(tr, lm)
    assert lm.global_step == steps_seq
    assert torch.isfinite(seq["loss"]["loss"]).all()
    moved = sum(not torch.equal(p.detach(), v) for p, v in snap["params"])
    assert moved > 0
    for key in ("loss", "rng", "params", "buffers", "opt"):
        bad = _diff(seq[key], pip[key])
        assert not bad, (key, len(bad), bad[:10])

    # and again from the same snapshot: the pipelined graphs replay (no re-capture), same result
    tr._restore(snap)
    torch.cuda.synchronize()
    pipe = tr._pipe
    tr.run_pipelined(batches)
    assert tr._pipe is pipe
    again = _state(tr, lm)
    for key in ("loss", "rng", "params", "buffers"):
        assert not _diff(pip[key], again[key]), key
    print(f"5 pipelined steps bit-identical to 5 sequential steps: {len(seq['params'])} parameters, "
          f"{len(seq['buffers'])} buffers, loss {seq['loss']['loss'].item():.6f}")


def test_pipeline_refused_when_encoders_train():
    from dmf_dp import FusionTrainer

    lm = _lm("B")
    tr = FusionTrainer(lm, world=1, use_graph=True)
    batches = [tuple(t.to(DEV) for t in MG.volume_batch(4, 64, 310 + i)) for i in range(2)]
    assert not tr.pipeline_ok(batches)
