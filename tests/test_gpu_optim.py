"""FusedAdamW checkpoint/resume (reference checkpoints are Lightning .ckpt
files holding torch.optim.AdamW state, run_training.py:93-99 / :123-131):
the state_dict carries a per-parameter 'step', loads into a fresh FusedAdamW
and into torch.optim.AdamW, and a resumed run matches an uninterrupted one.
Also: loading into an optimizer that already stepped rebuilds its device
tables over the loaded moments (no writes into the freed old buffers)."""
import copy

import pytest
import torch

import dmf_optim

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed=3):
    torch.manual_seed(seed)
    return [torch.randn(37, 5), torch.randn(129), torch.randn(4, 3, 3, 3), torch.randn(11)]


def _groups(ps):
    return [{"params": ps[:2], "lr": 1e-3, "weight_decay": 1e-4}, {"params": ps[2:], "lr": 5e-4, "weight_decay": 0.0}]


def _grads(ps, it):
    g = torch.Generator().manual_seed(100 + it)
    return [torch.randn(p.shape, generator=g) for p in ps]


def _run(opt, ps, iters):
    for it in iters:
        for p, g in zip(ps, _grads(ps, it)):
            p.grad = g.to(p.device)
        opt.step()


@pytest.mark.parametrize("target", ["fused_fresh", "fused_stepped", "torch"])
def test_adamw_resume_matches_uninterrupted(target):
    base = _params()
    # uninterrupted: 4 steps
    ref = [torch.nn.Parameter(p.clone().to(DEV)) for p in base]
    o_ref = dmf_optim.FusedAdamW(_groups(ref), eps=1e-8)
    _run(o_ref, ref, range(4))
    # interrupted after 3 steps (the last parameter never gets a grad in step 0)
    a = [torch.nn.Parameter(p.clone().to(DEV)) for p in base]
    o_a = dmf_optim.FusedAdamW(_groups(a), eps=1e-8)
    _run(o_a, a, range(3))
    sd = copy.deepcopy(o_a.state_dict())
    steps = [float(sd["state"][i]["step"]) for i in sorted(sd["state"])]
    assert steps == [3.0, 3.0, 3.0, 3.0], steps
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    if target == "torch":
        o_b = torch.optim.AdamW(_groups(b), eps=1e-8)
    else:
        o_b = dmf_optim.FusedAdamW(_groups(b), eps=1e-8)
        if target == "fused_stepped":  # already has device tables over its own moment buffers
            _run(o_b, b, [50])
            for p, q in zip(b, a):
                p.data.copy_(q.data)
    o_b.load_state_dict(sd)
    _run(o_b, b, [3])
    for x, y in zip(b, ref):
        assert torch.allclose(x.detach(), y.detach(), atol=1e-6, rtol=1e-5), (x - y).abs().max()
    if target != "torch":
        assert set(o_b.step_counts().values()) == {4}


def test_torch_adamw_state_loads_into_fused():
    base = _params(5)
    ref = [torch.nn.Parameter(p.clone().to(DEV)) for p in base]
    o_ref = torch.optim.AdamW(_groups(ref), eps=1e-8)
    _run(o_ref, ref, range(3))
    sd = copy.deepcopy(o_ref.state_dict())
    b = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    o_b = dmf_optim.FusedAdamW(_groups(b), eps=1e-8)
    o_b.load_state_dict(sd)
    _run(o_b, b, [3])
    _run(o_ref, ref, [3])
    for x, y in zip(b, ref):
        assert torch.allclose(x.detach(), y.detach(), atol=1e-6, rtol=1e-5)
