"""Shortcut-gradient hand-off (dmf_ops.GRAD_STASH): a Bottleneck's shortcut
gradient goes to the backward of the conv_bn_act that produced the block
input and is summed there inside dmf_act_bwd_bn_reduce(_acc) (its dy2), in
place of the autograd add of the two gradients of the block input. Two
blocks (identity and projection shortcut) after a producer conv, in fp32,
with the BN statistics arena (the training path: the fused dy2) and without
it (slab path: the explicit add): every parameter and input gradient must
equal the hand-off-free run's."""
import pytest
import torch
import torch.nn as nn

import dmf_ops as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


class Chain(nn.Module):
    def __init__(self, c=64, mid=32):
        super().__init__()
        self.c0, self.b0 = nn.Conv2d(16, c, 3, padding=1, bias=False), nn.BatchNorm2d(c)
        self.c1, self.b1 = nn.Conv2d(c, mid, 1, bias=False), nn.BatchNorm2d(mid)
        self.c2, self.b2 = nn.Conv2d(mid, c, 1, bias=False), nn.BatchNorm2d(c)
        self.c3, self.b3 = nn.Conv2d(c, mid, 1, bias=False), nn.BatchNorm2d(mid)
        self.c4, self.b4 = nn.Conv2d(mid, 2 * c, 1, bias=False), nn.BatchNorm2d(2 * c)
        self.cd, self.bd = nn.Conv2d(c, 2 * c, 1, bias=False), nn.BatchNorm2d(2 * c)
        self.caches = {k: (O.WeightCache(), O.WeightCache()) for k in ("c0", "c1", "c2", "c3", "c4", "cd")}

    def forward(self, x):
        ca = self.caches
        y = O.conv_bn_act(x, self.c0, ca["c0"], self.b0, "relu")                  # producer of block 1's input
        h = O.conv_bn_act(y, self.c1, ca["c1"], self.b1, "relu")
        y = O.conv_bn_act(h, self.c2, ca["c2"], self.b2, "relu", res=y)           # identity shortcut
        h = O.conv_bn_act(y, self.c3, ca["c3"], self.b3, "relu")
        return O.conv_bn_act(h, self.c4, ca["c4"], self.b4, "relu", skip=(y, self.cd, ca["cd"], self.bd))


def _grads(m, x, gout, handoff, arena):
    O.SHORTCUT_HANDOFF = handoff
    try:
        for p in m.parameters():
            p.grad = None
        xg = x.clone().requires_grad_(True)
        if arena:
            with O.bn_scope(m, DEV):
                out = m(xg)
        else:
            out = m(xg)
        (out.float() * gout).sum().backward()
        torch.cuda.synchronize()
        assert not O.GRAD_STASH, "a handed-over gradient was never consumed"
        return [xg.grad.clone()] + [p.grad.clone() for p in m.parameters()]
    finally:
        O.SHORTCUT_HANDOFF = True


@pytest.mark.parametrize("arena", [True, False])
def test_shortcut_handoff_matches_autograd_add(arena):
    torch.manual_seed(5)
    m = Chain().to(DEV).train()
    x = torch.randn(4, 16, 24, 24, device=DEV).contiguous(memory_format=torch.channels_last)
    gout = torch.randn(4, 128, 24, 24, device=DEV)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    ref = _grads(m, x, gout, False, arena)
    m.load_state_dict(state)
    got = _grads(m, x, gout, True, arena)
    for a, b in zip(got, ref):
        scale = b.abs().max().item()
        assert (a - b).abs().max().item() <= 1e-5 * max(scale, 1e-6), (a - b).abs().max().item()


def test_handoff_skipped_when_the_producer_is_pruned():
    """torch.autograd.grad(..., inputs=[h]) runs only the nodes between the loss and h: the shortcut
    producers of both blocks are pruned, so each consumer must hand its shortcut gradient to autograd
    (torch._C._will_engine_execute_node) instead of parking it for a backward that never runs -- nothing
    is left in GRAD_STASH, and the gradient at h equals the hand-off-free run's."""
    torch.manual_seed(6)
    m = Chain().to(DEV).train()
    ca = m.caches
    x = torch.randn(4, 16, 24, 24, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    gout = torch.randn(4, 128, 24, 24, device=DEV)
    state = {k: v.clone() for k, v in m.state_dict().items()}

    def run(handoff):
        m.load_state_dict(state)
        O.SHORTCUT_HANDOFF = handoff
        try:
            y = O.conv_bn_act(x, m.c0, ca["c0"], m.b0, "relu")
            h = O.conv_bn_act(y, m.c1, ca["c1"], m.b1, "relu")
            y = O.conv_bn_act(h, m.c2, ca["c2"], m.b2, "relu", res=y)
            h = O.conv_bn_act(y, m.c3, ca["c3"], m.b3, "relu")
            out = O.conv_bn_act(h, m.c4, ca["c4"], m.b4, "relu", skip=(y, m.cd, ca["cd"], m.bd))
            (g,) = torch.autograd.grad((out.float() * gout).sum(), inputs=[h])
            torch.cuda.synchronize()
            return g
        finally:
            O.SHORTCUT_HANDOFF = True

    ref = run(False)
    got = run(True)
    assert not O.GRAD_STASH, "a shortcut gradient was parked for a pruned producer"
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1e-5 * max(scale, 1e-6)
