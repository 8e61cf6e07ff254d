"""GPU: eval-mode BatchNorm folded into the conv (dmf_ops._eval_fold, knob
"eval_bn_fold"): config 2's inference forward (reference foundation_model.py:
260-267, eval BN) runs every conv -> BN -> act as ONE conv launch with the
folded weight and a bias + activation epilogue, and the Bottleneck conv3s as
the affine pass with a plain (folded-shortcut) residual.

* fp32: the folded forward against the unfolded one (same kernels' f32 forms)
  and against the CPU oracle, 2e-3 of each map's max (test_gpu_configs' bar);
* bf16: each map's relative L2 error against the fp32 oracle within 1.5x the
  unfolded forward's (+5e-3) and under test_gpu_configs' 3e-2 (the folded
  weight is rounded to bf16 as s*W instead of W);
* after one warm-up forward no BN apply / affine / finalize launch remains;
* a training-mode forward moves the running statistics on the device: the next
  eval forward must refold (equal to the unfolded one), and a BatchNorm whose
  training forward was recorded into a captured graph is never folded again.
"""
import pytest
import torch

import dmf_native as N
import dmf_ops as O
from test_gpu_configs import _config2_pair, _dce_volumes

pytestmark = pytest.mark.gpu
DEV = "cuda"
APPLY = ("dmf_bn_apply", "dmf_affine_act", "dmf_bn_finalize", "dmf_bn_finalize_acc")


class _Count:
    def __init__(self):
        self.names = []

    def __enter__(self):
        self._orig = N.call

        def call(name, *args):
            self.names.append(name)
            return self._orig(name, *args)
        N.call = call
        O.N.call = call
        return self

    def __exit__(self, *exc):
        N.call = self._orig
        O.N.call = self._orig


def _frozen(dtype):
    bb, ref = _config2_pair(dtype, seed=3)
    for p in bb.parameters():
        p.requires_grad = False
    return bb.eval(), ref.eval()


def _fwd(bb, x, fold):
    O.set_knobs(eval_bn_fold=fold)
    try:
        with torch.no_grad():
            return [f.float() for f in bb(x)]
    finally:
        O.set_knobs(eval_bn_fold=True)


def test_eval_fold_f32_matches_unfolded_and_oracle():
    bb, ref = _frozen(torch.float32)
    x = _dce_volumes(2, 5, 128, 4)
    got = _fwd(bb, x.to(DEV), True)
    base = _fwd(bb, x.to(DEV), False)
    with torch.no_grad():
        want = ref(x)
    for i, (a, b, w) in enumerate(zip(got, base, want)):
        tol = 2e-3 * max(1.0, w.abs().max().item())
        assert (a.cpu() - w).abs().max().item() < tol, f"C{i + 2} folded vs oracle"
        assert (a - b).abs().max().item() < tol, f"C{i + 2} folded vs unfolded"


def test_eval_fold_bf16_launches_and_error():
    bb, ref = _frozen(torch.bfloat16)
    x = _dce_volumes(4, 5, 128, 5)
    xd = x.to(DEV)
    base = _fwd(bb, xd, False)
    _fwd(bb, xd, True)  # warm: folds and preps every weight once
    with _Count() as c:
        got = _fwd(bb, xd, True)
    left = [n for n in c.names if n in APPLY]
    assert not left, f"eval forward still launches {sorted(set(left))}"
    with torch.no_grad():
        want = ref(x)
    for i, (a, b, w) in enumerate(zip(got, base, want)):
        e_fold = ((a.cpu() - w).norm() / w.norm().clamp_min(1e-12)).item()
        e_base = ((b.cpu() - w).norm() / w.norm().clamp_min(1e-12)).item()
        print(f"C{i + 2}: bf16 relative L2 vs fp32 oracle, folded {e_fold:.3e}, unfolded {e_base:.3e}")
        # one more bf16 rounding per weight (s*W instead of W): the fold stays at the unfolded error level
        assert e_fold < 3e-2 and e_fold <= 1.5 * e_base + 5e-3, (f"C{i + 2}", e_fold, e_base)


def test_eval_fold_follows_training_statistics():
    bb, _ = _frozen(torch.float32)
    x = _dce_volumes(2, 5, 128, 6).to(DEV)
    _fwd(bb, x, True)  # fold cached at the initial statistics
    bb.train()
    with torch.no_grad():
        bb(x * 1.7 + 0.2)  # moves every running mean / var on the device (no torch version bump)
    bb.eval()
    got = _fwd(bb, x, True)
    base = _fwd(bb, x, False)
    for i, (a, b) in enumerate(zip(got, base)):
        assert (a - b).abs().max().item() < 2e-3 * max(1.0, b.abs().max().item()), f"C{i + 2} stale fold"


def test_captured_training_forward_disables_the_fold():
    bb, _ = _frozen(torch.bfloat16)
    x = _dce_volumes(2, 5, 128, 7).to(DEV)
    bb.train()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        bb(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        bb(x)
    g.replay()
    torch.cuda.synchronize()
    bb.eval()
    bns = [m for m in bb.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    assert bns and all(m.__dict__.get("_dmf_svolatile") for m in bns)
    with _Count() as c:
        _fwd(bb, x, True)
    assert any(n in APPLY for n in c.names), "a BatchNorm trained inside a graph was folded"
