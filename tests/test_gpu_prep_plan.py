"""Batched conv weight re-layout (dmf_ops.PrepPlan, dmf_conv_weight_prep_multi):
the training steps re-lay-out every trainable conv weight in one launch.

Checked: (1) after each step's batched launch every planned buffer equals a
per-conv dmf_conv_weight_prep of the current weight (bit-exact: same element
mapping, same rounding); (2) three bf16 training steps with the plan follow
the unplanned steps (losses within 1e-3 relative; the BN statistics' float64
atomics make runs differ in the last bits, so not bit for bit); (3) the per-conv
launches disappear from the planned steps; (4) a weight changed in place by
torch after the batched launch is re-prepared (version check); (5) the
batched kernel against torch-written layouts over odd shapes, every mode and
dtype in one launch."""
import copy

import pytest
import torch

import dmf_native as N
import dmf_ops as O
import parameters as PR
import train as TR
from selector_helpers import get_classification_loss
from test_gpu_parity import batch, build_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _single(seed):
    P = PR.small_parameters(dropout=0.0)
    enc, _, P = build_pair(P, "dwi", 14, seed, dtype=torch.bfloat16)
    crit = get_classification_loss(P, torch.arange(64) % 4, "dwi", DEV)
    lm = TR.LightningSingleModel(model=enc, method="dwi", criterion_clf=crit, optimizer_fn=None,
                                 scheduler_fn=None, parameters_dict=P)
    lm.current_epoch = 3
    lm.train()
    return lm


def _run(lm, steps, counter=None):
    from dmf_optim import FusedAdamW
    opt = FusedAdamW([p for p in lm.parameters() if p.requires_grad], lr=1e-3, weight_decay=1e-2)
    dwi, _, masks, labels = batch(4, 64, 13)
    b = (dwi.to(DEV), masks.to(DEV), labels.to(DEV))
    per_step, losses = [], []
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        if counter is not None:
            counter.clear()
        loss = lm.training_step(b)
        loss.backward()
        losses.append(loss.item())
        if counter is not None:
            per_step.append(dict(counter))
        opt.step()
    torch.cuda.synchronize()
    return per_step, losses


def _count_calls(monkeypatch):
    calls = {}
    real = N.call

    def spy(name, *args):
        calls[name] = calls.get(name, 0) + 1
        return real(name, *args)

    monkeypatch.setattr(N, "call", spy)
    return calls


def test_prep_plan_matches_per_conv_and_unplanned_steps(monkeypatch):
    lm_a = _single(71)
    lm_b = copy.deepcopy(lm_a)
    calls = _count_calls(monkeypatch)
    O.PREP.enabled = True
    per_step, la = _run(lm_a, 3, calls)
    # the first step records the plan; later steps re-lay-out in one launch
    assert per_step[0].get("dmf_conv_weight_prep", 0) > 0
    for st in per_step[1:]:
        assert st.get("dmf_conv_weight_prep_multi", 0) == 1, st
        assert st.get("dmf_conv_weight_prep", 0) == 0, st
    # planned buffers == per-conv re-layout of the current weights (prep once more, then compare)
    O.PREP.prep_step(lm_a)
    torch.cuda.synchronize()
    n = 0
    for (ptr, dtype, cinp, mode), e in O.PREP.entries.items():
        w = e.ref()
        if w is None or e.gen != O.PREP.gen:
            continue
        co, ci, kh, kw = w.shape
        ref = torch.empty_like(e.out)
        N.load().dmf_conv_weight_prep(N.dtype_code(dtype), w.data_ptr(), ref.data_ptr(), co, ci, cinp, kh, kw, mode,
                                      N.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(ref, e.out), (tuple(w.shape), mode)
        n += 1
    assert n > 10
    O.PREP.invalidate()
    # the same three steps with the plan off
    O.PREP.enabled = False
    try:
        _, lb = _run(lm_b, 3)
    finally:
        O.PREP.enabled = True
    for x, y in zip(la, lb):
        assert abs(x - y) <= 1e-3 * max(1.0, abs(y)), (la, lb)
    for (na, pa), (_, pb) in zip(lm_a.named_parameters(), lm_b.named_parameters()):
        assert (pa.float() - pb.float()).abs().max().item() <= 1e-2, na


def test_prep_plan_version_check():
    lm = _single(72)
    _run(lm, 2)
    O.PREP.prep_step(lm)
    convs = [m for m in lm.modules() if isinstance(m, torch.nn.Conv2d) and m.weight.requires_grad
             and getattr(m, "_dmf_caches", None) is not None and m.weight.shape[0] > 1 and m.weight.shape[1] > 1]
    conv = convs[len(convs) // 2]
    key = next(k for k, e in O.PREP.entries.items() if e.ref() is conv.weight and k[3] == 0)
    e = O.PREP.entries[key]
    with torch.no_grad():
        conv.weight.mul_(2.0)  # torch in-place update: _version moves
    got = conv._dmf_caches[0].get(conv.weight, key[1], key[2], 0)
    torch.cuda.synchronize()
    co, ci, kh, kw = conv.weight.shape
    ref = torch.empty_like(got)
    N.load().dmf_conv_weight_prep(N.dtype_code(key[1]), conv.weight.data_ptr(), ref.data_ptr(), co, ci, key[2], kh,
                                  kw, 0, N.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert got.data_ptr() == e.out.data_ptr()  # re-prepared into the planned buffer
    O.PREP.invalidate()


# (Cout, Cin, CinP, KH, KW): partial 64x64 tiles on both sides, channel padding, 1x1 / 3x3 / 7x7, and a
# weight longer than one WPREP_SPAN run
WPREP_SHAPES = [(3, 5, 8, 7, 7), (70, 17, 24, 3, 3), (130, 64, 64, 1, 1), (64, 130, 136, 3, 3), (256, 96, 96, 3, 3)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_weight_prep_multi_layouts_vs_torch(dtype):
    """dmf_conv_weight_prep_multi against the layouts written out with torch:
    mode 0 [Cout][KH][KW][CinP], mode 1 [CinP][KH][KW][Cout], mode 2 the same
    with the taps flipped (the data-gradient filter); padded channels zero.
    Every shape and mode in ONE launch, as PrepPlan builds it; bit-exact."""
    import ctypes
    g = torch.Generator().manual_seed(5)
    cases, jobs, blk = [], [], []
    for co, ci, cinp, kh, kw in WPREP_SHAPES:
        w = torch.randn(co, ci, kh, kw, generator=g).to(DEV)
        wp = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, cinp - ci))
        for mode in range(3):
            if mode == 0:
                ref = wp.permute(0, 2, 3, 1)
            else:
                ref = (wp.flip(2, 3) if mode == 2 else wp).permute(1, 2, 3, 0)
            out = torch.full((ref.numel(),), float("nan"), device=DEV).to(dtype)
            j = len(jobs)
            jobs.append(O._WPrepJob(w.data_ptr(), out.data_ptr(), N.dtype_code(dtype), co, ci, cinp, kh, kw, mode, 0))
            if mode == 0:
                blk.extend((j << 40) | s for s in range(0, co * cinp * kh * kw, O.WPREP_SPAN))
            else:
                blk.extend((j << 40) | t for t in range(-(-cinp * kh * kw // 64) * -(-co // 64)))
            cases.append((w, out, ref.to(dtype).contiguous().reshape(-1), (co, ci, cinp, kh, kw, mode)))
    arr = (O._WPrepJob * len(jobs))(*jobs)
    jt = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(DEV)
    bt = torch.tensor(blk, dtype=torch.int64, device=DEV)
    assert ctypes.sizeof(O._WPrepJob) * len(jobs) == jt.numel()
    N.call("dmf_conv_weight_prep_multi", jt.data_ptr(), bt.data_ptr(), len(blk), O._stream())
    torch.cuda.synchronize()
    for _, out, ref, what in cases:
        assert torch.equal(out, ref), what
