#!/usr/bin/env python3
"""Per-block backward diagnosis: every Bottleneck of the backbone (and the
stem) in isolation, fp32 parity mode, HIP path vs the oracle's module on the
same random input / upstream gradient. Prints the worst relative error of
the input grad and of each parameter grad."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import foundation_model as FM  # noqa: E402
import model_module as MM  # noqa: E402
import dmf_ops as O  # noqa: E402
from oracle import model as OM  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return (a.float().cpu().reshape(b.shape) - b).abs().max().item() / max(1e-6, b.abs().max().item())


def check(name, mine, ref, xin, spatial):
    g = torch.Generator().manual_seed(7)
    x = xin.clone()
    xr = x.clone().requires_grad_(True)
    xm = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    ym = mine(xm)
    yr = ref(xr)
    gy = torch.randn(yr.shape, generator=g)
    ym.backward(gy.to(DEV).contiguous(memory_format=torch.channels_last))
    yr.backward(gy)
    out = {"y": rel(ym.detach(), yr.detach()), "dx": rel(xm.grad, xr.grad)}
    for (n, p1), (_, p2) in zip(mine.named_parameters(), ref.named_parameters()):
        out[n] = rel(p1.grad, p2.grad) if p2.grad is not None else -1
    bad = {k: round(v, 5) for k, v in out.items() if v > 2e-3}
    print(f"{name:24s} {tuple(xin.shape)} y={out['y']:.2e} dx={out['dx']:.2e} bad={bad}", flush=True)


def main():
    torch.manual_seed(0)
    bb = FM.ResNet50OS8(14, compute_dtype=torch.float32)
    ob = OM.ResNet50OS8(14)
    ob.load_state_dict(bb.state_dict())
    g = torch.Generator().manual_seed(1)
    for m in bb.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data = 1 + 0.2 * torch.randn(m.weight.shape, generator=g)
            m.bias.data = 0.1 * torch.randn(m.bias.shape, generator=g)
    ob.load_state_dict(bb.state_dict())
    MM.set_compute_dtype(bb, torch.float32)
    bb = bb.to(DEV).train()
    ob.train()
    S = int(os.environ.get("S", "8"))
    B = 2
    cin = 64
    for li in range(1, 5):
        for bi, (blk, rblk) in enumerate(zip(getattr(bb, f"layer{li}"), getattr(ob, f"layer{li}"))):
            hs = S * 2 if li == 1 or (li == 2 and bi == 0) else S
            x = torch.randn(B, cin, hs, hs, generator=g)
            check(f"layer{li}.{bi}", blk, rblk, x, hs)
            cin = rblk.conv3.out_channels


if __name__ == "__main__" and not os.environ.get("FULL"):
    main()


def full():
    import copy as _c
    import parameters as PR
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_parity import batch, build_pair

    P = PR.small_parameters(dropout=0.0)
    enc, ref, _ = build_pair(P, "dwi", 14, 41)
    enc.train()
    ref.train()
    dwi, _, _, _ = batch(2, 64, 3)
    lo, aux, mp = enc(dwi.to(DEV))
    lr_, auxr, mpr = ref(dwi)
    which = os.environ.get("OBJ", "all")
    if which == "logits":
        obj, objr = lo.float().pow(2).sum(), lr_.pow(2).sum()
    elif which == "mask":
        obj, objr = mp.float().mean(), mpr.mean()
    elif which == "f3":
        obj, objr = aux["raw_feats"][2].float().mean(), auxr["raw_feats"][2].mean()
    else:
        obj = lo.float().pow(2).sum() + mp.float().mean() + aux["raw_feats"][2].float().mean()
        objr = lr_.pow(2).sum() + mpr.mean() + auxr["raw_feats"][2].mean()
    ref64 = _c.deepcopy(ref).double()
    l6, a6, m6 = ref64(dwi.double())
    if which == "logits":
        o6 = l6.pow(2).sum()
    elif which == "mask":
        o6 = m6.mean()
    elif which == "f3":
        o6 = a6["raw_feats"][2].mean()
    else:
        o6 = l6.pow(2).sum() + m6.mean() + a6["raw_feats"][2].mean()
    obj.backward()
    objr.backward()
    o6.backward()
    print("objective", which, obj.item(), objr.item(), o6.item())
    print("  name: mine-vs-f64  oracle32-vs-f64")
    for (n, p1), (_, p2), (_, p3) in zip(enc.named_parameters(), ref.named_parameters(), ref64.named_parameters()):
        if p3.grad is None:
            continue
        r1 = rel(p1.grad, p3.grad.float())
        r2 = rel(p2.grad, p3.grad.float())
        if r1 > 2e-3 or r2 > 2e-3:
            print(f"  {n}: {r1:.3e} {r2:.3e} (max {p3.grad.abs().max().item():.3e})")


if __name__ == "__main__" and os.environ.get("FULL"):
    full()
