#!/usr/bin/env python3
"""Find the first module whose forward output is non-finite in the bench
configuration (eager, no graph). Usage: python tools/debug_nan.py [B] [S]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import torch  # noqa: E402

import bench  # noqa: E402


def finite(t):
    if isinstance(t, torch.Tensor):
        return bool(torch.isfinite(t.float()).all().item()) if t.is_floating_point() else True
    if isinstance(t, (list, tuple)):
        return all(finite(x) for x in t)
    if isinstance(t, dict):
        return all(finite(v) for v in t.values())
    return True


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    import parameters as PR
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = S
    lm = bench.build(P, dev, torch.bfloat16, "A")
    bad = []

    def hook(mod, inp, out, name=None):
        if not finite(out) and len(bad) < 10:
            torch.cuda.synchronize()
            bad.append((name, type(mod).__name__, finite(inp)))

    for n, m in lm.named_modules():
        m.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
    tr = FusionTrainer(lm, world=1, use_graph=False)
    batch = bench.synthetic_batch(B, S, dev, 2)
    for step in range(3):
        tr.step(batch)
        torch.cuda.synchronize()
        print("step", step, "loss", tr.loss.item(), flush=True)
        for b in bad:
            print("  non-finite output:", b, flush=True)
        for n, buf in lm.named_buffers():
            if buf.is_floating_point() and not torch.isfinite(buf).all():
                print("  non-finite buffer:", n, flush=True)
                break
        if bad:
            break


if __name__ == "__main__":
    main()
