#!/usr/bin/env python3
"""Count the torch (non-HIP-library) ops one eager training step issues, by
product call site -- to find stray copies/fills/adds left on the hot path.

    python tools/trace_ops.py [--batch 4] [--size 256] [--mode A]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

WATCH = ("copy_", "clone", "cat", "_to_copy", "fill_", "zero_", "add", "mul", "div", "sum", "mean", "zeros",
         "ones", "full", "stack", "index", "where", "sub", "neg", "pow", "sqrt", "exp", "log", "clamp", "lerp",
         "addcmul", "addcdiv", "empty_like", "new_zeros", "scatter", "gather", "bmm", "mm", "softmax")


class Tracer(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.counts = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        base = str(func.overloadpacket.__name__) if hasattr(func, "overloadpacket") else name
        if any(base.startswith(w) or base.endswith(w) for w in WATCH) and "empty" not in base and "view" not in base:
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if ("foundation_amd" in fr.filename or "bench.py" in fr.filename) and "dmf_native" not in fr.filename:
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno}"
                    break
            if site == "?":
                shp = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)][:2]
                dts = [str(a.dtype).replace("torch.", "") for a in args if isinstance(a, torch.Tensor)][:1]
                site = f"? {shp} {dts}"
            self.counts[(base, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--mode", default="A")
    a = ap.parse_args()
    import parameters as PR
    from dmf_dp import FusionTrainer

    dev = torch.device("cuda", 0)
    P = PR.default_parameters()
    P["dwi_model_parameters"]["input_size"] = a.size
    lm = bench.build(P, dev, torch.bfloat16, a.mode)
    tr = FusionTrainer(lm, world=1, use_graph=False)
    batch = bench.synthetic_batch(a.batch, a.size, dev, 2)
    tr.step(batch)
    torch.cuda.synchronize()
    t = Tracer()
    with t:
        tr.step(batch)
    torch.cuda.synchronize()
    for (op, site), n in sorted(t.counts.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {op:28s} {site}")
    print("total", sum(t.counts.values()))


if __name__ == "__main__":
    main()
