#!/usr/bin/env python3
"""Where autograd accumulates gradients in the mode-B training step: every (node, input slot) that two
or more consumers feed (each extra contribution is one add launch in the backward, the
CUDAFunctor_add kernels of the mode-B timeline). Walks the graph of one forward of bench.build's
mode-B model (no backward run) and prints the accumulation points with their producer names.

    python tools/grad_fanin.py [--mode B]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import bench  # noqa: E402
import parameters as PR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="B")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lm = bench.build(PR.default_parameters(), dev, torch.bfloat16, a.mode, seed=0)
    batch = bench.synthetic_batch(a.batch, 256, dev, 2)
    loss = lm.training_step(batch)
    feeds = collections.Counter()
    names = {}
    seen, stack = set(), [loss.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        for nxt, nr in fn.next_functions:
            if nxt is None:
                continue
            feeds[(id(nxt), nr)] += 1
            names[id(nxt)] = type(nxt).__name__
            stack.append(nxt)
    acc = [(k, c) for k, c in feeds.items() if c > 1 and names[k[0]] != "AccumulateGrad"]
    by = collections.Counter()
    for (fid, nr), c in acc:
        by[names[fid]] += c - 1
    print(f"nodes {len(seen)}, accumulation points {len(acc)}, extra contributions {sum(c - 1 for _, c in acc)}")
    for n, c in by.most_common():
        print(f"  {c:4d}  into {n}")
    leaf = [(k, c) for k, c in feeds.items() if c > 1 and names[k[0]] == "AccumulateGrad"]
    print(f"leaf (parameter) accumulations: {len(leaf)}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
