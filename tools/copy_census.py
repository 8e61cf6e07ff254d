#!/usr/bin/env python3
"""Where the runtime's copy kernels (__amd_rocclr_copyBuffer) -- or any kernel whose name contains
--match -- sit in one captured step: for the last step window of a rocprofv3 kernel trace, each one with
its queue, duration, grid, neighbours on its queue and whether another queue was busy meanwhile.

    python tools/copy_census.py gpurun_out/TAG/.../run_kernel_trace.csv [--match CUDAFunctor_add]
"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import timeline as T  # noqa: E402

MATCH = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "copyBuffer"
ks = T.load(sys.argv[1])
marks = [i for i, k in enumerate(ks) if "k_input_prep8" in k["name"]]
lo = marks[-4] if len(marks) >= 4 else 0  # last step: two windows (DWI + DCE prep) per forward
win = ks[lo:]
byq = {}
for k in win:
    byq.setdefault(k["q"], []).append(k)
idle = 0.0
for i, k in enumerate(win):
    if MATCH not in k["name"]:
        continue
    q = byq[k["q"]]
    j = q.index(k)
    prev = q[j - 1]["name"][:60] if j else "-"
    nxt = q[j + 1]["name"][:60] if j + 1 < len(q) else "-"
    other = any(o["q"] != k["q"] and o["s"] < k["e"] and o["e"] > k["s"] for o in win)
    if not other:
        idle += (k["e"] - k["s"]) / 1e3
    print(f"q{k['q']} {(k['e'] - k['s']) / 1e3:6.1f}us grid {k['grid']:>8} overlap={int(other)}  after {prev} | before {nxt}")
print(f"{MATCH}: {sum(MATCH in k['name'] for k in win)}, alone on the GPU {idle:.1f} us, window "
      f"{(win[-1]['e'] - win[0]['s']) / 1e3:.1f} us")
