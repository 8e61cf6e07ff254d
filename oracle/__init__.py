"""CPU oracle for the DCE x DWI fusion hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker or as
the timed CPU baseline. The product path (the package next to
``include/dmf_hip.h``) never imports it and has no CPU fallback.

PARITY UNPINNED: importing the reference's Python modules was refused by the
environment, the reference ships no tests, fixtures or golden
vectors, and its backbone arithmetic lives in timm (absent, version unpinned).
This oracle is therefore a clean-room fp32 restatement written from the
reference source text, each function citing the file:line it follows.
"""
