#!/usr/bin/env python3
"""GPU data path throughput vs the reference's CPU
transforms restated in oracle/datapath.py (test infrastructure, timed here as
the CPU baseline only): one batch of config-3 volumes -- DWI [14, 256, 256]
(DWINormalize + ADC fit / preprocess) and DCE [6, 256, 256] (Nyul
transform with landmarks fitted on the batch). Prints one JSON line.

    python tools/datapath_bench.py [--batch 32] [--cpu-volumes 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dataset as DS  # noqa: E402
import preprocess_helpers as PH  # noqa: E402

BVALS = [0, 50, 100, 200, 400, 600, 800, 1000, 1200, 1400, 1600, 1800, 2000, 2500]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-volumes", type=int, default=2)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    dwi = (0.5 + torch.randn(a.batch, 14, a.size, a.size, generator=g) / 6).clamp(0.01, 1)
    dce = torch.rand(a.batch, 6, a.size, a.size, generator=g)
    dwi_d, dce_d = dwi.cuda(), dce.cuda()
    norm = DS.DWINormalize(adc=False)
    nyul = PH.NyulStandardizer()
    nyul.fit([dce_d])

    def gpu():
        d = norm(dwi_d)
        adc = PH.compute_adc_map(dwi_d, BVALS, preprocess=True)
        c = nyul.transform(dce_d)
        return d, adc, c

    gpu()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        gpu()
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / a.reps

    from oracle import datapath as OD
    ref = OD.Nyul()
    ref.fit([x.numpy() for x in dce[:a.cpu_volumes]])
    t0 = time.perf_counter()
    for i in range(a.cpu_volumes):
        OD.dwi_normalize(dwi[i], adc=False)
        OD.preprocess_adc(OD.compute_adc_map(dwi[i], BVALS))
        ref.transform(dce[i].numpy())
    tc = (time.perf_counter() - t0) / a.cpu_volumes
    print(json.dumps({
        "metric": "data path volumes/s (DWINormalize + ADC fit + Nyul on one DWI+DCE volume)",
        "gpu_volumes_per_s": round(a.batch / tg, 1), "gpu_ms_per_batch": round(tg * 1e3, 3),
        "cpu_baseline": {"volumes_per_s": round(1 / tc, 3), "cores": torch.get_num_threads(), "kind": "port",
                         "sample": f"{a.cpu_volumes} volumes, reference transforms restated (torch CPU + numpy)"},
        "batch": a.batch, "size": a.size, "data": "synthetic"}))


if __name__ == "__main__":
    main()
