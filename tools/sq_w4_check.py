#!/usr/bin/env python3
"""The 4-wave (128x128 per wave) k_conv_fwd_sq against the 8-wave one on the
square-tile shapes: outputs must be bit-identical (same MFMA accumulation
order per output element), and the BN partial statistics equal to fp32
rounding. Prints max differences; exits non-zero on a mismatch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

import dmf_native as N  # noqa: E402
import dmf_ops as O  # noqa: E402

SHAPES = [(32, 32, 32, 512, 512, 3, 1, 4), (32, 32, 32, 256, 256, 3, 1, 1), (8, 32, 32, 3072, 256, 3, 1, 1),
          (32, 32, 32, 2048, 512, 1, 1, 1), (3, 20, 20, 512, 256, 3, 1, 2)]


def run(shape, w4, stats):
    n, h, w, ci, co, k, st, dl = shape
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(ci, co, k, stride=st, padding=(k // 2) * dl, dilation=dl, bias=False).cuda()
    x = torch.randn(n, ci, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    N.call("dmf_conv_tune", 2, 6)
    N.call("dmf_conv_tune", 15, 1)
    N.call("dmf_conv_tune", 16, w4)
    try:
        with torch.no_grad():
            y, part = O._conv_forward_raw(x, conv.weight, None, O.ConvGeom(conv), (O.WeightCache(), O.WeightCache()),
                                          stats, "none")
        form = N.FORMS.get(N.load().dmf_conv_last_form())
        torch.cuda.synchronize()
    finally:
        N.call("dmf_conv_tune", 16, 0)
        N.call("dmf_conv_tune", 2, 0)
        N.call("dmf_conv_tune", 15, 256)
    return y, part, form


def main():
    bad = 0
    for shp in SHAPES:
        for stats in (False, True):
            y8, p8, f8 = run(shp, 0, stats)
            y4, p4, f4 = run(shp, 1, stats)
            dy = (y8.float() - y4.float()).abs().max().item()
            dp = (p8 - p4).abs().max().item() / max(1e-6, p8.abs().max().item()) if stats else 0.0
            ok = f8 == f4 == "sq" and dy == 0.0 and dp < 1e-5
            bad += not ok
            print(f"{shp} stats={stats} forms {f8}/{f4}: max |dy| {dy:.3e}, stats rel {dp:.2e} {'ok' if ok else 'MISMATCH'}",
                  flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
