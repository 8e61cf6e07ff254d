"""GPU data path -- MI355X build of the reference's ``code/dataset.py``
transforms. Device tensors only (no CPU fallback)."""
from __future__ import annotations

import torch

import dmf_native as N


class DWINormalize:
    """dataset.py:9-41: per image and channel, z-score with the unbiased std
    (clamped at 1e-6), clip to clip_z, map to [0, 1]. With ``adc=True`` the
    last channel is the ADC slot and -- as in the reference, whose output
    starts as zeros_like(img) -- comes out 0 (quirk Q12). Accepts [C, H, W]
    or a batch [N, C, H, W]; one launch for the whole batch."""

    def __init__(self, clip_z=(-3, 3), adc=True):
        self.z_lo, self.z_hi = clip_z
        self.adc = adc

    def __call__(self, img):
        N.require_cuda(img)
        if img.dim() not in (3, 4):
            raise ValueError(f"expected [C,H,W] or [N,C,H,W], got {tuple(img.shape)}")
        xb = (img.unsqueeze(0) if img.dim() == 3 else img).contiguous().float()
        n, c, h, w = xb.shape
        out = torch.empty_like(xb)
        N.call("dmf_dwi_normalize", xb.data_ptr(), n, c, h * w, 1 if self.adc else 0, float(self.z_lo),
               float(self.z_hi), out.data_ptr(), N.stream_ptr())
        return out[0] if img.dim() == 3 else out
