"""CPU oracle (test infrastructure only) for the GPU data path, restated from
the reference's text: DWINormalize (code/dataset.py:9-41), compute_adc_map
(code/preprocess_helpers.py:133-167), preprocess_adc / normalize_adc (:33-49)
and NyulStandardizer (:52-120; numpy percentile + interp, as the reference).
Parity unpinned beyond these restatements: the reference ships no fixtures."""
import numpy as np
import torch


def dwi_normalize(img, clip_z=(-3, 3), adc=True):
    """dataset.py:14-41 on one [C, H, W] tensor."""
    z_lo, z_hi = clip_z
    c, _, _ = img.shape
    out = torch.zeros_like(img)
    if adc:
        c -= 1
    for ch in range(c):
        x = img[ch]
        mean = x.mean()
        std = x.std().clamp(min=1e-6)
        x = (x - mean) / std
        x = torch.clamp(x, z_lo, z_hi)
        out[ch] = (x - z_lo) / (z_hi - z_lo)
    return out


def compute_adc_map(dwi_imgs, bvals, eps=1e-6):
    """preprocess_helpers.py:133-167."""
    c, _, _ = dwi_imgs.shape
    b = torch.tensor(bvals, dtype=torch.float32).view(c, 1, 1)
    log_s = torch.log(torch.clamp(dwi_imgs, min=eps))
    mean_b = b.mean()
    mean_log = log_s.mean(dim=0)
    cov = ((b - mean_b) * (log_s - mean_log)).sum(dim=0)
    var = ((b - mean_b) ** 2).sum()
    return (-(cov / (var + eps))).unsqueeze(0)


def preprocess_adc(adc_map):
    """preprocess_helpers.py:33-49."""
    adc = torch.log1p(adc_map.clamp(min=0))
    return adc.clamp(0, 3e-3) / 3e-3


class Nyul:
    """preprocess_helpers.py:52-120 (numpy, per channel)."""

    def __init__(self, landmarks=(1, 10, 25, 30, 40, 50, 60, 75, 80, 90, 99), target_range=(0, 1)):
        self.landmarks = list(landmarks)
        self.standard_scale = np.linspace(target_range[0], target_range[1], len(self.landmarks))
        self.channel_landmarks = None

    def fit(self, images, num_channels=6):
        acc = {c: [] for c in range(num_channels)}
        for img in images:
            for c in range(num_channels):
                acc[c].append(np.percentile(img[c].flatten(), self.landmarks))
        self.channel_landmarks = {c: np.mean(acc[c], axis=0) for c in range(num_channels)}

    def transform(self, img, num_channels=6):
        out = np.zeros_like(img, dtype=np.float32)
        for c in range(num_channels):
            x = img[c]
            orig = np.percentile(x.flatten(), self.landmarks)
            avg = self.channel_landmarks[c]
            mid = np.interp(x.flatten(), orig, avg)
            mid = np.interp(mid, avg, self.standard_scale)
            out[c] = mid.reshape(x.shape)
        return out
