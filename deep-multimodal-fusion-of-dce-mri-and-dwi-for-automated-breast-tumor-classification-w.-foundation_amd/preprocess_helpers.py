"""GPU data path -- MI355X build of the reference's ``code/preprocess_helpers.py``
(SURVEY 8(f) rank 1): ADC fit, ADC scaling and the Nyul DCE standardizer on
device tensors, batched over volumes (csrc/datapath.hip).

Same names and argument meaning as the reference; inputs are device tensors
[C, H, W] (one volume, as the reference's Dataset transform sees it) or
[N, C, H, W] (a batch). There is no CPU fallback: CPU tensors raise.
"""
from __future__ import annotations

import numpy as np
import torch

import dmf_native as N


def _planes(x):
    N.require_cuda(x)
    if x.dim() not in (3, 4):
        raise ValueError(f"expected [C,H,W] or [N,C,H,W], got {tuple(x.shape)}")
    xb = x.unsqueeze(0) if x.dim() == 3 else x
    return xb.contiguous().float(), x.dim() == 3


def compute_adc_map(dwi_imgs, bvals, eps=1e-6, preprocess=False):
    """preprocess_helpers.py:133-167: per-pixel least-squares slope of
    log(max(S, eps)) against the b-values, ADC = -slope -> [1, H, W] (or
    [N, 1, H, W] for a batch). ``preprocess=True`` fuses preprocess_adc."""
    xb, single = _planes(dwi_imgs)
    n, c, h, w = xb.shape
    if len(bvals) != c:
        raise ValueError(f"{len(bvals)} b-values for {c} channels")
    b = torch.as_tensor(bvals, dtype=torch.float32).to(xb.device)
    out = torch.empty((n, 1, h, w), dtype=torch.float32, device=xb.device)
    N.call("dmf_adc_map", xb.data_ptr(), n, c, h * w, b.data_ptr(), float(eps), 1 if preprocess else 0,
           out.data_ptr(), N.stream_ptr())
    return out[0] if single else out


def preprocess_adc(adc_map):
    """preprocess_helpers.py:39-49: log1p(max(adc, 0)) -> normalize_adc
    (elementwise plumbing on a [1, H, W] map; the batched path fuses it into
    compute_adc_map(preprocess=True))."""
    return normalize_adc(torch.log1p(adc_map.clamp(min=0)))


def normalize_adc(adc_map):
    """preprocess_helpers.py:33-37."""
    return adc_map.clamp(0, 3e-3) / 3e-3


def zero_to_one_adc(adc_map, adc_min=None, adc_max=None):
    """preprocess_helpers.py:27-31."""
    return ((adc_map - adc_min) / (adc_max - adc_min + 1e-8)).clamp(0, 1)


def plane_percentiles(x, q):
    """np.percentile(plane, q) (method 'linear') of every [H, W] plane of a
    [N, C, H, W] device tensor -> float64 [N, C, len(q)], from exact order
    statistics (multi-target radix select, dmf_plane_select)."""
    xb, _ = _planes(x)
    n, c, h, w = xb.shape
    hw = h * w
    qs = np.true_divide(np.asarray(q, dtype=np.float64), 100)
    vi = (hw - 1) * qs
    lo = np.floor(vi)
    gamma = vi - lo
    lo = lo.astype(np.int64)
    hi = np.minimum(lo + 1, hw - 1)
    lo = np.minimum(lo, hw - 1)
    ranks = np.unique(np.concatenate([lo, hi]))
    if len(ranks) > 64:
        raise ValueError("at most 64 distinct order statistics per plane")
    pos = {int(r): i for i, r in enumerate(ranks)}
    dev = xb.device
    r_t = torch.as_tensor(ranks.astype(np.int32), device=dev)
    lo_t = torch.as_tensor(np.array([pos[int(v)] for v in lo], dtype=np.int32), device=dev)
    hi_t = torch.as_tensor(np.array([pos[int(v)] for v in hi], dtype=np.int32), device=dev)
    g_t = torch.as_tensor(gamma, dtype=torch.float64, device=dev)
    vals = torch.empty((n * c, len(ranks)), dtype=torch.float32, device=dev)
    s = N.stream_ptr()
    N.call("dmf_plane_select", xb.data_ptr(), n * c, hw, r_t.data_ptr(), len(ranks), vals.data_ptr(), s)
    perc = torch.empty((n, c, len(qs)), dtype=torch.float64, device=dev)
    N.call("dmf_plane_percentiles", vals.data_ptr(), len(ranks), lo_t.data_ptr(), hi_t.data_ptr(), g_t.data_ptr(),
           len(qs), n * c, perc.data_ptr(), s)
    return perc


class NyulStandardizer:
    """preprocess_helpers.py:52-129: per-channel average landmarks over a
    training set (fit), then per image: its own percentiles -> average
    landmarks -> linspace(target_range) by two np.interp (transform)."""

    def __init__(self, landmarks=(1, 10, 25, 30, 40, 50, 60, 75, 80, 90, 99), target_range=(0, 1)):
        self.landmarks = list(landmarks)
        self.fitted = False
        self.channel_landmarks = None
        self.standard_scale = np.linspace(target_range[0], target_range[1], len(self.landmarks))

    def fit(self, images, num_channels=6):
        """images: iterable of device tensors [C,H,W] or [N,C,H,W]."""
        acc, count = None, 0
        for img in images:
            p = plane_percentiles(img[:, :num_channels] if img.dim() == 4 else img[:num_channels], self.landmarks)
            s = p.sum(0)
            acc = s if acc is None else acc + s
            count += p.shape[0]
        if not count:
            raise ValueError("NyulStandardizer.fit: no images")
        mean = (acc / count).cpu().numpy()
        self.channel_landmarks = {c: mean[c] for c in range(num_channels)}
        self.fitted = True

    def transform(self, img, num_channels=6):
        if not self.fitted:
            raise RuntimeError("Call fit() first")
        xb, single = _planes(img)
        n, c, h, w = xb.shape
        if num_channels != c:
            raise ValueError(f"num_channels={num_channels} but the image has {c} channels")
        perc = plane_percentiles(xb, self.landmarks)
        dev = xb.device
        avg = torch.as_tensor(np.stack([self.channel_landmarks[k] for k in range(c)]), dtype=torch.float64,
                              device=dev)
        sc = torch.as_tensor(self.standard_scale, dtype=torch.float64, device=dev)
        out = torch.empty_like(xb)
        N.call("dmf_nyul_apply", xb.data_ptr(), n * c, c, h * w, perc.data_ptr(), avg.data_ptr(), sc.data_ptr(),
               len(self.landmarks), out.data_ptr(), N.stream_ptr())
        return out[0] if single else out

    def save(self, path):
        """npz (no pickle) instead of the reference's pickled dict."""
        np.savez(path, landmarks=np.asarray(self.landmarks),
                 channel_landmarks=np.stack([self.channel_landmarks[c] for c in sorted(self.channel_landmarks)]),
                 fitted=np.asarray(self.fitted))

    def load(self, path):
        d = np.load(path if str(path).endswith(".npz") else str(path) + ".npz")
        cl = d["channel_landmarks"]
        self.channel_landmarks = {c: cl[c] for c in range(cl.shape[0])}
        self.fitted = bool(d["fitted"])


def preprocess_dce(dce_tensor, nyul_model, apply_zscore=False):
    """preprocess_helpers.py:4-20 (apply_zscore is off on the reference path)."""
    if apply_zscore:
        raise NotImplementedError("preprocess_dce(apply_zscore=True) is not on the reference path")
    c = dce_tensor.shape[-3]
    return nyul_model.transform(dce_tensor, num_channels=c)
