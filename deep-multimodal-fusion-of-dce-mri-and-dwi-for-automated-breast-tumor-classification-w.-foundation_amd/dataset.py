"""GPU data path -- MI355X build of the reference's ``code/dataset.py``
transforms. Device tensors only (no CPU fallback)."""
from __future__ import annotations

import math

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


# ------------------------------------------------------------ augmentation
def affine_params(degrees, translate, shear, h, w, generator=None):
    """torchvision RandomAffine.get_params + F.affine's matrix for one image
    of size h x w: the four uniform draws (angle, tx, ty, shear_x; scale
    None, a 2-tuple shear draws only x) in torchvision's order on the given
    torch generator (the process-global one when None), then
    _get_inverse_affine_matrix about the centre (centre (0, 0) in centred
    coordinates, scale 1). Returns the 6 floats of the inverse matrix."""
    def uni(a, b):
        return float(torch.empty(1).uniform_(a, b, generator=generator).item())
    lo, hi = (-degrees, degrees) if isinstance(degrees, (int, float)) else degrees
    angle = uni(float(lo), float(hi))
    tx = int(round(uni(-translate[0] * w, translate[0] * w))) if translate is not None else 0
    ty = int(round(uni(-translate[1] * h, translate[1] * h))) if translate is not None else 0
    sx = sy = 0.0
    if shear is not None:
        sh = [-shear, shear] if isinstance(shear, (int, float)) else list(shear)
        sx = uni(sh[0], sh[1])
        if len(sh) == 4:
            sy = uni(sh[2], sh[3])
    rot, sxr, syr = math.radians(angle), math.radians(sx), math.radians(sy)
    a = math.cos(rot - syr) / math.cos(syr)
    b = -math.cos(rot - syr) * math.tan(sxr) / math.cos(syr) - math.sin(rot)
    c = math.sin(rot - syr) / math.cos(syr)
    d = -math.sin(rot - syr) * math.tan(sxr) / math.cos(syr) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m[2] += m[0] * (-tx) + m[1] * (-ty)
    m[5] += m[3] * (-tx) + m[4] * (-ty)
    return m


class TrainAugment:
    """The reference's training transform chain, prepare_single_model.py:107-113:

        RandomAffine(degrees=90, translate=(0.1, 0.1), shear=(0.1, 0.1))
        -> RandomHorizontalFlip() -> RandomVerticalFlip() -> Resize(input_size)
        -> normalizer (DWINormalize / NyulStandardizer)

    applied to a device batch [N, C, H, W] (f32) in one gather launch for
    affine + flips (dmf_affine_flip) and one separable antialiased resize
    (dmf_resize_aa, skipped when the size already matches, as torchvision's
    resize returns the image unchanged). The random parameters are drawn on
    the host per volume in the order the reference's per-item Compose draws
    them (angle, tx, ty, shear_x, hflip, vflip), from ``generator`` (the
    process-global torch generator when None), so a seeded run reproduces
    torchvision's draws."""

    def __init__(self, input_size, normalizer=None, degrees=90, translate=(0.1, 0.1), shear=(0.1, 0.1), p_hflip=0.5,
                 p_vflip=0.5, generator=None):
        self.size = int(input_size)
        self.normalizer = normalizer
        self.degrees, self.translate, self.shear = degrees, translate, shear
        self.p_h, self.p_v = p_hflip, p_vflip
        self.generator = generator

    def draw(self, n, h, w):
        rows = []
        for _ in range(n):
            m = affine_params(self.degrees, self.translate, self.shear, h, w, self.generator)
            hf = float(torch.rand(1, generator=self.generator).item() < self.p_h)
            vf = float(torch.rand(1, generator=self.generator).item() < self.p_v)
            rows.append(m + [hf, vf])
        return torch.tensor(rows, dtype=torch.float32)

    def __call__(self, batch, params=None):
        N.require_cuda(batch)
        if batch.dim() != 4:
            raise ValueError(f"TrainAugment: expected [N, C, H, W], got {tuple(batch.shape)}")
        x = batch.contiguous().float()
        n, c, h, w = x.shape
        if params is None:
            params = self.draw(n, h, w)
        if tuple(params.shape) != (n, 8):
            raise ValueError(f"TrainAugment: params must be [{n}, 8], got {tuple(params.shape)}")
        pd = params.to(device=x.device, dtype=torch.float32, non_blocking=True).contiguous()
        y = torch.empty_like(x)
        N.call("dmf_affine_flip", x.data_ptr(), n, c, h, w, pd.data_ptr(), y.data_ptr(), N.stream_ptr())
        y = resize(y, self.size)
        return self.normalizer(y) if self.normalizer is not None else y


def resize(x, size):
    """torchvision Resize(size) on a device batch [N, C, H, W] f32 (bilinear,
    antialias): the shorter side -> size, the longer int(size * long / short)."""
    N.require_cuda(x)
    n, c, h, w = x.shape
    if h <= w:
        oh, ow = size, int(size * w / h)
    else:
        oh, ow = int(size * h / w), size
    if (oh, ow) == (h, w):
        return x
    x = x.contiguous().float()
    y = torch.empty((n, c, oh, ow), dtype=torch.float32, device=x.device)
    tmp = torch.empty((n, c, h, ow), dtype=torch.float32, device=x.device) if (oh != h and ow != w) else None
    N.call("dmf_resize_aa", x.data_ptr(), n * c, h, w, oh, ow, tmp.data_ptr() if tmp is not None else None,
           y.data_ptr(), N.stream_ptr())
    return y
