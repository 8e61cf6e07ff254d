"""CPU restatement of the reference's training augmentation -- TEST
INFRASTRUCTURE ONLY (tests/ import it as the checker).

code/prepare_single_model.py:107-113 composes torchvision transforms:
RandomAffine(degrees=90, translate=(0.1, 0.1), shear=(0.1, 0.1)) ->
RandomHorizontalFlip() -> RandomVerticalFlip() -> Resize(input_size).
torchvision is a third-party dependency absent from this image (and unpinned
by the reference, a Colab notebook); this restates its published tensor
code path (torchvision >= 0.15, transforms v1), step by step, with the same
torch primitives it calls:
  RandomAffine.get_params: angle ~ U(-90, 90); tx, ty = int(round(U(-0.1 W,
    0.1 W))), int(round(U(-0.1 H, 0.1 H))); scale 1; shear (0.1, 0.1) -> one
    draw shear_x ~ U(0.1, 0.1), shear_y = 0; each draw torch.empty(1).uniform_;
  F.affine -> _get_inverse_affine_matrix(center=(0, 0), ...) ->
    F_t.affine: theta float32, _gen_affine_grid (linspace base grid, bmm with
    theta^T / (W/2, H/2)), _apply_grid_transform: grid_sample(nearest, zeros,
    align_corners=False) with the mask channel for fill=0;
  RandomHorizontalFlip / RandomVerticalFlip: torch.rand(1) < 0.5 -> flip;
  Resize(int): F.resize -> interpolate(bilinear, antialias=True,
    align_corners=False), unchanged when the size already matches.
Parity unpinned (no torchvision / reference run here)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def get_params(h, w, generator=None, degrees=90.0, translate=(0.1, 0.1), shear=(0.1, 0.1)):
    angle = float(torch.empty(1).uniform_(-degrees, degrees, generator=generator).item())
    max_dx, max_dy = float(translate[0] * w), float(translate[1] * h)
    tx = int(round(torch.empty(1).uniform_(-max_dx, max_dx, generator=generator).item()))
    ty = int(round(torch.empty(1).uniform_(-max_dy, max_dy, generator=generator).item()))
    shear_x = float(torch.empty(1).uniform_(shear[0], shear[1], generator=generator).item())
    return angle, (tx, ty), 1.0, (shear_x, 0.0)


def inverse_affine_matrix(center, angle, translate, scale, shear):
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [x / scale for x in [d, -b, 0.0, -c, a, 0.0]]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def affine_tensor(img, matrix):
    """F_t.affine(img [C, H, W], matrix, nearest, fill=[0]*C)."""
    c, h, w = img.shape
    theta = torch.tensor(matrix, dtype=img.dtype).reshape(1, 2, 3)
    d = 0.5
    base = torch.empty(1, h, w, 3, dtype=theta.dtype)
    base[..., 0].copy_(torch.linspace(-w * 0.5 + d, w * 0.5 + d - 1, steps=w))
    base[..., 1].copy_(torch.linspace(-h * 0.5 + d, h * 0.5 + d - 1, steps=h).unsqueeze_(-1))
    base[..., 2].fill_(1)
    rescaled = theta.transpose(1, 2) / torch.tensor([0.5 * w, 0.5 * h], dtype=theta.dtype)
    grid = base.view(1, h * w, 3).bmm(rescaled).view(1, h, w, 2)
    x = torch.cat((img[None], torch.ones((1, 1, h, w), dtype=img.dtype)), dim=1)
    x = F.grid_sample(x, grid, mode="nearest", padding_mode="zeros", align_corners=False)
    mask = x[:, -1:].expand_as(x[:, :-1]) < 0.5
    out = x[:, :-1].clone()
    out[mask] = 0.0
    return out[0]


def resize(img, size):
    c, h, w = img.shape
    oh, ow = (size, int(size * w / h)) if h <= w else (int(size * h / w), size)
    if (oh, ow) == (h, w):
        return img
    return F.interpolate(img[None], size=(oh, ow), mode="bilinear", align_corners=False, antialias=True)[0]


def train_transform(img, size, generator=None):
    """One image [C, H, W] through the reference's train Compose (minus the
    normalizer); returns (out, params) with params the 8 numbers the build's
    kernel takes (inverse matrix, hflip, vflip)."""
    c, h, w = img.shape
    angle, tr, scale, sh = get_params(h, w, generator)
    m = inverse_affine_matrix([0.0, 0.0], angle, [float(t) for t in tr], scale, sh)
    out = affine_tensor(img, m)
    hf = bool(torch.rand(1, generator=generator) < 0.5)
    if hf:
        out = out.flip(-1)
    vf = bool(torch.rand(1, generator=generator) < 0.5)
    if vf:
        out = out.flip(-2)
    return resize(out, size), m + [float(hf), float(vf)]
