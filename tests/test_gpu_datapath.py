"""GPU data path against the CPU oracle restatements
(oracle/datapath.py): DWINormalize, compute_adc_map (+ preprocess_adc) and
the Nyul standardizer (exact percentiles + np.interp), batched over volumes.
Tolerances: percentiles / Nyul bit-level (<= 1e-6, float64 arithmetic as
numpy), z-score map 1e-5 (torch float32 reductions vs double), ADC 1e-4
relative (float32 logs)."""
import numpy as np
import pytest
import torch

import dataset as DS
import preprocess_helpers as PH
from oracle import datapath as OD

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dwi(n, c, s, seed):
    g = torch.Generator().manual_seed(seed)
    b = torch.linspace(1.0, 0.2, c).view(1, c, 1, 1)
    return ((0.5 + torch.randn(n, c, s, s, generator=g) / 6).clamp(0.01, 1) * b).float()


def test_dwi_normalize_batched():
    x = _dwi(3, 15, 64, 0)
    for adc in (True, False):
        y = DS.DWINormalize(adc=adc)(x.to(DEV)).cpu()
        for i in range(3):
            ref = OD.dwi_normalize(x[i], adc=adc)
            assert torch.allclose(y[i], ref, atol=1e-5), (y[i] - ref).abs().max()
        if adc:
            assert torch.equal(y[:, -1], torch.zeros_like(y[:, -1]))
    # single volume form
    y1 = DS.DWINormalize()(x[1].to(DEV)).cpu()
    assert torch.allclose(y1, OD.dwi_normalize(x[1]), atol=1e-5)


def test_adc_map_and_preprocess():
    bvals = [0, 50, 100, 200, 400, 600, 800, 1000, 1200, 1400, 1600, 1800, 2000, 2500]
    x = _dwi(2, len(bvals), 48, 1)
    a = PH.compute_adc_map(x.to(DEV), bvals).cpu()
    ap = PH.compute_adc_map(x.to(DEV), bvals, preprocess=True).cpu()
    for i in range(2):
        ref = OD.compute_adc_map(x[i], bvals)
        assert torch.allclose(a[i], ref, rtol=1e-4, atol=1e-9), (a[i] - ref).abs().max()
        assert torch.allclose(ap[i], OD.preprocess_adc(ref), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("kind", ["uniform", "ties"])
def test_plane_percentiles_exact(kind):
    g = torch.Generator().manual_seed(2)
    x = torch.rand(2, 3, 37, 53, generator=g)
    if kind == "ties":  # background zeros and repeated values (duplicate landmarks)
        x = torch.where(x < 0.4, torch.zeros_like(x), (x * 8).floor() / 8)
        x[0, 0] = 0.0
    q = [1, 10, 25, 30, 40, 50, 60, 75, 80, 90, 99]
    p = PH.plane_percentiles(x.to(DEV), q).cpu().numpy()
    for i in range(2):
        for c in range(3):
            ref = np.percentile(x[i, c].numpy().flatten(), q)
            assert np.array_equal(p[i, c], ref), (p[i, c], ref)


@pytest.mark.parametrize("kind", ["uniform", "ties"])
def test_nyul_fit_transform(kind):
    g = torch.Generator().manual_seed(3)
    imgs = torch.rand(4, 6, 40, 40, generator=g)
    if kind == "ties":
        imgs = torch.where(imgs < 0.3, torch.zeros_like(imgs), imgs)
    ref = OD.Nyul()
    ref.fit([im.numpy() for im in imgs[:3]])
    gpu = PH.NyulStandardizer()
    gpu.fit([imgs[:3].to(DEV)])
    for c in range(6):
        assert np.allclose(gpu.channel_landmarks[c], ref.channel_landmarks[c], rtol=0, atol=1e-12)
    y = gpu.transform(imgs.to(DEV)).cpu().numpy()
    for i in range(4):
        r = ref.transform(imgs[i].numpy())
        assert np.abs(y[i] - r).max() <= 1e-6, np.abs(y[i] - r).max()
    with pytest.raises(RuntimeError):
        PH.NyulStandardizer().transform(imgs[0].to(DEV))


def test_no_cpu_fallback():
    with pytest.raises(RuntimeError):
        DS.DWINormalize()(torch.rand(3, 8, 8))
