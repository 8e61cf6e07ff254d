"""Training augmentation on the GPU (prepare_single_model.py:107-113;
SURVEY 8(f) rank 1) against oracle/augment.py, the step-by-step restatement
of torchvision's tensor path, on the same seeded parameter draws:

* RandomAffine + flips (one gather, dmf_affine_flip): nearest sampling, so
  the outputs are source pixels -- bit-exact except where a sample
  coordinate sits within float32 rounding of a pixel boundary (the oracle's
  grid goes through a CPU bmm whose summation / FMA use is the BLAS's); the
  mismatch fraction is bounded at 1e-4 of the pixels;
* Resize (antialiased bilinear, dmf_resize_aa): up and down, square and
  not, within 2e-5 (weights in float32 as aten, summation order may differ);
* the whole chain at the BASELINE shape (B=32, 14 x 256 x 256) with identity
  parameters is an exact copy, and the default chain keeps every value a
  source value or 0."""
import pytest
import torch

import dataset as DS
from oracle import augment as OA

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _images(n, c, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(n, c, h // 4 + 1, w // 4 + 1, generator=g)
    x = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
    return x + 0.01 * torch.rand(n, c, h, w, generator=g)


@pytest.mark.parametrize("shape", [(6, 14, 96, 96), (4, 6, 80, 64), (3, 5, 65, 77)])
def test_affine_flip_matches_oracle(shape):
    n, c, h, w = shape
    x = _images(n, c, h, w, sum(shape))
    g1 = torch.Generator().manual_seed(11)
    g2 = torch.Generator().manual_seed(11)
    aug = DS.TrainAugment(min(h, w), generator=g1)
    # no resize in this case: size = the short side keeps the image size only when square
    params = aug.draw(n, h, w)
    y = torch.empty(n, c, h, w, device=DEV)
    import dmf_native as N
    xd = x.to(DEV)
    pd = params.to(DEV)
    N.call("dmf_affine_flip", xd.data_ptr(), n, c, h, w, pd.data_ptr(), y.data_ptr(), N.stream_ptr())
    got = y.cpu()
    want = []
    for i in range(n):
        angle, tr, scale, sh = OA.get_params(h, w, g2)
        m = OA.inverse_affine_matrix([0.0, 0.0], angle, [float(t) for t in tr], scale, sh)
        o = OA.affine_tensor(x[i], m)
        if bool(torch.rand(1, generator=g2) < 0.5):
            o = o.flip(-1)
        if bool(torch.rand(1, generator=g2) < 0.5):
            o = o.flip(-2)
        want.append(o)
    want = torch.stack(want)
    mism = (got != want).float().mean().item()
    print(f"{shape}: mismatch fraction {mism:.2e}, zero fraction {(want == 0).float().mean().item():.3f}")
    assert mism <= 1e-4, mism


@pytest.mark.parametrize("case", [((2, 3, 128, 128), 96), ((2, 3, 64, 64), 96), ((2, 2, 90, 120), 60),
                                  ((1, 4, 256, 256), 256)])
def test_resize_matches_oracle(case):
    (n, c, h, w), size = case
    x = _images(n, c, h, w, h + w)
    got = DS.resize(x.to(DEV), size).cpu()
    want = torch.stack([OA.resize(x[i], size) for i in range(n)])
    assert got.shape == want.shape
    assert (got - want).abs().max().item() <= 2e-5


def test_chain_at_baseline_shape():
    n, c, s = 32, 14, 256
    x = torch.rand(n, c, s, s, device=DEV)
    ident = torch.tensor([[1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0]] * n)
    aug = DS.TrainAugment(s)
    assert torch.equal(aug(x, ident), x)
    both = ident.clone()
    both[:, 6:] = 1.0
    assert torch.equal(aug(x, both), x.flip(-1).flip(-2))
    y = aug(x)  # random parameters: every output is a source value of its plane or the fill
    assert y.shape == x.shape
    torch.cuda.synchronize()
    v = y[0, 0].flatten()
    src = set(x[0, 0].flatten().cpu().tolist())
    assert all(float(t) in src or float(t) == 0.0 for t in v[:: 97].cpu().tolist())
    # with a normalizer at the end (the reference's special_normalizer slot)
    out = DS.TrainAugment(192, normalizer=DS.DWINormalize())(x[:4])
    assert out.shape == (4, c, 192, 192) and torch.isfinite(out).all()
