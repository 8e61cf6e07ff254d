"""CPU: the host half of the training augmentation (prepare_single_model.py
:107-113): the build draws torchvision RandomAffine / flip parameters in the
same order, from the same generator, with the same inverse matrix as the
oracle's restatement (oracle/augment.py) -- the GPU gather then only has to
agree on the sampling (tests/test_gpu_augment.py)."""
import torch

import dataset as DS
from oracle import augment as OA


def test_draws_and_matrices_match_oracle():
    for h, w in ((96, 96), (128, 96), (37, 50)):
        g1 = torch.Generator().manual_seed(5)
        g2 = torch.Generator().manual_seed(5)
        ours = DS.TrainAugment(64, generator=g1).draw(7, h, w)
        for i in range(7):
            _, params = OA.train_transform(torch.zeros(1, h, w), 64, generator=g2)
            assert torch.allclose(ours[i], torch.tensor(params, dtype=torch.float32)), (i, ours[i], params)


def test_translation_rounds_half_to_even_and_shear_is_x_only():
    g = torch.Generator().manual_seed(0)
    for _ in range(50):
        angle, (tx, ty), scale, (sx, sy) = OA.get_params(100, 100, g)
        assert -90 <= angle <= 90 and abs(tx) <= 10 and abs(ty) <= 10
        assert scale == 1.0 and abs(sx - 0.1) < 1e-6 and sy == 0.0
    # identity parameters -> identity inverse matrix
    assert DS.affine_params((0.0, 0.0), None, None, 8, 8) == [1.0, -0.0, 0.0, -0.0, 1.0, 0.0]
