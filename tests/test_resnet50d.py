"""CPU: the resnet50d backbone option (reference foundation_model.py:15-68,
dispatched at :503 for backbone_str 'resnet50d'): timm's ResNet-D at output
stride 8 -- deep stem and avg_down shortcuts -- restated in the product
(foundation_model.ResNet50OS8(variant='resnet50d')) and in the oracle.

* module / state_dict layout: timm's names (``conv1.0 / .1 / .3 / .4 / .6``,
  ``bn1``, ``layerN.0.downsample.1`` = the 1x1 projection, ``.2`` = its BN; the
  pool at ``downsample.0`` has no parameters), identical between the product
  and the oracle so weights interchange;
* the shortcut pools timm's downsample_avg picks at output stride 8: none in
  layer1 (stride 1, dilation 1), AvgPool2d(2, 2) in layer2, AvgPool2dSame(2, 1)
  in the dilated layer3 / layer4;
* the oracle's pool against an explicit loop over the windows (known answers:
  clipped ceil-mode windows divided by their in-range count; 'same' windows with
  the padded zeros counted), odd and even sizes.
The GPU parity of the HIP path is tests/test_gpu_resnet50d.py."""
import copy

import numpy as np
import pytest
import torch

import foundation_model as FM
import parameters as PR
from oracle import model as OM


def _loop_pool(x, s, same):
    n, c, h, w = x.shape
    if same:
        ho, wo = h, w
    else:
        ho = -(-(h - 2) // s) + 1
        wo = -(-(w - 2) // s) + 1
        ho -= (ho - 1) * s >= h
        wo -= (wo - 1) * s >= w
    y = np.zeros((n, c, ho, wo))
    for i in range(ho):
        for j in range(wo):
            vals, cnt = 0.0, 0
            for r in range(2):
                for q in range(2):
                    hi, wi = i * s + r, j * s + q
                    if hi < h and wi < w:
                        vals = vals + x[:, :, hi, wi].double().numpy()
                        cnt += 1
            y[:, :, i, j] = vals / (4 if same else cnt)
    return y


@pytest.mark.parametrize("h,w", [(8, 8), (7, 9), (5, 4)])
@pytest.mark.parametrize("s,same", [(2, False), (1, True)])
def test_oracle_avg_down_known_answers(h, w, s, same):
    torch.manual_seed(h * 10 + w)
    x = torch.randn(2, 3, h, w)
    got = OM.AvgDown(s, same)(x)
    want = _loop_pool(x, s, same)
    assert got.shape == want.shape
    np.testing.assert_allclose(got.double().numpy(), want, rtol=1e-6, atol=1e-6)
    # the product's output-size rule is the same
    import dmf_ops as O
    assert O.avgpool2_out(h, s, same) == want.shape[2] and O.avgpool2_out(w, s, same) == want.shape[3]


def test_resnet50d_layout_matches_oracle_and_timm_names():
    torch.manual_seed(0)
    bb = FM.ResNet50OS8(in_chans=6, variant="resnet50d", compute_dtype=torch.float32)
    ref = OM.ResNet50OS8(6, variant="resnet50d")
    sd, rsd = bb.state_dict(), ref.state_dict()
    assert list(sd) == list(rsd)
    assert all(sd[k].shape == rsd[k].shape for k in sd)
    for k in ("conv1.0.weight", "conv1.1.running_var", "conv1.3.weight", "conv1.4.weight", "conv1.6.weight",
              "bn1.weight", "layer1.0.downsample.1.weight", "layer2.0.downsample.2.running_mean",
              "layer4.0.downsample.1.weight"):
        assert k in sd, k
    assert not any(".downsample.0." in k for k in sd)
    assert tuple(sd["conv1.0.weight"].shape) == (32, 6, 3, 3) and tuple(sd["conv1.6.weight"].shape) == (64, 32, 3, 3)
    assert tuple(sd["layer2.0.downsample.1.weight"].shape) == (512, 256, 1, 1)
    ref.load_state_dict(sd)  # interchangeable
    pools = [getattr(bb, f"layer{i}")[0].downsample[0] for i in range(1, 5)]
    assert isinstance(pools[0], torch.nn.Identity)
    assert (pools[1].stride, pools[1].same) == (2, False)
    assert all((p.stride, p.same) == (1, True) for p in pools[2:])
    assert all(getattr(bb, f"layer{i}")[0].downsample[1].stride == (1, 1) for i in range(1, 5))
    assert bb.layer2[0].conv2.stride == (2, 2) and bb.layer3[0].conv2.dilation == (1, 1)
    assert bb.layer3[1].conv2.dilation == (2, 2) and bb.layer4[1].conv2.dilation == (4, 4)
    assert bb.feature_info.channels() == [256, 512, 1024, 2048] and bb.feature_info.reduction() == [4, 8, 8, 8]


def test_build_medical_backbone_dispatches_resnet50d():
    P = copy.deepcopy(PR.default_parameters())
    P["dwi_model_parameters"]["backbone_str"] = "resnet50d"
    bb = FM.build_medical_backbone(P, "cpu", "dwi", 14)
    assert isinstance(bb, FM.ResNet50OS8) and bb.variant == "resnet50d"
    assert bb.output_dims == [256, 512, 1024, 2048]
    mp = P["dwi_model_parameters"]
    assert mp["backbone_index_lists"] == [[0], [1], [2, 3]] and mp["downsample"] == (True, False, False)
    with pytest.raises(NotImplementedError):
        FM.build_imagenet_backbone(name="resnet101", device="cpu", in_channels=3)
