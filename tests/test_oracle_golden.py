"""CPU: the oracle against the committed golden vectors (tests/golden,
made by tools/make_golden.py) and against independent numpy restatements of
the reference's criteria (known-answer checks written from loss.py /
train.py / selector_helpers.py as text).

PARITY UNPINNED: the reference could not be imported; these
pin the oracle's own behaviour and its agreement with a second, independent
formulation of each formula."""
import os

import numpy as np
import pytest
import torch

from oracle import losses as OL

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
import make_golden as MG  # noqa: E402  (tools/, on sys.path via conftest)


@pytest.fixture(scope="module")
def L():
    return dict(np.load(os.path.join(GOLD, "losses.npz")))


def _t(a):
    return torch.from_numpy(np.asarray(a))


# ------------------------------------------------------------ numpy restatements
def np_log_softmax(x):
    m = x.max(1, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(1, keepdims=True))


def np_focal(logits, targets, gamma, w):
    """loss.py:157-187 SoftWeightedFocalLoss, restated in numpy (float64)."""
    lp = np_log_softmax(logits.astype(np.float64))
    if targets.ndim == 1:
        targets = np.eye(logits.shape[1])[targets]
    fw = (1 - np.exp(lp)) ** gamma * w[None, :]
    return -(targets * fw * lp).sum(1)


def np_sigmoid(x):
    return 1 / (1 + np.exp(-x.astype(np.float64)))


def test_golden_files_present():
    for f in ("losses.npz", "encoder_small.npz", "fusion_step_small.npz"):
        assert os.path.exists(os.path.join(GOLD, f)), f


def test_class_weights_known_answer(L):
    tl = L["train_labels"]
    counts = np.bincount(tl)
    want = len(tl) / (len(counts) * (counts + 1e-6))
    np.testing.assert_allclose(L["class_weights"], want, rtol=1e-6)
    np.testing.assert_allclose(OL.class_weights_from_labels(_t(tl)).numpy(), want, rtol=1e-6)


def test_label_smoothing_known_answer(L):
    K = L["logits"].shape[1]
    want = np.full(L["logits"].shape, 0.1 / (K - 1))
    want[np.arange(len(L["labels"])), L["labels"]] = 0.9
    np.testing.assert_allclose(L["smooth_targets"], want, rtol=1e-6)
    got = OL.label_smoothing(_t(L["logits"]), _t(L["labels"]), K, 0.1).numpy()
    np.testing.assert_allclose(got, want, rtol=1e-6)


def test_focal_known_answer(L):
    rows = np_focal(L["logits"], L["smooth_targets"], 2.0, L["class_weights"])
    np.testing.assert_allclose(L["focal_rows"], rows, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(L["focal_w"], rows.mean(), rtol=1e-5)
    hard = np_focal(L["logits"], L["labels"], 2.0, L["class_weights"]).mean()
    np.testing.assert_allclose(L["focal_w_hard"], hard, rtol=1e-5)
    got = OL.soft_weighted_focal(_t(L["logits"]), _t(L["smooth_targets"]), 2.0, _t(L["class_weights"]))
    np.testing.assert_allclose(got.numpy(), rows.mean(), rtol=1e-5)


def test_dice_known_answer(L):
    p = np_sigmoid(L["mask_logits"])
    t = L["mask_target"].astype(np.float64)
    inter = (p * t).sum((2, 3))
    union = p.sum((2, 3)) + t.sum((2, 3))
    want = 1 - ((2 * inter + 1e-6) / (union + 1e-6)).mean()
    np.testing.assert_allclose(L["dice"], want, rtol=1e-5)
    bce = np.mean(np.maximum(L["mask_logits"], 0) - L["mask_logits"] * t + np.log1p(np.exp(-np.abs(L["mask_logits"]))))
    d = 2 * (p * t).reshape(4, -1).sum(1) / (p.reshape(4, -1).sum(1) + t.reshape(4, -1).sum(1) + 1e-6)
    np.testing.assert_allclose(L["dice_bce"], bce + 1 - d.mean(), rtol=1e-5)


def _np_bilinear(x, H, W):
    """align_corners=False bilinear upsampling (half-pixel centres, clamped)."""
    n, c, h, w = x.shape

    def idx(o, i):
        s = np.maximum((np.arange(o) + 0.5) * i / o - 0.5, 0)
        i0 = np.minimum(np.floor(s).astype(int), i - 1)
        i1 = np.minimum(i0 + 1, i - 1)
        return i0, i1, s - i0

    y0, y1, fy = idx(H, h)
    x0, x1, fx = idx(W, w)
    a = x[:, :, y0][:, :, :, x0]
    b = x[:, :, y0][:, :, :, x1]
    cc = x[:, :, y1][:, :, :, x0]
    d = x[:, :, y1][:, :, :, x1]
    fy = fy[None, None, :, None]
    fx = fx[None, None, None, :]
    return (a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + cc * fy * (1 - fx) + d * fy * fx)


def test_recon_known_answer(L):
    rec, img = L["recon"].astype(np.float64), L["image"].astype(np.float64)
    up = _np_bilinear(rec, 64, 64)
    want = np.sqrt((np_sigmoid(up) - img) ** 2 + 1e-6).mean()
    np.testing.assert_allclose(L["recon_same"], want, rtol=1e-5)
    up1 = _np_bilinear(rec[:, :1], 64, 64)
    want1 = np.sqrt((np_sigmoid(up1) - img.mean(1, keepdims=True)) ** 2 + 1e-6).mean()
    np.testing.assert_allclose(L["recon_mean"], want1, rtol=1e-5)


def test_mimic_known_answer(L):
    s = L["mimic_s"].reshape(4, -1).astype(np.float64)
    t = L["mimic_t"].reshape(4, -1).astype(np.float64)
    s /= np.maximum(np.linalg.norm(s, axis=1, keepdims=True), 1e-12)
    t /= np.maximum(np.linalg.norm(t, axis=1, keepdims=True), 1e-12)
    want = (1 - np.clip((s * t).sum(1), -1 + 1e-6, 1 - 1e-6)).mean()
    np.testing.assert_allclose(L["mimic"], want, rtol=1e-5)


def test_oracle_reproduces_loss_golden(L):
    got = MG.losses_fixture()
    for k, v in got.items():
        np.testing.assert_allclose(v, L[k], rtol=1e-6, atol=1e-7, err_msg=k)


def test_oracle_reproduces_encoder_golden():
    G = np.load(os.path.join(GOLD, "encoder_small.npz"))
    got = MG.encoder_fixture()
    np.testing.assert_array_equal(got["dwi"], G["dwi"])
    np.testing.assert_allclose(got["logits"], G["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(got["mask_logits"], G["mask_logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(got["raw_feat_sums"], G["raw_feat_sums"], rtol=1e-4, atol=1e-3)


def test_oracle_reproduces_step_golden():
    G = np.load(os.path.join(GOLD, "fusion_step_small.npz"))
    got = MG.step_fixture()
    np.testing.assert_allclose(got["terms"], G["terms"], rtol=1e-5)
    np.testing.assert_allclose(got["logits"], G["logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(got["fusion_grad_norms"], G["fusion_grad_norms"], rtol=1e-3, atol=1e-7)


def test_oracle_reproduces_full_width_resnet_maps():
    """SURVEY 8(c) fixture (5) pins the oracle's ResNet-50 OS8 (B=1, S=64)."""
    import make_golden as MG

    G = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resnet50_os8_maps.npz")))
    _, ref = MG.seeded_backbone(6, 51)
    ref.eval()
    with torch.no_grad():
        feats = ref(MG.backbone_input(1, 6, 64, 52))
    for i, f in enumerate(feats):
        np.testing.assert_allclose(f.numpy(), G[f"C{i + 2}"], rtol=1e-4, atol=1e-5)
