"""CPU: checkpoint / metrics I/O (reference
run_training.py:93-131, :316-326, :352-407, prepare_single_model.py:214-216).
Lightning-layout .ckpt round trips for the single-modality and the fusion
modules, the reference's state_dict key layout (including the duplicate
``backbone._orig_mod`` / ``backbone_adapter.backbone._orig_mod`` entries),
the legacy model-dict file and the metrics JSON schema."""
import copy
import json
import os

import numpy as np
import pytest
import torch

import foundation_model as FM
import model_module as MM
import parameters as PR
import run_training as RT
import train as TR
import train_fusion as TF
from dmf_optim import FusedAdamW
from selector_helpers import get_classification_loss


def _encoder(P, method, cin, seed):
    torch.manual_seed(seed)
    bb = FM.build_medical_backbone(P, "cpu", method, cin)
    return MM.initialize_model(MM.ModelMaskHeadBackbone(method, P, bb), True)


def _perturb(module):
    with torch.no_grad():
        for p in module.parameters():
            p.add_(1.0)


def test_single_ckpt_round_trip(tmp_path):
    P = copy.deepcopy(PR.small_parameters())
    enc = _encoder(P, "dwi", 14, 1)
    lm = TR.LightningSingleModel(model=enc, method="dwi", parameters_dict=P)
    opt = FusedAdamW(lm.parameters(), lr=1e-4)
    lm.current_epoch, lm.global_step = 7, 123
    path = RT.save_checkpoint(lm, str(tmp_path / "checkpoints" / "best.ckpt"), optimizer=opt)
    ck = RT.read_checkpoint(path)
    keys = list(ck["state_dict"])
    assert any(k.startswith("model.backbone._orig_mod.") for k in keys)
    assert any(k.startswith("model.backbone_adapter.backbone._orig_mod.") for k in keys)
    assert ck["epoch"] == 7 and ck["global_step"] == 123 and len(ck["optimizer_states"]) == 1
    want = {k: v.clone() for k, v in lm.state_dict().items()}
    fresh = _encoder(P, "dwi", 14, 2)
    _perturb(fresh)
    got = TR.LightningSingleModel.load_from_checkpoint(path, model=fresh, method="dwi", parameters_dict=P)
    assert got.current_epoch == 7 and got.global_step == 123
    for k, v in got.state_dict().items():
        assert torch.equal(v, want[k]), k
    RT.load_optimizer_state(FusedAdamW(got.parameters(), lr=1e-4), path)
    # prepare_single_model.py:216 strips every "model." occurrence
    stripped = RT.strip_model_prefix(ck["state_dict"])
    assert "backbone._orig_mod.conv1.weight" in stripped


def test_strict_load_reports_key_mismatch(tmp_path):
    P = copy.deepcopy(PR.small_parameters())
    lm = TR.LightningSingleModel(model=_encoder(P, "dwi", 14, 1), method="dwi", parameters_dict=P)
    path = RT.save_checkpoint(lm, str(tmp_path / "a.ckpt"))
    P2 = copy.deepcopy(PR.small_parameters(channels=(16, 32, 32)))
    with pytest.raises(RuntimeError):
        TR.LightningSingleModel.load_from_checkpoint(path, model=_encoder(P2, "dwi", 14, 1), method="dwi",
                                                     parameters_dict=P2)
    with pytest.raises(FileNotFoundError):
        RT.read_checkpoint(str(tmp_path / "missing.ckpt"))


def test_fusion_ckpt_and_model_dict(tmp_path):
    P = copy.deepcopy(PR.small_parameters())
    dwi, dce = _encoder(P, "dwi", 14, 1), _encoder(P, "dce", 6, 2)
    torch.manual_seed(3)
    fm = MM.FusionModel(P)
    crit = get_classification_loss(P, torch.arange(64) % 4, "fusion", "cpu")
    lm = TF.LightningFusionModel(dwi, dce, fm, P, crit)
    path = RT.save_checkpoint(lm, str(tmp_path / "fusion.ckpt"), epoch=3, global_step=9)
    want = {k: v.clone() for k, v in lm.state_dict().items()}
    d2, c2 = _encoder(P, "dwi", 14, 5), _encoder(P, "dce", 6, 6)
    f2 = MM.FusionModel(P)
    _perturb(f2)
    got = TF.LightningFusionModel.load_from_checkpoint(path, dwi_model=d2, dce_model=c2, fusion_model=f2,
                                                       parameters_dict=P, criterion_clf=crit)
    for k, v in got.state_dict().items():
        assert torch.equal(v, want[k]), k
    md = str(tmp_path / "fusion_model_dict.pth")
    RT.update_model_dict(md, 0, fm, dwi, dce)
    RT.update_model_dict(md, 1, f2, d2, c2)
    loaded = RT.read_checkpoint(md)
    assert sorted(loaded) == ["dce_0", "dce_1", "dwi_0", "dwi_1", "fusion_0", "fusion_1"]
    for k, v in fm.state_dict().items():
        assert torch.equal(loaded["fusion_0"][k], v)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _ref_layout_modules():
    P = copy.deepcopy(PR.small_parameters(dropout=0.0, use_backbone=False))
    dwi = MM.ModelMaskHeadBackbone("dwi", P, None)
    dce = MM.ModelMaskHeadBackbone("dce", P, None)
    fm = MM.FusionModel(P)
    crit = get_classification_loss(P, torch.arange(64) % 4, "fusion", "cpu")
    return P, dict(dwi_model=dwi, dce_model=dce, fusion_model=fm, parameters_dict=P, criterion_clf=crit)


def test_reference_layout_fusion_ckpt_loads_strictly(tmp_path):
    """tests/golden/fusion_reference_layout.ckpt is keyed the way the
    REFERENCE's fusion run writes it (doubly wrapped encoders,
    dwi_model.model.model.*; quirk Q2, run_training.py:66-74, :123-131;
    made by tools/make_golden.py from the oracle). It must load strictly --
    every key mapped, none left over -- with epoch / global_step restored."""
    path = os.path.join(GOLDEN, "fusion_reference_layout.ckpt")
    ck = RT.read_checkpoint(path)
    assert any(k.startswith("dwi_model.model.model.") for k in ck["state_dict"])
    _, kw = _ref_layout_modules()
    got = TF.LightningFusionModel.load_from_checkpoint(path, **kw)
    assert got.current_epoch == 17 and got.global_step == 544
    own = got.state_dict()
    for k, v in ck["state_dict"].items():
        kk = k.replace("_model.model.model.", "_model.")
        assert torch.equal(own[kk], v), k
    # a single-model ckpt in the reference's doubly wrapped layout (model.model.*)
    P, _ = _ref_layout_modules()
    enc = MM.ModelMaskHeadBackbone("dwi", P, None)
    sd = {"model.model." + k: v for k, v in got.dwi_model.state_dict().items()}
    p1 = str(tmp_path / "ref_layout_single.ckpt")
    torch.save({"state_dict": sd, "epoch": 2, "global_step": 5}, p1)
    lm = TR.LightningSingleModel.load_from_checkpoint(p1, model=enc, method="dwi", parameters_dict=P)
    for k, v in got.dwi_model.state_dict().items():
        assert torch.equal(lm.model.state_dict()[k], v), k
    # keys that match nothing still fail loudly
    bad = dict(sd)
    bad["model.model.not_a_layer.weight"] = torch.zeros(1)
    torch.save({"state_dict": bad}, p1)
    with pytest.raises(RuntimeError):
        TR.LightningSingleModel.load_from_checkpoint(p1, model=MM.ModelMaskHeadBackbone("dwi", P, None),
                                                     method="dwi", parameters_dict=P)


def test_metrics_json_schema(tmp_path):
    P = {"save_dir": "lightning_logs", "class_num": 4}
    paths = RT.prepare_output_paths("fusion", 2, P, base_dir=str(tmp_path))
    assert paths["metrics_json"].endswith("fusion/fold_2/metrics.json")
    train = {"train_loss": [torch.tensor(1.5), torch.tensor(1.25)], "val_acc": [0.5]}
    test = {"test_results": [{"test_auc": torch.tensor(0.75)}], "model_preds": np.zeros((2, 4), np.float32),
            "target_labels": None}
    RT.save_metrics(train, test, P, paths["metrics_json"])
    with open(paths["metrics_json"]) as f:
        d = json.load(f)
    assert set(d) == {"train_val_metrics", "test_metrics", "parameters"}
    assert d["train_val_metrics"]["train_loss"] == [1.5, 1.25]
    assert d["test_metrics"]["test_results"][0]["test_auc"] == 0.75
    assert d["test_metrics"]["model_preds"] == [[0.0] * 4] * 2
