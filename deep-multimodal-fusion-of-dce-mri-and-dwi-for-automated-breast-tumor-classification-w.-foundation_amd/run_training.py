"""Checkpoint / metrics I/O of the reference's ``code/run_training.py``
 -- the pieces that make trained models and results
interchange with the reference; the Lightning Trainer, callbacks and CLI
around them are control plane and out of scope.

- ``save_checkpoint`` / ``load_from_checkpoint``: the Lightning ``.ckpt``
  layout that ``ModelCheckpoint(filename="best")`` writes
  (run_training.py:93-99) and ``LightningSingleModel.load_from_checkpoint``
  reads back (:123-131): ``state_dict`` keyed by the Lightning module's
  attribute paths (``model.backbone._orig_mod...`` for a single model,
  ``dwi_model.model...`` / ``fusion_model...`` for the fusion module), plus
  ``epoch`` / ``global_step`` and the optimizer state. Loads go through
  ``torch.load(weights_only=True)``: nothing in the file is executed.
- ``strip_model_prefix``: the key rewrite of prepare_single_model.py:214-216.
- ``update_model_dict``: the legacy ``fusion_model_dict.pth`` of
  run_training.py:316-326 (``{fusion_k, dwi_k, dce_k}`` state_dicts per fold).
- ``prepare_output_paths`` / ``convert_tensors`` / ``save_metrics``:
  run_training.py:352-407, same folder layout and JSON schema.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

# the .ckpt layout version these files follow (Lightning 2.x top-level keys)
CKPT_LAYOUT_VERSION = "2.0.0"


def save_checkpoint(module, path, optimizer=None, epoch=None, global_step=None, hyper_parameters=None):
    """Write ``module`` (a LightningSingleModel / LightningFusionModel) in the
    Lightning checkpoint layout. Tensors are saved from the device they live
    on (torch.save copies them to host)."""
    optimizer = optimizer if optimizer is not None else getattr(module, "optimizer", None)
    ckpt = {
        "epoch": int(getattr(module, "current_epoch", 0) if epoch is None else epoch),
        "global_step": int(getattr(module, "global_step", 0) if global_step is None else global_step),
        "pytorch-lightning_version": CKPT_LAYOUT_VERSION,
        "state_dict": {k: v.detach() for k, v in module.state_dict().items()},
        "optimizer_states": [optimizer.state_dict()] if optimizer is not None else [],
        "lr_schedulers": [],
        "loops": None,
        "callbacks": {},
    }
    if hyper_parameters is not None:
        ckpt["hyper_parameters"] = hyper_parameters
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    torch.save(ckpt, path)
    return path


def read_checkpoint(path, map_location="cpu"):
    """The checkpoint dict, loaded without executing anything from the file."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"Checkpoint not found: {path}")
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except Exception as e:  # a pickled object the safe loader refuses
        raise RuntimeError(f"{path}: not loadable with weights_only=True ({e})") from e


# The reference's encoders are Lightning-wrapped twice (quirk Q2:
# prepare_single_model.py:198-206 returns a LightningSingleModel that
# run_training.py:66-74 wraps again; the fusion run then holds that
# double-wrapped module as dwi_model / dce_model). Its checkpoints therefore
# key an encoder as ``model.model.<encoder>`` (single run) or
# ``dwi_model.model.model.<encoder>`` (fusion run); the build holds the
# encoder directly (``model.<encoder>`` / ``dwi_model.<encoder>``). A module
# compiled as a whole (parameters["compile"], run_training.py:90-91, :239-241)
# adds a leading ``_orig_mod.``.
REFERENCE_KEY_PREFIXES = (
    ("dwi_model.model.model.", "dwi_model."), ("dce_model.model.model.", "dce_model."),
    ("dwi_model.model.", "dwi_model."), ("dce_model.model.", "dce_model."),
    ("model.model.", "model."),
)


def to_build_keys(state_dict, build_keys):
    """Map a reference-layout state_dict onto the build's key names (keys the
    build already has are kept as they are); returns a new dict."""
    build_keys = set(build_keys)
    out = {}
    for k, v in state_dict.items():
        if k.startswith("_orig_mod.") and k not in build_keys:
            k = k[len("_orig_mod."):]
        if k not in build_keys:
            for src, dst in REFERENCE_KEY_PREFIXES:
                if k.startswith(src) and dst + k[len(src):] in build_keys:
                    k = dst + k[len(src):]
                    break
        if k in out:
            raise RuntimeError(f"checkpoint maps two entries onto {k!r}")
        out[k] = v
    return out


def load_from_checkpoint(cls, checkpoint_path, map_location="cpu", strict=True, **kwargs):
    """``cls.load_from_checkpoint(path, **init_kwargs)`` (run_training.py:123-131):
    build ``cls(**kwargs)``, load the checkpoint's state_dict, restore epoch /
    global_step. Checkpoints written by the reference (doubly wrapped
    encoders, see REFERENCE_KEY_PREFIXES) load as well as the build's own.
    Raises RuntimeError on missing / unexpected keys when strict."""
    ckpt = read_checkpoint(checkpoint_path, map_location)
    sd = ckpt["state_dict"] if isinstance(ckpt, dict) and "state_dict" in ckpt else ckpt
    module = cls(**kwargs)
    sd = to_build_keys(sd, module.state_dict().keys())
    res = module.load_state_dict(sd, strict=strict)
    module.current_epoch = int(ckpt.get("epoch", 0)) if isinstance(ckpt, dict) else 0
    module.global_step = int(ckpt.get("global_step", 0)) if isinstance(ckpt, dict) else 0
    module._load_result = res
    return module


def load_optimizer_state(optimizer, checkpoint_path, index=0):
    ckpt = read_checkpoint(checkpoint_path)
    states = ckpt.get("optimizer_states", [])
    if len(states) <= index:
        raise RuntimeError(f"{checkpoint_path}: no optimizer state #{index}")
    optimizer.load_state_dict(states[index])
    return optimizer


def strip_model_prefix(state_dict):
    """prepare_single_model.py:216: ``k.replace("model.", "")`` on every key
    (every occurrence, as str.replace does)."""
    return {k.replace("model.", ""): v for k, v in state_dict.items()}


def update_model_dict(model_dict_path, fold, fusion_model, dwi_model, dce_model):
    """run_training.py:316-326: add this fold's three state_dicts to the legacy
    model dict file (created when absent)."""
    model_dict = read_checkpoint(model_dict_path) if os.path.exists(model_dict_path) else {}
    model_dict[f"fusion_{fold}"] = fusion_model.state_dict()
    model_dict[f"dwi_{fold}"] = dwi_model.state_dict()
    model_dict[f"dce_{fold}"] = dce_model.state_dict()
    torch.save(model_dict, model_dict_path)
    return model_dict


def prepare_output_paths(method, fold, parameters, base_dir="results"):
    """run_training.py:352-379."""
    root = os.path.join(base_dir, method, f"fold_{fold}")
    paths = {
        "root": root,
        "checkpoints": os.path.join(root, "checkpoints"),
        "logs": os.path.join(root, parameters["save_dir"]),
        "metrics_json": os.path.join(root, "metrics.json"),
        "model_state": os.path.join(root, "model_state_dict.pth"),
    }
    for d in (paths["root"], paths["checkpoints"], paths["logs"]):
        os.makedirs(d, exist_ok=True)
    return paths


def convert_tensors(obj):
    """run_training.py:381-392: tensors / arrays -> (nested) lists or scalars."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu().tolist()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: convert_tensors(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [convert_tensors(v) for v in obj]
    return obj


def save_metrics(train_metrics, test_metrics, parameters, path):
    """run_training.py:394-407: {train_val_metrics, test_metrics, parameters}
    as indented JSON."""
    all_data = {
        "train_val_metrics": convert_tensors(train_metrics),
        "test_metrics": convert_tensors(test_metrics),
        "parameters": parameters,
    }
    with open(path, "w") as f:
        json.dump(all_data, f, indent=4)
    return all_data
