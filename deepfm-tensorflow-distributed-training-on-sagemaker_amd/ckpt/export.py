"""Servable export + loader (reference C16 / C33).

The reference exports a TF-Serving SavedModel with ``build_raw_serving_input_receiver_fn``
(PS:451-467): ``<servable_model_dir>/<unix_ts>/saved_model.pb + variables/``, signature
``serving_default``: inputs ``feat_ids int64[-1,F]``, ``feat_vals float32[-1,F]``, output
``prob float32[-1]``.  Without TensorFlow we write the same directory layout with

  variables/variables.index + variables.data-00000-of-00001   TF tensor_bundle (tf_bundle.py),
                                                              reference variable names/layouts
  saved_model.json                                            the signature_def + model config
                                                              (a GraphDef-free SavedModel stand-in)

and ``load_servable`` serves it with the native HIP kernels (GPU) or the golden model (CPU).
A real ``saved_model.pb`` needs TensorFlow's GraphDef; that part is out of reach here and is
documented as such (parity unpinned).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import numpy as np
import torch

from .tf_bundle import read_bundle, write_bundle

SIGNATURE = {
    "serving_default": {
        "inputs": {"feat_ids": {"dtype": "int64", "shape": [-1, "F"]},
                   "feat_vals": {"dtype": "float32", "shape": [-1, "F"]}},
        "outputs": {"prob": {"dtype": "float32", "shape": [-1]}},
        "method_name": "tensorflow/serving/predict",
    }
}

_TRAINING_ONLY = ("/Adam", "/Adagrad", "/Momentum", "/Ftrl", "beta1_power", "beta2_power")


def export_servable(variables: Dict[str, torch.Tensor], model_config: dict, servable_dir: str,
                    timestamp: Optional[int] = None) -> str:
    ts = int(time.time()) if timestamp is None else int(timestamp)
    d = os.path.join(servable_dir, str(ts))
    tmp = d + ".tmp"
    os.makedirs(os.path.join(tmp, "variables"), exist_ok=True)
    serve_vars = {k: v for k, v in variables.items() if not is_training_only(k)}
    write_bundle(os.path.join(tmp, "variables", "variables"), serve_vars)
    return finish_servable(tmp, d, model_config)


def is_training_only(name: str) -> bool:
    return any(s in name for s in _TRAINING_ONLY)


def finish_servable(tmp: str, final: str, model_config: dict) -> str:
    """Complete an export whose ``variables/`` bundle is written: saved_model.pb (MetaGraphDef
    with the serving graph and signature, ckpt/saved_model.py), saved_model.json (the same
    signature + model config, read by load_servable), then the atomic rename."""
    from .saved_model import write_saved_model
    sig = json.loads(json.dumps(SIGNATURE))
    F = model_config["field_size"]
    for spec in sig["serving_default"]["inputs"].values():
        spec["shape"] = [-1, F]
    write_saved_model(os.path.join(tmp, "saved_model.pb"), model_config)
    with open(os.path.join(tmp, "saved_model.json"), "w") as f:
        json.dump({"signature_def": sig, "model": model_config, "format": "hipfm-servable-v1",
                   "tags": ["serve"]}, f, indent=1)
    if os.path.exists(final):
        import shutil
        shutil.rmtree(final)
    os.replace(tmp, final)
    return final


def latest_export(servable_dir: str) -> Optional[str]:
    if not os.path.isdir(servable_dir):
        return None
    ts = sorted((int(x) for x in os.listdir(servable_dir) if x.isdigit()))
    return os.path.join(servable_dir, str(ts[-1])) if ts else None


class Servable:
    """predict(feat_ids[N,F], feat_vals[N,F]) -> prob[N] from an exported directory."""

    def __init__(self, export_dir: str, device=None):
        meta = json.load(open(os.path.join(export_dir, "saved_model.json")))
        self.signature = meta["signature_def"]["serving_default"]
        cfg = meta["model"]
        self.F = cfg["field_size"]
        v = {k: torch.from_numpy(a) for k, a in
             read_bundle(os.path.join(export_dir, "variables", "variables")).items()}
        layers = cfg["deep_layers"]
        keep = [1.0] * len(layers)
        if device is not None and torch.device(device).type == "cuda":
            from ..models.deepfm import NativeDeepFM
            self.model = NativeDeepFM(cfg["feature_size"], self.F, cfg["embedding_size"], layers, keep,
                                      batch_size=1024, device=device, init=False)
            self.model.load_tf_params(v)
            self._native = True
        else:
            from ..models.reference import GoldenDeepFM
            self.model = GoldenDeepFM(cfg["feature_size"], self.F, cfg["embedding_size"], layers,
                                      keep, params=v)
            self._native = False

    def predict(self, feat_ids, feat_vals) -> torch.Tensor:
        ids = torch.as_tensor(feat_ids).reshape(-1, self.F)
        vals = torch.as_tensor(feat_vals, dtype=torch.float32).reshape(-1, self.F)
        if self._native:
            dev = self.model.device
            return self.model.predict(ids.to(dev, torch.int32), vals.to(dev)).cpu()
        return self.model.predict(ids, vals)


def load_servable(export_dir: str, device=None) -> Servable:
    return Servable(export_dir, device)
