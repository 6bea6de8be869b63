"""End-to-end on CPU (BASELINE config #1: tiny synthetic libsvm -> TFRecord, single process):
train / eval / infer / export / resume through the flag-compatible CLI."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import hipfm
from hipfm.cli import main
from hipfm.ckpt.export import latest_export, load_servable

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    d = tmp_path_factory.mktemp("syn")
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:20000", "--train_rows", "3000",
                           "--val_rows", "1000", "--test_rows", "300", "--files", "3",
                           "--format", "both"], cwd=REPO)
    return str(d)


def _flags(dataset, model_dir, extra=()):
    return ["--training_data_dir", dataset, "--val_data_dir", dataset, "--model_dir", model_dir,
            "--feature_size", "20000", "--field_size", "39", "--embedding_size", "8",
            "--batch_size", "128", "--deep_layers", "32,16", "--dropout", "0.9,0.9",
            "--learning_rate", "0.005", "--log_steps", "10", "--device", "cpu",
            "--perform_shuffle", "0"] + list(extra)


def test_train_eval_infer_export_resume(dataset, tmp_path):
    md, sd = str(tmp_path / "model"), str(tmp_path / "serve")
    res = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "3",
                                    "--servable_model_dir", sd]))
    assert res["global_step"] == 3 * (3000 // 128)
    assert res["auc"] > 0.68, res             # teacher labels are learnable
    idx = json.load(open(os.path.join(md, "hipfm_checkpoint.json")))
    assert idx["latest"] == f"ckpt-{res['global_step']}"
    # TensorBoard scalars like the Estimator's default hooks: train loss in model_dir, eval in eval/
    from hipfm.utils.tfevents import read_events
    import glob
    ev_train = [e for f in glob.glob(os.path.join(md, "events.out.tfevents.*")) for e in read_events(f)]
    ev_eval = [e for f in glob.glob(os.path.join(md, "eval", "events.out.tfevents.*")) for e in read_events(f)]
    assert ev_train and ev_train[0].get("file_version") == "brain.Event:2"
    assert any("loss" in e["scalars"] for e in ev_train)
    aucs = [e["scalars"]["auc"] for e in ev_eval if "auc" in e["scalars"]]
    assert aucs and abs(aucs[-1] - res["auc"]) < 1e-6
    # eval restores the latest checkpoint and reproduces the final metrics exactly
    ev = main(_flags(dataset, md, ["--task_type", "eval"]))
    assert ev["global_step"] == res["global_step"] and abs(ev["auc"] - res["auc"]) < 1e-9
    # infer -> pred.txt with one "%f" line per test row (PS:445-449)
    inf = main(_flags(dataset, md, ["--task_type", "infer", "--pred_path", str(tmp_path / "p.txt")]))
    lines = open(tmp_path / "p.txt").read().splitlines()
    assert inf["rows"] == 300 and len(lines) == 300 and all(0.0 < float(x) < 1.0 for x in lines)
    # exported servable predicts like the trained model
    s = load_servable(latest_export(sd))
    ids = torch.zeros(4, 39, dtype=torch.long) + torch.arange(39)
    p = s.predict(ids, torch.ones(4, 39))
    assert p.shape == (4,) and torch.all((p > 0) & (p < 1))
    # resume continues from the saved step
    res2 = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "1"]))
    assert res2["global_step"] == res["global_step"] + 3000 // 128


def test_libsvm_input_and_clear_existing_model(dataset, tmp_path):
    md = str(tmp_path / "m")
    os.makedirs(md)
    open(os.path.join(md, "junk"), "w").write("x")
    res = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "1", "--data_format",
                                    "libsvm", "--clear_existing_model", "True", "--optimizer",
                                    "Adagrad", "--sparse_update", "lazy"]))
    assert not os.path.exists(os.path.join(md, "junk"))
    assert res["global_step"] == 3000 // 128 and np.isfinite(res["loss"])


@pytest.mark.parametrize("opt", ["Momentum", "ftrl", "GD"])
def test_all_optimizers_train(dataset, tmp_path, opt):
    res = main(_flags(dataset, str(tmp_path / opt), ["--task_type", "train", "--num_epochs", "1",
                                                     "--optimizer", opt, "--max_steps", "8"]))
    assert res["global_step"] == 8 and np.isfinite(res["loss"])
