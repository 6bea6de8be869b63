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


def test_cache_budget_streams_and_trains_identically(dataset, tmp_path):
    """cache_data had no size check (a dataset larger than free HBM would OOM in
    epoch 0).  An epoch that outgrows the cache budget is not cached; every epoch streams from the
    files in the same (once-per-job shuffled) order, so the run ends with exactly the parameters
    of the fully cached run."""
    from hipfm.ckpt.native import CheckpointManager
    out = {}
    for name, budget in (("cached", "-1"), ("streamed", "0")):
        md = str(tmp_path / name)
        res = main(_flags(dataset, md, ["--task_type", "train", "--num_epochs", "2",
                                        "--cache_budget_mb", budget, "--export_tf_bundle", "false"]))
        m = CheckpointManager(md)
        out[name] = (res, m.load_rank(m.latest(), 0))
    (ra, a), (rb, b) = out["cached"], out["streamed"]
    assert ra["global_step"] == rb["global_step"] == 2 * (3000 // 128)
    assert set(a) == set(b)
    # (the CPU golden path is not bitwise run-to-run reproducible: multi-threaded CPU reductions;
    # two identical cached runs differ by ~1e-6 as well)
    for k in a:
        assert torch.allclose(a[k].double(), b[k].double(), rtol=1e-4, atol=1e-5), k


def test_pipeline_cache_budget_overflow_falls_back(tmp_path):
    from hipfm.data import native_io as nio
    from hipfm.data.pipeline import InputPipeline
    rng = np.random.default_rng(0)
    F = 5
    for k in range(2):
        nio.write_examples(str(tmp_path / f"tr-{k}.tfrecords"), rng.random(300).astype(np.float32),
                           rng.integers(0, 50, (300, F)), rng.random((300, F)).astype(np.float32))
    files = sorted(str(p) for p in tmp_path.glob("tr-*"))
    batch_bytes = 64 * F * 8 + 64 * F * 4 + 64 * 4
    small = InputPipeline(files, F, 64, cache=True, cache_budget=3 * batch_bytes, seed=2)
    big = InputPipeline(files, F, 64, cache=True, cache_budget=None, seed=2)
    e0s, e0b = list(small.iter_epoch(0)), list(big.iter_epoch(0))
    assert small.cache_overflow and small.cached_batches == 0 and big.cached_batches == len(e0b) == 9
    e1s, e1b = list(small.iter_epoch(1)), list(big.iter_epoch(1))
    assert not small.from_cache and big.from_cache
    for x, y in zip(e0s + e1s, e0b + e1b):          # same batches, same order, every epoch
        assert all(torch.equal(p, q) for p, q in zip(x, y))
    assert small.field_minmax() is not None and torch.equal(small.field_minmax()[0], big.field_minmax()[0])
