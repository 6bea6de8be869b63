"""Fault injection + auto-resume: a run killed mid-training resumes from its last
checkpoint and finishes with the same parameters as an uninterrupted run."""
import os
import subprocess
import sys

import numpy as np
import torch

import hipfm
from hipfm.ckpt.native import CheckpointManager
from hipfm.utils.fault import Watchdog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ, PYTHONPATH=REPO, **(env_extra or {}))
    return subprocess.run([sys.executable, "-m", "hipfm"] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=300)


def test_kill_and_resume_reproduces(tmp_path):
    d = tmp_path / "data"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:5000", "--train_rows", "2048",
                           "--val_rows", "256", "--files", "1"], cwd=REPO)
    base = ["--training_data_dir", str(d), "--val_data_dir", str(d), "--feature_size", "5000",
            "--field_size", "39", "--embedding_size", "4", "--batch_size", "64", "--deep_layers", "16",
            "--dropout", "0.5", "--num_epochs", "1", "--device", "cpu", "--save_checkpoints_steps", "8",
            "--log_steps", "100"]
    ref = _run(base + ["--model_dir", str(tmp_path / "ref")])
    assert ref.returncode == 0, ref.stderr[-2000:]
    crash = _run(base + ["--model_dir", str(tmp_path / "crash")], {"HIPFM_FAULT_STEP": "20"})
    assert crash.returncode == 17                      # injected exit at step 20
    m = CheckpointManager(str(tmp_path / "crash"))
    assert m.latest().endswith("ckpt-16")              # last checkpoint before the fault
    res = _run(base + ["--model_dir", str(tmp_path / "crash")])
    assert res.returncode == 0, res.stderr[-2000:]
    assert "Restoring parameters" in res.stdout
    ra = CheckpointManager(str(tmp_path / "ref"))
    a = ra.load_rank(ra.latest(), 0)
    b = m.load_rank(m.latest(), 0)
    # the checkpoint restores the data position (epoch 0, batch 16): the resumed run trains only
    # batches 16..31 and ends bitwise equal to the uninterrupted run (params, slots, step)
    assert int(a["global_step"]) == 32 and int(b["global_step"]) == 32
    assert "epoch 0 batch 16" in res.stdout
    assert set(a) == set(b)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert ra.load_manifest(ra.latest())["meta"]["data_pos"] == {"epoch": 1, "batch": 0}


def test_watchdog_fires_on_stall():
    code = ("import time,sys; sys.path.insert(0, %r); import hipfm; from hipfm.utils.fault import Watchdog; "
            "w = Watchdog(1.0, rank=3).start(); time.sleep(30)") % REPO
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 86 and "rank 3" in r.stderr
