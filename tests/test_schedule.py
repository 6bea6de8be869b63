"""The PS recipe's orchestration (reference C29, PS:439-442): ``--schedule ps`` runs
train_and_evaluate(TrainSpec(all epochs), EvalSpec(start_delay_secs, throttle_secs)); evaluation
happens on a freshly saved checkpoint whenever the throttle allows, plus once at the end.  Time
decisions are rank 0's and broadcast: at world 2 both ranks evaluate together (no hang)."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from hipfm.utils.net import free_port
    s = socket.socket()
    s.bind(("127.0.0.1", free_port()))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("data")
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:8000", "--train_rows", "2048",
                           "--val_rows", "256", "--files", "4"], cwd=REPO)
    return str(d)


def _flags(data, md, extra):
    return ["--training_data_dir", data, "--val_data_dir", data, "--model_dir", md,
            "--feature_size", "8000", "--field_size", "39", "--embedding_size", "4",
            "--batch_size", "64", "--deep_layers", "16", "--dropout", "1.0", "--num_epochs", "2",
            "--device", "cpu", "--log_steps", "100", "--schedule", "ps",
            "--save_checkpoints_secs", "100000"] + extra


@pytest.mark.parametrize("world", [1, 2])
def test_ps_schedule_throttled_evaluation(data, tmp_path, world):
    md = str(tmp_path / "m")
    env = dict(os.environ, PYTHONPATH=REPO)
    extra = ["--eval_start_delay_secs", "0", "--eval_throttle_secs", "0", "--time_check_steps", "8"]
    if world == 1:
        cmd = [sys.executable, "-m", "hipfm"] + _flags(data, md, extra)
    else:
        cmd = [sys.executable, "-m", "hipfm.launch", "--nproc_per_node", "2", "--master_port",
               str(_port()), "-m", "hipfm"] + _flags(data, md, extra)
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    steps = 2 * 2048 // (64 * world)
    n_eval = r.stdout.count("auc = ")
    # one throttled evaluation at every time check (throttle 0) + the final one
    assert n_eval == steps // 8 + 1, (n_eval, r.stdout[-2000:])
    idx = json.load(open(os.path.join(md, "hipfm_checkpoint.json")))
    assert idx["latest"] == f"ckpt-{steps}"


def test_ps_schedule_start_delay_skips_evaluation(data, tmp_path):
    """The reference's defaults (start delay 1000 s, throttle 1200 s): a short run evaluates only
    at its end."""
    md = str(tmp_path / "m")
    r = subprocess.run([sys.executable, "-m", "hipfm"] + _flags(data, md, ["--time_check_steps", "4"]),
                       cwd=REPO, env=dict(os.environ, PYTHONPATH=REPO), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("auc = ") == 1
