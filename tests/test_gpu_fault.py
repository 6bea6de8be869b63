"""Native kill + resume on the GPU: a CLI run on the HIP
path -- epoch 0 streamed and cached in HBM, epoch 1 replayed as captured multi-step graphs with
the next batch's sort prefetched on a side stream -- is killed mid-epoch 1 (injected fault), then
resumed from its last checkpoint.  The resumed run restores tables, optimizer slots, dense state,
the step counter and the data position (it reads epoch 1 from the files, past the trained
batches), and must end BITWISE equal to an uninterrupted run."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
from hipfm.ckpt.native import CheckpointManager  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ, PYTHONPATH=REPO, **(env_extra or {}))
    return subprocess.run([sys.executable, "-m", "hipfm"] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("update", ["lazy", "tf1_dense"])
def test_native_kill_and_resume_bitwise(tmp_path, update):
    d = tmp_path / "data"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "gen_synthetic_criteo.py"),
                           "--out", str(d), "--preset", "total:5000", "--train_rows", "2048",
                           "--val_rows", "256", "--files", "1"], cwd=REPO)
    base = ["--training_data_dir", str(d), "--val_data_dir", str(d), "--feature_size", "5000",
            "--field_size", "39", "--embedding_size", "8", "--batch_size", "64", "--deep_layers", "32,16",
            "--dropout", "0.5,0.5", "--num_epochs", "2", "--device", "cuda", "--save_checkpoints_steps", "8",
            "--graph_steps", "4", "--log_steps", "100", "--sparse_update", update,
            "--export_tf_bundle", "false"]
    ref = _run(base + ["--model_dir", str(tmp_path / "ref")])
    assert ref.returncode == 0, ref.stderr[-3000:]
    crash = _run(base + ["--model_dir", str(tmp_path / "crash")], {"HIPFM_FAULT_STEP": "44"})
    assert crash.returncode == 17, crash.stderr[-3000:]           # injected exit inside epoch 1
    m = CheckpointManager(str(tmp_path / "crash"))
    assert m.latest().endswith("ckpt-40")
    res = _run(base + ["--model_dir", str(tmp_path / "crash")])
    assert res.returncode == 0, res.stderr[-3000:]
    assert "epoch 1 batch 8" in res.stdout
    ra = CheckpointManager(str(tmp_path / "ref"))
    a, b = ra.load_rank(ra.latest(), 0), m.load_rank(m.latest(), 0)
    assert int(a["global_step"]) == int(b["global_step"]) == 64
    assert set(a) == set(b)
    for k in a:
        assert torch.equal(a[k], b[k]), k
