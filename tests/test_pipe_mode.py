"""SageMaker Pipe mode on real FIFOs (reference C05/C31/B4: PipeModeDataset over
/opt/ml/input/data/<channel>_<epoch>, PS:109-111, HVD:103-120,396-405).

A writer thread per FIFO streams TFRecord bytes into ``<channel>_<epoch>`` (like SageMaker does)
while the CLI trains ``num_epochs`` epochs, one FIFO per epoch and per local rank, then rank 0
evaluates the evaluation channel.  Nothing may count records on a stream (a drained FIFO would
leave training with no data or block forever); at world 2 with uneven streams all ranks stop
together at the first rank's end of data."""
import os
import socket
import subprocess
import sys
import threading

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = 39


def _port():
    from hipfm.utils.net import free_port
    s = socket.socket()
    s.bind(("127.0.0.1", free_port()))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(tmp, name, rows, step):
    import hipfm  # noqa: F401
    from hipfm.data.native_io import write_examples
    from hipfm.data.synthetic import make_synth
    ids, vals, lab = make_synth("total:8000", seed=3).batch(rows, step=step)
    p = os.path.join(tmp, name + ".tfrecords")
    write_examples(p, lab.numpy(), ids.numpy(), vals.numpy())
    return open(p, "rb").read()


class _FifoWriter(threading.Thread):
    """Opens a FIFO for writing (blocks until a reader opens it) and streams ``data`` into it."""

    def __init__(self, path, data):
        super().__init__(daemon=True)
        self.path, self.data, self.state = path, data, "waiting"
        os.mkfifo(path)

    def run(self):
        try:
            with open(self.path, "wb") as f:
                self.state = "open"
                for o in range(0, len(self.data), 1 << 16):
                    f.write(self.data[o:o + (1 << 16)])
            self.state = "done"
        except BrokenPipeError:
            self.state = "closed_by_reader"      # the reader stopped early (equal-steps rule)


def _run_cli(tmp, world, channels, streams, epochs):
    root = os.path.join(tmp, "pipes")
    os.makedirs(root)
    writers = {}
    for name, data in streams.items():
        w = _FifoWriter(os.path.join(root, name), data)
        w.start()
        writers[name] = w
    env = dict(os.environ, PYTHONPATH=REPO, HIPFM_PIPE_ROOT=root,
               SM_CHANNELS='[' + ",".join(f'"{c}"' for c in channels) + ']')
    md = os.path.join(tmp, "model")
    cmd = [sys.executable, "-m", "hipfm.launch", "--nproc_per_node", str(world), "--master_port",
           str(_port()), "-m", "hipfm", "--task_type", "train", "--pipe_mode", "1",
           "--enable_data_multi_path", "1", "--model_dir", md, "--feature_size", "8000",
           "--field_size", str(F), "--embedding_size", "4", "--batch_size", "64", "--deep_layers", "16",
           "--dropout", "1.0", "--num_epochs", str(epochs), "--device", "cpu", "--log_steps", "4",
           "--save_checkpoints_secs", "0"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    return r, writers, md


def test_pipe_mode_one_rank_two_epochs(tmp_path):
    tmp = str(tmp_path)
    streams = {"training_0": _records(tmp, "t0", 640, 0), "training_1": _records(tmp, "t1", 640, 1),
               "evaluation_0": _records(tmp, "e0", 256, 9)}
    r, writers, md = _run_cli(tmp, 1, ["evaluation", "training"], streams, epochs=2)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "auc = " in r.stdout
    assert all(w.state == "done" for w in writers.values()), {k: w.state for k, w in writers.items()}
    import json
    assert json.load(open(os.path.join(md, "hipfm_checkpoint.json")))["latest"] == "ckpt-20"


def test_pipe_mode_two_ranks_uneven_streams_stop_together(tmp_path):
    """Rank 0 streams 10 batches per epoch, rank 1 only 9: both stop after 18 steps (the first
    rank's end of data over 2 epochs), nothing hangs, and the evaluation FIFO is read once."""
    tmp = str(tmp_path)
    streams = {"training_0": _records(tmp, "a0", 640, 0), "training_1": _records(tmp, "a1", 640, 1),
               "training-1_0": _records(tmp, "b0", 576, 2), "training-1_1": _records(tmp, "b1", 576, 3),
               "evaluation_0": _records(tmp, "e0", 256, 9)}
    r, writers, md = _run_cli(tmp, 2, ["evaluation", "training", "training-1"], streams, epochs=2)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "auc = " in r.stdout
    states = {k: w.state for k, w in writers.items()}
    assert states["evaluation_0"] == "done" and states["training-1_0"] == "done", states
    assert states["training-1_1"] == "done" and states["training_0"] == "done", states
    assert states["training_1"] in ("done", "closed_by_reader"), states
    import json
    assert json.load(open(os.path.join(md, "hipfm_checkpoint.json")))["latest"] == "ckpt-18"
