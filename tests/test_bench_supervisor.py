"""bench.py's multi-rank supervisor (CPU, fake rank work): a rung that fails or stalls on any
rank moves every rank to the next execution rung, and only a rung that every rank completed
prints the result line."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fake, hang_s="4"):
    env = dict(os.environ, HIPFM_BENCH_FAKE=fake, HIPFM_BENCH_HANG_S=hang_s)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120, cwd=REPO)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, lines


@pytest.mark.parametrize("fake,rung", [
    ("none:0:fail", "graph+prefetch"),
    ("graph+prefetch:1:fail", "eager+prefetch+fused"),
    ("graph+prefetch:1:fail,eager+prefetch+fused:0:fail", "graph+prefetch+allreduce"),
    ("graph+prefetch:1:fail,eager+prefetch+fused:1:fail,graph+prefetch+allreduce:0:fail",
     "eager+prefetch"),
    ("graph+prefetch:0:hang,eager+prefetch+fused:0:fail,graph+prefetch+allreduce:1:fail,"
     "eager+prefetch:1:fail", "eager"),
])
def test_supervisor_falls_back_and_prints_one_line(fake, rung):
    rc, lines = _run(fake)
    assert rc == 0
    assert len(lines) == 1 and lines[0]["config"]["exec"] == rung and lines[0]["n_gpus"] == 2


@pytest.mark.parametrize("n", [2, 3])
def test_plain_bench_gpus_n_spawns_n_ranks(n):
    """The driver's SCALE shape without a launcher: ``python bench.py --gpus N`` starts N ranks
    itself (torchrun-style env, 127.0.0.1) and prints exactly one line with n_gpus == N."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
    env.update(HIPFM_BENCH_FAKE="none:0:fail", HIPFM_BENCH_HANG_S="20")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "3"],
                       env=env, capture_output=True, text=True, timeout=180, cwd=REPO)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1 and lines[0]["n_gpus"] == n


def test_supervisor_fails_when_every_rung_fails():
    rc, lines = _run("graph+prefetch:0:fail,eager+prefetch+fused:0:fail,graph+prefetch+allreduce:0:fail,"
                     "eager+prefetch:0:fail,eager:1:fail")
    assert rc != 0 and not lines
