"""bench.py's multi-rank supervisor (CPU, fake rank work): a rung that fails or stalls on any
rank moves every rank to the next execution rung, and only a rung that every rank completed
prints the result line."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _port():
    from hipfm.utils.net import free_port
    s = socket.socket()
    s.bind(("127.0.0.1", free_port()))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fake, hang_s="4", first_s="20"):
    # first_s: a healthy fake child marks progress within a second; the margin is for a loaded host
    # (the supervisor's per-rung temp dirs fixed the real early fallback: a stale progress file of
    # a recycled pid read as an old mark)
    env = dict(os.environ, HIPFM_BENCH_FAKE=fake, HIPFM_BENCH_HANG_S=hang_s, HIPFM_BENCH_FIRST_S=first_s)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2"]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180, cwd=REPO)
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, lines, time.time() - t0


@pytest.mark.parametrize("fake,rung", [
    ("none:0:fail", "graph+run-routing"),
    ("graph+run-routing:1:fail", "graph+prefetch"),
    ("graph+run-routing:1:stall", "graph+prefetch"),
    ("graph+run-routing:0:hang,graph+prefetch:1:stall", "eager"),
    ("graph+run-routing:1:fail,graph+prefetch:0:fail", "eager"),
])
def test_supervisor_falls_back_and_prints_one_line(fake, rung):
    rc, lines, _ = _run(fake)
    assert rc == 0
    assert len(lines) == 1 and lines[0]["config"]["exec"] == rung and lines[0]["n_gpus"] == 2


def test_worst_case_ladder_fits_the_driver_timeout():
    """hung rungs must hand over to the next one fast enough that the LAST rung still
    runs inside a 600 s driver run.  With the production limits, every rung hanging costs at most
    ladder_budget_s(); a fake run with every rung hung (scaled limits) ends within that bound."""
    import bench
    assert bench.ladder_budget_s() < 400
    names = [n for n, _ in bench.LADDER]
    spec = ",".join(f"{n}:{i % 2}:{'hang' if i % 2 else 'stall'}" for i, n in enumerate(names))
    rc, lines, wall = _run(spec, hang_s="3", first_s="5")
    assert rc != 0 and not lines
    # scaled bound: per rung max(first_s, hang_s) + polling/teardown slack, plus process start-up
    assert wall < len(names) * (5 + 6) + 60, wall


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
    rc, lines, _ = _run("graph+run-routing:0:fail,graph+prefetch:0:fail,eager:1:fail")
    assert rc != 0 and not lines
