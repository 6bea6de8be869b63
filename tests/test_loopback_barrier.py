"""The same-device engine's host barrier (csrc/kernels/loopback.hip lb_barrier: the host node
between every group's pack and pull kernels, parallel/loopback.py), exercised on the CPU in real
processes through its host-only self-test entry: thousands of generations with a check word that
no rank may see short of (i + 1) * N after barrier i, and the timeout path -- a stalled rank makes
the waiting ranks time out and poison the shared page, and the late rank then fails fast instead
of hanging."""
import multiprocessing as mp
import os
import time

import pytest

import hipfm  # noqa: F401
from hipfm.ops import _lib

if not _lib.available():
    pytest.skip("kernel library not built (python -m hipfm.ops.build)", allow_module_level=True)


def _rank(path, n, r, timeout_ms, iters, stall_rank, stall_at, stall_ms, q):
    import hipfm  # noqa: F401
    from hipfm.ops import _lib
    lib = _lib.get_lib()
    t0 = time.time()
    while True:
        rc = lib.hfm_lb_barrier_selftest(path.encode(), n, r, 1 if r == 0 else 0, timeout_ms, iters,
                                         stall_rank, stall_at, stall_ms)
        if rc != -1 or r == 0 or time.time() - t0 > 20:
            break
        time.sleep(0.01)                 # (rank 0 has not created the page yet)
    q.put((r, rc))


def _run(n, **kw):
    path = f"/dev/shm/hipfm_lbtest_{os.getpid()}_{n}_{kw.get('stall_ms', 0)}"
    if os.path.exists(path):
        os.unlink(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    args = dict(timeout_ms=60000, iters=2000, stall_rank=-1, stall_at=-1, stall_ms=0)
    args.update(kw)
    ps = [ctx.Process(target=_rank, args=(path, n, r, args["timeout_ms"], args["iters"], args["stall_rank"],
                                          args["stall_at"], args["stall_ms"], q)) for r in range(n)]
    for p in ps:
        p.start()
        if p is ps[0]:
            time.sleep(0.5)              # rank 0 creates the page first
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    if os.path.exists(path):
        os.unlink(path)
    return out


@pytest.mark.parametrize("n", [2, 4])
def test_loopback_barrier_generations(n):
    out = _run(n, iters=3000)
    assert out == {r: 0 for r in range(n)}, out


def test_loopback_barrier_timeout_poisons_and_late_rank_fails_fast():
    t0 = time.time()
    out = _run(3, timeout_ms=300, iters=20, stall_rank=2, stall_at=5, stall_ms=1500)
    assert out[2] == 2, out                      # the late rank finds the page poisoned
    assert {out[0], out[1]} <= {1, 2} and 1 in (out[0], out[1]), out
    assert time.time() - t0 < 60
