"""The streamed input path's device ring protocol (data/pipeline.py ``_DeviceRing``) on the CPU:
a fill thread per epoch writes batches into ring slots, a consumer that looks one batch ahead (the
Estimator / CLI all-epochs generator) trains runs of up to G consecutive batches and releases their
slots.  Across epoch boundaries, short epochs and early exits: no deadlock, and no slot is ever
refilled while the consumer still holds it."""
import queue
import threading

import pytest
import torch

import hipfm  # noqa: F401
from hipfm.data import pipeline as P


class _Ev:                                   # stands in for torch.cuda.Event on the CPU
    def record(self, stream=None):
        pass


@pytest.fixture(autouse=True)
def _cpu_events(monkeypatch):
    monkeypatch.setattr(torch.cuda, "Event", _Ev)


def _producer(ring, n, content, q, stop):
    """One epoch's fill thread: the slot order of ``_DeviceFeeder._fill``."""
    k = ring.start()
    for i in range(n):
        s = k % ring.nslots
        k += 1
        ring.next = k
        w = ring.acquire(s, lambda: stop.is_set())
        if w is P._DeviceRing.STOPPED:
            return
        if stop.is_set():
            ring.giveback(s, w)
            return
        content[s] = (id(q), i)                   # "the copy": the slot now holds batch i
        q.put((s, (id(q), i)))
    q.put(None)


def _all_batches(ring, lengths, content, stop, threads=None):
    """The CLI's all-epochs generator: epoch e + 1's producer starts once epoch e is exhausted."""
    for n in lengths:
        q = queue.Queue()
        th = threading.Thread(target=_producer, args=(ring, n, content, q, stop), daemon=True)
        if threads is not None:
            threads.append(th)
        th.start()
        while True:
            item = q.get(timeout=5)               # (a deadlock surfaces as queue.Empty)
            if item is None:
                break
            yield item
        th.join(timeout=5)


@pytest.mark.parametrize("G,lengths", [(4, [13, 7, 16, 3]), (8, [39, 39, 39]), (3, [1, 2, 10, 5, 6])])
def test_ring_runs_across_epochs_never_overwrite_held_slots(G, lengths):
    ring = P._DeviceRing(2, 3, "cpu", torch.int32, 2 * G)
    content, stop = {}, threading.Event()
    it = _all_batches(ring, lengths, content, stop)
    cur = next(it, None)
    trained = 0
    try:
        while cur is not None:
            run = [cur]
            nxt = next(it, None)
            while len(run) < G and nxt is not None:
                run.append(nxt)
                nxt = next(it, None)
            # "enqueue the run": every slot still holds the batch it was handed out with
            for s, tag in run:
                assert content[s] == tag, (s, content[s], tag)
            if nxt is not None:
                assert content[nxt[0]] == nxt[1]
            trained += len(run)
            ring.release([s for s, _ in run], None)
            cur = nxt
    finally:
        stop.set()
    assert trained == sum(lengths)
    assert all(ring.free)


def test_ring_early_exit_releases_held_slots():
    G = 4
    ring = P._DeviceRing(2, 3, "cpu", torch.int32, 2 * G)
    content, stop, ths = {}, threading.Event(), []
    it = _all_batches(ring, [20], content, stop, ths)
    held = [next(it) for _ in range(G + 1)]          # a run plus the look-ahead batch, never trained
    stop.set()
    for th in ths:                                   # (the feeder joins its fill thread on close)
        th.join(timeout=5)
    assert sum(1 for f in ring.free if not f) >= len(held)
    ring.release_all(None)
    assert all(ring.free)
    # a later epoch of the same pipeline starts on the next run boundary and is not blocked
    stop2 = threading.Event()
    it2 = _all_batches(ring, [5], content, stop2)
    got = [next(it2) for _ in range(5)]
    assert got[0][0] % G == 0
    stop2.set()


@pytest.mark.parametrize("seed", range(6))
def test_ring_random_epochs(seed):
    import random
    rng = random.Random(seed)
    G = rng.choice([2, 3, 4, 5, 8])
    lengths = [rng.randint(1, 3 * G + 2) for _ in range(rng.randint(2, 6))]
    test_ring_runs_across_epochs_never_overwrite_held_slots(G, lengths)


@pytest.mark.parametrize("skip", [1, 5, 9, 16])
def test_ring_skipped_batches_are_released(skip):
    """Resume mid-epoch: the pipeline reads past the first ``skip`` batches and releases their
    slots at once (pipeline._release_unread); the rest of the epoch trains in runs."""
    G = 4
    ring = P._DeviceRing(2, 3, "cpu", torch.int32, 2 * G)
    content, stop = {}, threading.Event()
    it = _all_batches(ring, [skip + 11, 7], content, stop)
    for _ in range(skip):
        s, _ = next(it)
        ring.release([s], None)
    cur, trained = next(it, None), skip
    try:
        while cur is not None:
            run = [cur]
            nxt = next(it, None)
            while len(run) < G and nxt is not None:
                run.append(nxt)
                nxt = next(it, None)
            for s, tag in run:
                assert content[s] == tag
            trained += len(run)
            ring.release([s for s, _ in run], None)
            cur = nxt
    finally:
        stop.set()
    assert trained == skip + 11 + 7


def test_ring_stop_right_after_acquire_gives_the_slot_back():
    """max_batches / close() can set the stop flag between a successful acquire and the copy: the
    fill thread must return that slot, or the next epoch's fill thread waits on it forever."""
    G = 2
    ring = P._DeviceRing(2, 3, "cpu", torch.int32, 2 * G)
    s = ring.start()
    w = ring.acquire(s, lambda: False)            # taken ...
    assert w is not P._DeviceRing.STOPPED and not ring.free[s]
    ring.giveback(s, w)                           # ... and the stop is seen: handed back
    assert all(ring.free)
    # a consumer holds every slot: a stopped acquire returns STOPPED without taking anything
    for k in range(ring.nslots):
        ring.acquire(k, lambda: False)
    stop = threading.Event()
    out = []
    th = threading.Thread(target=lambda: out.append(ring.acquire(0, stop.is_set)), daemon=True)
    th.start()
    stop.set()
    th.join(timeout=5)
    assert out == [P._DeviceRing.STOPPED] and not any(ring.free)
    ring.release_all(None)
    # the next epoch is not blocked
    content, stop2 = {}, threading.Event()
    n = 0
    for s_, _ in _all_batches(ring, [5], content, stop2):
        ring.release([s_], None)
        n += 1
    assert n == 5


@pytest.mark.parametrize("compact", [True, False])
def test_wire_layout_one_copy_of_a_prefix(tmp_path, compact):
    """Ring slot layout (``_ring_layout``): the host buffer is a prefix of the device slot's
    layout, so one copy of ``wire_bytes(mask)`` bytes moves ids + labels (+ the shipped value
    columns in compact mode); expanding the staged columns (the host twin of sparse.hip
    expand_vals) then fills the vals view bit for bit.  Fed by the real loader."""
    import numpy as np
    from hipfm.data import native_io as nio
    B, F = 64, 6
    rng = np.random.default_rng(3)
    ids = rng.integers(0, 1000, (B, F)).astype(np.int64)
    vals = np.ones((B, F), np.float32)
    vals[:, 2] = rng.standard_normal(B)
    vals[:, 5] = rng.random(B)
    lab = (rng.random(B) < 0.3).astype(np.float32)
    p = str(tmp_path / "w.tfrecords")
    nio.write_examples(p, lab, ids, vals)
    ring = P._DeviceRing(B, F, "cpu", torch.int32, 2, compact=compact)
    lay = ring.lay
    host = torch.zeros(lay["host"], dtype=torch.uint8)
    h_ids, h_vals, h_lab = P._flat_views(host, B, F, torch.int32, lay)
    ld = nio.NativeLoader([p], F, B, ids32=True)
    if compact:
        assert h_vals is None and lay["host"] < lay["total"]
        st = lay["stage"]
        r, mask = ld.next_into_compact(h_lab, h_ids, host[st[0]:st[1]].view(torch.float32))
        assert mask == (1 << 2) | (1 << 5)
        assert ring.wire_bytes(mask) == B * F * 4 + B * 4 + B * 2 * 4
    else:
        r, mask = ld.next_into(h_lab, h_ids, h_vals), 0
        assert lay["host"] == lay["total"] == ring.wire_bytes(0)
    ld.close()
    assert r == B
    nb = ring.wire_bytes(mask)
    ring.flat[0][:nb].copy_(host[:nb])                   # the one host-to-device copy
    d_ids, d_vals, d_lab = ring.views[0]
    if compact:
        cols = ring.stage[0][:B * 2].view(B, 2).numpy()
        d_vals.copy_(torch.from_numpy(nio.expand_values(cols, B, F, mask)))
    assert torch.equal(d_ids, torch.from_numpy(ids.astype(np.int32)))
    assert torch.equal(d_lab, torch.from_numpy(lab))
    assert np.array_equal(d_vals.numpy().view(np.uint32), vals.view(np.uint32))
