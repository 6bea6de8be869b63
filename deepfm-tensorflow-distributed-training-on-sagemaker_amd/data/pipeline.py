"""Input pipeline: file discovery, shard policy, batching, epochs, cache (reference L2).

Reference behaviour:
  glob tr*/va*/te* recursively (PS:373-385) -> TFRecordDataset | PipeModeDataset
  -> shard(n, i) -> batch(B, drop_remainder=True) -> vectorized parse -> repeat -> prefetch.

Here the record source / framing / parse / batch / prefetch run in the native loader
(csrc/io, threads + bounded queues); this module decides WHICH files / records each rank reads:

* ``policy="file"`` (default, fixes quirk Q1): a seeded file order that is identical on every
  rank, files dealt round-robin to ranks, so rank shards are disjoint and complete and no rank
  reads bytes it drops.  Falls back to record-level sharding when there are fewer files than
  ranks.
* ``policy="record"``: the reference's ``dataset.shard(n, i)`` over the concatenated stream.

The shard (n, i) itself follows the reference's flag matrix (C06, HVD:95-120, RD:86-112):
  file mode : enable_s3_shard -> (worker_per_host, local_rank) else (world, rank)
  pipe mode : enable_data_multi_path x enable_s3_shard as in HVD:107-120.
``cache=True`` keeps the decoded epoch resident (device memory when given a device) — the
reference's commented-out ``dataset.cache()`` (PS:125) done right (before repeat, DOC p.43-44).
``cache_budget`` bounds it: an epoch whose decoded batches outgrow the budget is not cached, and
every epoch streams from the files instead (the reference's behaviour, which has no cache) -- a
dataset larger than free HBM (Criteo-1TB decodes to ~1.4 TB) trains instead of failing.
"""
from __future__ import annotations

import glob
import os
import random
import threading
from dataclasses import dataclass
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .native_io import FMT_LIBSVM, FMT_TFRECORD, NativeLoader, count_records
from ..utils.capture import CAPTURE_LOCK
from ..utils.knobs import knob

_H2D_STREAMS = int(knob("HIPFM_H2D_STREAMS"))

PIPE_ROOT = "/opt/ml/input/data"
_pipe_lock = threading.Lock()
_pipe_opened = {}        # channel -> number of epoch streams opened so far (this process)


def discover_files(data_dir: str, prefix: str, fmt: str = "tfrecord") -> List[str]:
    """Recursive ``<data_dir>/**/<prefix>*.tfrecords`` (PS:374-377); libsvm: any extension."""
    if not data_dir:
        return []
    pat = f"{prefix}*.tfrecords" if fmt == "tfrecord" else f"{prefix}*"
    files = glob.glob(os.path.join(data_dir, "**", pat), recursive=True)
    files = [f for f in files if os.path.isfile(f)]
    if fmt != "tfrecord":   # libsvm text: anything named like the split except TFRecords
        files = [f for f in files if not f.endswith(".tfrecords")]
    return sorted(files)


def shard_spec(world: int, rank: int, local_rank: int = 0, worker_per_host: int = 1,
               num_hosts: int = 1, enable_s3_shard: bool = False, pipe_mode: bool = False,
               enable_data_multi_path: bool = False) -> Tuple[int, int]:
    """(n, i) of the reference's dataset.shard for this rank (HVD:95-120)."""
    if not pipe_mode:
        return (worker_per_host, local_rank) if enable_s3_shard else (world, rank)
    if enable_data_multi_path:
        if not enable_s3_shard and num_hosts > 1:
            return num_hosts, rank // max(1, worker_per_host)
        return 1, 0
    return (worker_per_host, local_rank) if enable_s3_shard else (world, rank)


@dataclass
class ShardPlan:
    files: List[str]
    record_shard: Tuple[int, int]


def plan_shard(files: Sequence[str], n: int, i: int, policy: str = "file", seed: int = 0,
               epoch: int = 0, shuffle: bool = True) -> ShardPlan:
    """The files (and record shard) this rank reads.  The seeded shuffle is identical on every
    rank AND every epoch (``epoch`` does not enter it): the reference shuffles its file list once
    per job (PS:375), and an epoch streamed from the files then trains exactly like the epoch-0
    order the HBM cache replays (a cache-budget fallback or a resume mid-epoch reproduces it)."""
    files = list(files)
    if shuffle:
        random.Random(seed * 1000003).shuffle(files)   # identical on every rank and epoch
    if n <= 1:
        return ShardPlan(files, (1, 0))
    if policy == "file" and len(files) >= n:
        return ShardPlan(files[i::n], (1, 0))
    return ShardPlan(files, (n, i))


def pipe_root() -> str:
    return knob("HIPFM_PIPE_ROOT") or PIPE_ROOT


def pipe_channel_path(channel: str, epoch: int) -> str:
    """SageMaker Pipe-mode FIFO of a channel for an epoch (PipeModeDataset, PS:111)."""
    return os.path.join(pipe_root(), f"{channel}_{epoch}")


def next_pipe_stream(channel: str) -> str:
    """The next unread epoch stream of a Pipe-mode channel.  Pipe mode hands out every epoch of
    a channel exactly once, as ``<channel>_0``, ``<channel>_1``, ... (a FIFO can be read only
    once), so each reader that opens the channel -- a training epoch, every evaluation pass --
    takes the next index instead of re-opening a drained stream (reference HVD:396: re-entering
    PipeModeDataset on the same FIFO breaks)."""
    with _pipe_lock:
        k = _pipe_opened.get(channel, 0)
        _pipe_opened[channel] = k + 1
    return pipe_channel_path(channel, k)


class RingBatch(tuple):
    """(ids, vals, labels) views of one slot of a ``_DeviceRing``: the consumer calls
    ``ring.release`` once every kernel that reads the slot is enqueued."""

    def __new__(cls, views, ring, slot):
        t = super().__new__(cls, views)
        t.ring, t.slot = ring, slot
        return t


def _ring_layout(B: int, F: int, esz: int, compact: bool):
    """Byte ranges of one flat ring buffer: plain [ids | vals | labels]; compact [ids | labels |
    staged value columns | vals] (the host buffer stops after the staged columns: one copy of
    ids + labels + the nc shipped columns, the device expands them into vals)."""
    ids = (0, B * F * esz)
    if not compact:
        vals = (ids[1], ids[1] + B * F * 4)
        lab = (vals[1], vals[1] + B * 4)
        return dict(ids=ids, vals=vals, lab=lab, stage=None, total=lab[1], host=lab[1])
    lab = (ids[1], ids[1] + B * 4)
    stage = (lab[1], lab[1] + B * F * 4)
    vals = (stage[1], stage[1] + B * F * 4)
    return dict(ids=ids, vals=vals, lab=lab, stage=stage, total=vals[1], host=stage[1])


def _flat_views(flat, B: int, F: int, id_dtype, lay):
    """(ids [B, F], vals [B, F], labels [B]) typed views of one flat ring buffer (``_ring_layout``;
    the host buffer of the compact format has no vals range: None)."""
    def v(r, dt):
        return flat[r[0]:r[1]].view(dt) if r is not None and r[1] <= flat.numel() else None
    vals = v(lay["vals"], torch.float32)
    return (v(lay["ids"], id_dtype).view(B, F), vals.view(B, F) if vals is not None else None,
            v(lay["lab"], torch.float32))


def _release_unread(item):
    """A ring batch the pipeline drops unread (skipped on resume, past max_batches): its slot is
    free again at once (no kernel will read it)."""
    if isinstance(item, RingBatch):
        item.ring.release([item.slot], torch.cuda.current_stream())


class _DeviceRing:
    """Persistent device staging ring of the streamed (uncached) input path: ``nslots`` flat
    [ids | vals | labels] buffers, filled by ONE host-to-device copy each, straight from the
    pinned buffer the loader assembled the batch into.  The same slot views serve every epoch, so
    a run of consecutive slots is one captured multi-step graph, replayed (with the executor's
    host fast path: ``run_list`` returns the same list object for the same slots).  A slot is
    refilled only after the consumer released it (``release``: every kernel reading it is enqueued;
    the refill's copy waits on that point of the compute stream).

    ``compact`` (int32 ids, F <= 64, HIPFM_WIRE_COMPACT): the wire format drops the value columns
    of fields whose values are all 1.0 in the batch (Criteo's 26 categorical fields): one copy of
    [ids | labels | nc value columns] into the slot's staging range, then ``expand_vals`` on the
    same copy stream writes the [B, F] vals view the graphs read -- 212 instead of 316 bytes per
    Criteo row, bit-identical values."""

    def __init__(self, B: int, F: int, device, id_dtype, nslots: int, compact: Optional[bool] = None):
        import threading
        esz = torch.empty(0, dtype=id_dtype).element_size()
        if compact is None:
            compact = knob("HIPFM_WIRE_COMPACT") == "1" and id_dtype == torch.int32 and F <= 64
        self.B, self.F, self.id_dtype, self.nslots, self.compact = B, F, id_dtype, nslots, bool(compact)
        self.lay = _ring_layout(B, F, esz, self.compact)
        self.flat = [torch.empty(self.lay["total"], dtype=torch.uint8, device=device) for _ in range(nslots)]
        self.views = [_flat_views(x, B, F, id_dtype, self.lay) for x in self.flat]
        st = self.lay["stage"]
        self.stage = [x[st[0]:st[1]].view(torch.float32) for x in self.flat] if st else None
        self.ev = [None] * nslots
        self.free = [True] * nslots
        self.cv = threading.Condition()
        self._runs = {}
        self.G = max(1, nslots // 2)
        self.next = 0             # the next slot a fill thread writes (continues across epochs)

    def fits(self, B: int, F: int, id_dtype, nslots: int, compact: Optional[bool] = None) -> bool:
        same = (self.B, self.F, self.id_dtype, self.nslots) == (B, F, id_dtype, nslots)
        return same and (compact is None or bool(compact) == self.compact)

    def wire_bytes(self, mask: int) -> int:
        """Bytes one full batch copies host-to-device (compact: with popcount(mask) columns)."""
        if not self.compact:
            return self.lay["total"]
        return self.lay["lab"][1] + self.B * bin(mask).count("1") * 4

    STOPPED = object()      # acquire(): ``stop()`` turned true before the slot was taken

    def acquire(self, slot: int, stop) -> Optional[torch.cuda.Event]:
        """(fill thread) Wait until ``slot`` was released and take it; returns the compute-stream
        event its refill must wait for (or ``STOPPED``: the slot was not taken)."""
        with self.cv:
            while not self.free[slot]:
                if stop():
                    return _DeviceRing.STOPPED
                self.cv.wait(0.05)
            self.free[slot] = False
            return self.ev[slot]

    def giveback(self, slot: int, ev) -> None:
        """(fill thread) Return a slot taken by ``acquire`` but never filled (the feeder stopped):
        free again, with the same compute-stream event its next refill must wait for."""
        with self.cv:
            self.ev[slot] = ev
            self.free[slot] = True
            self.cv.notify_all()

    def start(self) -> int:
        """First slot of a new epoch's feeder.  Numbering continues across epochs: a consumer
        looking one batch ahead still holds the last run of the previous epoch (and a run may span
        the epoch boundary) while the next epoch's first batches are filled, so restarting at slot
        0 could wait for a slot that is only released after those batches arrive.  Filling the
        slots in cyclic order is safe (the consumer holds at most G + 1 of the 2G slots, the most
        recently filled ones); the start may jump ahead to the next run-aligned block (fewer
        distinct run graphs) only when that whole block is free, so the next G batches never wait.
        (tests/test_ring_cpu.py)"""
        with self.cv:
            cur = self.next % self.nslots
            t = (-(-self.next // self.G) * self.G) % self.nslots
            if t != cur and all(self.free[(t + i) % self.nslots] for i in range(self.G)):
                cur = t
            self.next = cur
            return cur

    def release(self, slots, stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        with self.cv:
            for s in slots:
                self.ev[s] = ev
                self.free[s] = True
            self.cv.notify_all()

    def release_all(self, stream):
        """The consumer stopped (early exit): slots it still held are free once the work enqueued
        so far is done."""
        self.release([s for s in range(self.nslots) if not self.free[s]], stream)

    def run_list(self, first: int, n: int):
        key = (first, n)
        r = self._runs.get(key)
        if r is None:
            r = self._runs[key] = [self.views[first + i] for i in range(n)]
        return r


class _DeviceFeeder:
    """Loader batches -> device batches: the C++ loader threads decode and a copy pool assembles
    each batch straight into a ring of pinned host buffers (ids narrowed to the device id type
    there) -- driven by a background fill thread, so the training loop never waits on the
    assembly -- and each buffer goes to the GPU with an async copy on a dedicated copy stream.
    The compute stream waits on the copy's event, never the host; a pinned buffer is refilled only
    after its previous copy finished (depth-deep ring: assembly of batches i+1.., copy of i and
    compute of i-1 overlap).  With a ``_DeviceRing`` (streamed epochs trained by a consumer that
    releases slots) the fill thread also issues the copy -- one per batch, into the next ring slot
    -- and the consumer receives ``RingBatch`` views: no per-batch allocation, copy or Python work
    on the training thread."""

    def __init__(self, loader, F: int, B: int, device, id_dtype, depth: int = 4, ring=None, id_limit: int = 0):
        self.loader, self.F, self.B, self.device, self.id_dtype = loader, F, B, device, id_dtype
        self.copy = torch.cuda.Stream(device)
        # ring mode: consecutive batches alternate over copy streams (each its own DMA queue; one
        # stream measured ~35 GB/s host-to-device, one 5.2 MB batch per ~150 us)
        self.copies = [self.copy] + [torch.cuda.Stream(device) for _ in range(max(0, _H2D_STREAMS - 1))]
        self.dev_ring = ring
        pin = dict(pin_memory=True)
        self.compact = ring is not None and ring.compact
        # GPU decode (a raw loader: ring mode only): pinned slots of record bytes + offsets, one
        # device staging pair per copy stream (a stream's next copy is ordered after its decode)
        self.raw = bool(getattr(loader, "raw", False))
        self.dcrc = bool(getattr(loader, "device_crc", False))    # data CRCs checked by the decoder
        self.id_limit = int(id_limit)
        if self.raw:
            if ring is None or ring.compact:
                raise ValueError("raw records need a plain-layout device ring")
            cap = B * int(knob("HIPFM_RAW_ROW_BYTES"))
            self.praw = [(torch.empty(cap, dtype=torch.uint8, **pin), torch.empty(B + 1, dtype=torch.int32, **pin))
                         for _ in range(depth)]
            self.draw = [(torch.empty(cap, dtype=torch.uint8, device=device),
                          torch.empty(B + 1, dtype=torch.int32, device=device)) for _ in self.copies]
            self.derr = torch.tensor([0, 0x7FFFFFFF], dtype=torch.int32, device=device)
            self.ring = [None] * depth
            loader.start_ring_raw(self.praw)
            self.asm = True
            self.done = [None] * depth
            self.h2d_s = self.h2d_bytes = 0
            self.fill_take_s = self.fill_issue_s = 0.0
            import queue
            self._free, self._full = queue.Queue(), queue.Queue()
            self._stop = False
            self._th = None
            self._batches = 0
            return
        if ring is not None:
            self.pflat = [torch.empty(ring.lay["host"], dtype=torch.uint8, **pin) for _ in range(depth)]
            self.ring = []
            self.pstage = []
            for x in self.pflat:
                ids, vals, lab = _flat_views(x, B, F, id_dtype, ring.lay)
                if self.compact:
                    # full host values only for a final partial batch (expanded on the host)
                    vals = torch.empty(B, F, dtype=torch.float32, **pin)
                    st = ring.lay["stage"]
                    self.pstage.append(x[st[0]:st[1]].view(torch.float32))
                self.ring.append((lab, ids, vals))             # (the loader's argument order)
        else:
            self.ring = [(torch.empty(B, dtype=torch.float32, **pin),
                          torch.empty(B, F, dtype=id_dtype, **pin),
                          torch.empty(B, F, dtype=torch.float32, **pin)) for _ in range(depth)]
        for lab, ids, vals in self.ring:     # (labels, ids, vals) in the loader's argument order
            assert lab.shape == (B,) and lab.dtype == torch.float32
            assert ids.shape == (B, F) and ids.dtype == id_dtype
            assert vals.shape == (B, F) and vals.dtype == torch.float32
        # ring mode with int32 ids: the loader assembles ahead into the pinned buffers on its own
        # C++ thread (NativeLoader.start_ring), so this feeder's per-batch Python work overlaps
        # the next batch's assembly instead of alternating with it
        self.asm = (ring is not None and id_dtype == torch.int32 and knob("HIPFM_ASM_RING") == "1"
                    and hasattr(loader, "start_ring"))
        if self.asm:
            loader.start_ring([(lab, ids, self.pstage[i] if self.compact else vals)
                               for i, (lab, ids, vals) in enumerate(self.ring)], compact=self.compact)
        self.done = [None] * depth
        self.h2d_s = 0.0         # host time spent issuing copies (the copies themselves are async)
        self.h2d_bytes = 0       # host-to-device bytes of the ring copies (the wire format's size)
        self.fill_take_s = 0.0   # fill thread: waiting for assembled batches (the loader's pace)
        self.fill_issue_s = 0.0  # fill thread: slot acquire + copy / expand / event issue
        import queue
        self._free, self._full = queue.Queue(), queue.Queue()
        for i in range(depth):
            self._free.put(i)
        self._stop = False
        self._th = None

    def _issue(self, R, k: int, slot: int, mask):
        """Copy pinned buffer ``slot`` (a full batch) into ring slot k % nslots on the next copy
        stream (compact values expanded there); returns (event after the whole batch, ring slot,
        event after the host-to-device copy alone: the pinned buffer is free again from there, the
        expand kernel may queue behind a run's kernels), or (None, ring slot, None) when the feeder
        stopped before the ring slot was free (the slot is handed back untouched)."""
        s = k % R.nslots
        wait = R.acquire(s, lambda: self._stop)
        if wait is _DeviceRing.STOPPED:      # stopped before the slot was taken
            return None, s, None
        if self._stop:
            # stopped right after taking slot s: hand it back untouched, or a later epoch's fill
            # thread waits on it forever
            R.giveback(s, wait)
            return None, s, None
        cs = self.copies[(k + 1) % len(self.copies)]
        with CAPTURE_LOCK, torch.cuda.stream(cs):     # (never inside a graph capture)
            if wait is not None:
                cs.wait_event(wait)
            ev_copy = None
            if mask is None:
                R.flat[s].copy_(self.pflat[slot], non_blocking=True)
            else:
                nb = R.wire_bytes(mask)
                R.flat[s][:nb].copy_(self.pflat[slot][:nb], non_blocking=True)
                ev_copy = torch.cuda.Event()
                ev_copy.record(cs)
                from ..ops import kernels as K
                K.expand_vals(R.stage[s], bin(mask).count("1"), mask, self.F, self.B, R.views[s][1])
            ev = torch.cuda.Event()
            ev.record(cs)
        self.h2d_bytes += R.wire_bytes(mask or 0)
        return ev, s, (ev_copy or ev)

    def _issue_raw(self, R, k: int, slot: int, nbytes: int):
        """Raw mode ``_issue``: the batch's record bytes + offsets to the device on the next copy
        stream, decoded there into ring slot k % nslots (csrc/kernels/decode.hip)."""
        s = k % R.nslots
        wait = R.acquire(s, lambda: self._stop)
        if wait is _DeviceRing.STOPPED:
            return None, s, None
        if self._stop:
            R.giveback(s, wait)
            return None, s, None
        i = (k + 1) % len(self.copies)
        cs = self.copies[i]
        draw, doffs = self.draw[i]
        praw, poffs = self.praw[slot]
        from ..ops import kernels as K
        with CAPTURE_LOCK, torch.cuda.stream(cs):     # (never inside a graph capture)
            if wait is not None:
                cs.wait_event(wait)
            draw[:nbytes].copy_(praw[:nbytes], non_blocking=True)
            doffs.copy_(poffs, non_blocking=True)
            ev_copy = torch.cuda.Event()
            ev_copy.record(cs)
            ids, vals, lab = R.views[s]
            K.decode_examples(draw, doffs, self.B, self.F, self.id_limit, ids, vals, lab, self.derr,
                              crc=self.dcrc)
            ev = torch.cuda.Event()
            ev.record(cs)
        self.h2d_bytes += nbytes + 4 * (self.B + 1)
        return ev, s, ev_copy

    def _decode_partial(self, slot: int, r: int, nbytes: int, k: int):
        """Raw mode, a final partial batch: decoded into fresh device tensors (the plain path's
        per-batch tensors, marked for the compute stream by the consumer)."""
        i = (k + 1) % len(self.copies)
        cs = self.copies[i]
        draw, doffs = self.draw[i]
        praw, poffs = self.praw[slot]
        from ..ops import kernels as K
        with CAPTURE_LOCK, torch.cuda.stream(cs):
            draw[:nbytes].copy_(praw[:nbytes], non_blocking=True)
            doffs[:r + 1].copy_(poffs[:r + 1], non_blocking=True)
            t = (torch.empty(r, self.F, dtype=self.id_dtype, device=self.device),
                 torch.empty(r, self.F, dtype=torch.float32, device=self.device),
                 torch.empty(r, dtype=torch.float32, device=self.device))
            K.decode_examples(draw, doffs, r, self.F, self.id_limit, t[0], t[1], t[2], self.derr, crc=self.dcrc)
            ev = torch.cuda.Event()
            ev.record(cs)
        self.h2d_bytes += nbytes + 4 * (r + 1)
        return t, ev

    def check_decode(self):
        """Raw mode: raise on records the GPU decoder flagged (one host sync: end of the epoch)."""
        if not self.raw:
            return
        e, first = (int(x) for x in self.derr.tolist())
        if e:
            what = []
            if e & 1:
                what.append("a record does not match the fixed Example schema (label, ids[F], values[F])")
            if e & 2:
                what.append("a feature id lies outside [0, feature_size) or int32")
            if e & 4:
                what.append("TFRecord data CRC mismatch (corrupt record)")
            raise IOError("GPU Example decode: " + "; ".join(what) +
                          f" (first bad record: index {first} of its batch; its row was zeroed)")

    def _fill_asm(self, R, k: int):
        """Ring mode over the loader's assembler thread: take assembled pinned slots in order,
        issue their copies, hand each pinned slot back once its copy finished."""
        import time
        from collections import deque
        inflight = deque()                      # (pinned slot, copy event), in take order
        depth = len(self.ring)
        while True:
            # the assembler fills slots in cyclic order: the oldest in-flight slot goes back first,
            # once two newer copies are queued behind it (long finished by then: the wait is a
            # formality).  No event queries: hipEventQuery from this thread while the training
            # thread captures a run graph invalidated the capture (hipErrorStreamCaptureInvalidated
            # in the one-process GPU suite); the synchronize the old path used is safe.
            while len(inflight) > 2 or (inflight and len(inflight) >= depth - 1):
                slot, ev = inflight.popleft()
                with CAPTURE_LOCK:
                    ev.synchronize()
                self.loader.ring_give(slot)
            if self._stop:
                return
            t0 = time.perf_counter()
            r, slot, mask = self.loader.ring_take()      # (ctypes: the GIL is released)
            t1 = time.perf_counter()
            self.fill_take_s += t1 - t0
            if self._stop:
                return
            if r == self.B:
                k += 1
                R.next = k
                if self.raw:
                    ev, s, ev_copy = self._issue_raw(R, k - 1, slot, mask)   # (mask: the byte count)
                else:
                    ev, s, ev_copy = self._issue(R, k - 1, slot, mask if self.compact else None)
                self.fill_issue_s += time.perf_counter() - t1
                if ev is None:
                    return
                inflight.append((slot, ev_copy))
                self._full.put((("ring", s), r, ev))
                continue
            if r > 0 and self.raw:               # final partial batch: fresh decoded tensors
                t, ev = self._decode_partial(slot, r, mask, k)
                inflight.append((slot, ev))
                self._full.put((("dev", t), r, ev))
                continue
            if r > 0 and self.compact:           # final partial batch: the plain path
                from .native_io import expand_values
                lab, ids, vals = self.ring[slot]
                vals.numpy()[:r] = expand_values(self.pstage[slot].numpy(), r, self.F, mask)
            self._full.put((slot, r, None))
            return

    def _fill(self):
        try:
            R = self.dev_ring
            k = R.start() if R is not None else 0
            if self.asm:
                return self._fill_asm(R, k)
            while True:
                slot = self._free.get()
                if slot is None or self._stop:
                    return
                ev = self.done[slot]
                if ev is not None:
                    with CAPTURE_LOCK:
                        ev.synchronize()             # this pinned buffer's last copy is over
                lab, ids, vals = self.ring[slot]
                mask = None
                if self.compact:
                    r, mask = self.loader.next_into_compact(lab, ids, self.pstage[slot])
                    if 0 < r < self.B:                # final partial batch: the plain path
                        from .native_io import expand_values
                        vals.numpy()[:r] = expand_values(self.pstage[slot].numpy(), r, self.F, mask)
                else:
                    r = self.loader.next_into(lab, ids, vals)   # (ctypes: the GIL is released)
                if R is not None and r == self.B:
                    k += 1
                    R.next = k
                    ev, s, ev_copy = self._issue(R, k - 1, slot, mask)
                    if ev is None:
                        return
                    self.done[slot] = ev_copy
                    self._free.put(slot)
                    self._full.put((("ring", s), r, ev))
                    continue
                self._full.put((slot, r, None))
                if r == 0:
                    return
        except BaseException as e:  # noqa: BLE001  (surfaced in the consumer)
            self._full.put((None, 0, e))

    def close(self):
        """Stop the fill thread (before the loader it reads from is closed); ring slots it filled
        that were never handed to the consumer are released (nothing reads them)."""
        if self._th is not None:
            self._stop = True
            self._free.put(None)
            self._th.join()
            self._th = None
            if self.dev_ring is not None:
                left = []
                while not self._full.empty():
                    slot, _, _ = self._full.get_nowait()
                    if isinstance(slot, tuple) and slot[0] == "ring":
                        left.append(slot[1])
                if left:
                    self.dev_ring.release(left, torch.cuda.current_stream(self.device))

    def __iter__(self):
        import threading
        import time
        compute = torch.cuda.current_stream(self.device)
        self._th = threading.Thread(target=self._fill, daemon=True)
        self._th.start()
        try:
            while True:
                slot, r, x = self._full.get()
                if isinstance(x, BaseException):
                    raise x
                if isinstance(slot, tuple) and slot[0] == "dev":   # decoded partial batch
                    compute.wait_event(x)
                    for t in slot[1]:
                        t.record_stream(compute)
                    yield slot[1]
                    continue
                if isinstance(slot, tuple):          # a ring slot, copied by the fill thread
                    compute.wait_event(x)
                    yield RingBatch(self.dev_ring.views[slot[1]], self.dev_ring, slot[1])
                    continue
                if r == 0:
                    self.check_decode()
                    return
                lab, ids, vals = self.ring[slot]
                t0 = time.perf_counter()
                with torch.cuda.stream(self.copy):
                    # allocated on the copy stream (free there: no wait on the compute stream's
                    # queued steps -- a wait_stream(compute) here serialized every copy behind the
                    # previous run's graph, ~40 M samples/s), then marked as used by the compute
                    # stream so the allocator keeps them until its reads are done
                    d_ids = torch.empty(r, self.F, dtype=self.id_dtype, device=self.device)
                    d_vals = torch.empty(r, self.F, dtype=torch.float32, device=self.device)
                    d_lab = torch.empty(r, dtype=torch.float32, device=self.device)
                    d_ids.copy_(ids[:r], non_blocking=True)
                    d_vals.copy_(vals[:r], non_blocking=True)
                    d_lab.copy_(lab[:r], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.copy)
                for t in (d_ids, d_vals, d_lab):
                    t.record_stream(compute)
                self.done[slot] = ev
                self._free.put(slot)
                compute.wait_event(ev)
                self.h2d_s += time.perf_counter() - t0
                yield d_ids, d_vals, d_lab
        finally:
            self.close()


def derive_field_ranges(fmin: torch.Tensor, fmax: torch.Tensor, V: int):
    """Per-field id ranges from the per-field min / max ids seen in the data: [lo_f, hi_f) with
    lo_0 = 0, hi_f = lo_{f+1} = min_{f+1}, hi_last = V (gaps between fields are covered, so any id
    a field can take between its neighbours' ranges stays valid).  None unless the observed
    intervals are disjoint and increasing in field order (then the per-field sort cannot apply)."""
    mn, mx = [int(x) for x in fmin.tolist()], [int(x) for x in fmax.tolist()]
    F = len(mn)
    for f in range(F - 1):
        if not mx[f] < mn[f + 1]:
            return None
    if mn[0] < 0 or mx[-1] >= V:
        return None
    lo = [0] + mn[1:]
    hi = mn[1:] + [V]
    return list(zip(lo, hi))


def agreed_field_ranges(pipeline, V: int, world: int = 1, group=None):
    """Per-field id ranges every rank agrees on: the per-field min / max ids of each rank's cached
    shard are combined with MIN / MAX all-reduces (``group``: a host-side gloo group) before
    ``derive_field_ranges`` -- so no rank's ids fall outside the ranges it sorts with.  None on
    every rank when any rank has no cached epoch or the combined ranges are not disjoint."""
    mm = pipeline.field_minmax() if hasattr(pipeline, "field_minmax") else None
    if world > 1:
        import torch.distributed as dist
        have = torch.tensor([0 if mm is None else 1], dtype=torch.int64)
        dist.all_reduce(have, op=dist.ReduceOp.MIN, group=group)
        if int(have.item()) == 0:
            return None
        mn, mx = mm[0].clone(), mm[1].clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
        mm = (mn, mx)
    if mm is None:
        return None
    return derive_field_ranges(mm[0], mm[1], V)


class InputPipeline:
    """Epoch-aware batch source (the reference's ``input_fn``, PS:76-133 / HVD:74-133)."""

    def __init__(self, files: Sequence[str], field_size: int, batch_size: int, num_epochs: int = 1,
                 fmt: str = "tfrecord", shard: Tuple[int, int] = (1, 0), policy: str = "file",
                 seed: int = 0, shuffle_files: bool = True, threads: int = 4, cache: bool = False,
                 device=None, drop_remainder: bool = True, pipe_channel: Optional[str] = None,
                 id_dtype=torch.int64, id_limit: int = 0, cache_budget: Optional[int] = None):
        self.files = list(files)
        self.F, self.B = int(field_size), int(batch_size)
        self.num_epochs = max(1, int(num_epochs))
        self.fmt = FMT_TFRECORD if fmt == "tfrecord" else FMT_LIBSVM
        self.fmt_name = fmt
        self.shard = shard
        self.policy = policy
        self.seed = seed
        self.shuffle_files = shuffle_files
        self.threads = threads
        self.cache = cache
        self.device = device
        self.drop_remainder = drop_remainder
        self.pipe_channel = pipe_channel
        self.id_dtype = id_dtype
        self.id_limit = int(id_limit)            # > 0: ids must lie in [0, V) (checked by the loader)
        self.cache_budget = cache_budget          # bytes the cached epoch may take (None: no bound)
        self.cache_overflow = False               # the epoch outgrew the budget: stream every epoch
        self._cached: Optional[List[Tuple[torch.Tensor, ...]]] = None
        self.max_batches: Optional[int] = None   # equal-steps enforcement across ranks
        self.from_cache = False                  # the epoch being iterated replays the cache
        self.h2d_s = 0.0                          # host time issuing H2D copies (last epoch)
        self.h2d_bytes = 0                        # ring copies' host-to-device bytes (last epoch)
        self.fill_take_s = self.fill_issue_s = 0.0   # fill thread's wait / issue time (last epoch)
        self._fmin = self._fmax = None           # per-field id min / max over the first epoch
        self._stats_done = False
        # > 1: the consumer trains streamed batches in runs of this many steps and releases ring
        # slots (RingBatch.ring.release) -- set by Estimator.train around its loop
        self.ring_steps = 0
        self._ring = None

    @property
    def countable(self) -> bool:
        """Files can be counted ahead of training; a Pipe-mode stream can only be read once."""
        return self.pipe_channel is None

    def epoch_plan(self, epoch: int) -> ShardPlan:
        if self.pipe_channel is not None:
            return ShardPlan([next_pipe_stream(self.pipe_channel)], self.shard)
        return plan_shard(self.files, self.shard[0], self.shard[1], self.policy, self.seed, epoch,
                          self.shuffle_files)

    def local_records(self, epoch: int = 0) -> int:
        if not self.countable:
            raise RuntimeError("a Pipe-mode channel is a stream: its records cannot be counted "
                               "before training (equal steps are agreed per step instead)")
        plan = self.epoch_plan(epoch)
        total = sum(count_records(f, self.fmt) for f in plan.files)
        n, i = plan.record_shard
        if n > 1:
            total = total // n + (1 if i < total % n else 0)
        return total

    def _to_tensors(self, lab, ids, vals):
        t = (torch.from_numpy(np.array(ids)).to(self.id_dtype), torch.from_numpy(np.array(vals)),
             torch.from_numpy(np.array(lab)))
        if self.device is not None:
            t = tuple(x.to(self.device) for x in t)
        return t

    def iter_epoch(self, epoch: int, skip: int = 0) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """Batches of one epoch; ``skip`` drops the first batches (resume mid-epoch: they are
        read past, never decoded to tensors or trained on).  ``max_batches`` counts the skipped
        ones too (it is the epoch's length)."""
        if self.cache and self._cached is not None:
            end = self.max_batches if self.max_batches else len(self._cached)
            self.from_cache = True
            yield from self._cached[skip:end]
            return
        self.from_cache = False
        plan = self.epoch_plan(epoch)
        loader = NativeLoader(plan.files, self.F, self.B, self.fmt, self.drop_remainder,
                              self.threads, plan.record_shard, id_limit=self.id_limit,
                              ids32=self.id_dtype == torch.int32)
        store = [] if (self.cache and skip == 0 and not self.cache_overflow) else None
        stored = 0
        # per-field id min / max of the first complete epoch (cached or streamed)
        stats = skip == 0 and not self._stats_done
        if stats:
            self._fmin = self._fmax = None
        on_gpu = self.device is not None and torch.device(self.device).type == "cuda"
        ring = None
        if on_gpu and self.ring_steps > 1 and store is None:
            # streamed epoch whose consumer releases ring slots (Estimator.train): batches land in
            # the persistent device ring, two runs deep
            n = 2 * int(self.ring_steps)
            # GPU decode (HIPFM_GPU_DECODE): the loader ships raw Example bytes, the ring slots take
            # the decoded plain layout
            gd = knob("HIPFM_GPU_DECODE")
            raw = (gd in ("1", "2") and self.fmt == FMT_TFRECORD and self.id_dtype == torch.int32)
            compact = False if raw else None
            if self._ring is None or not self._ring.fits(self.B, self.F, self.id_dtype, n, compact):
                self._ring = _DeviceRing(self.B, self.F, torch.device(self.device), self.id_dtype, n,
                                         compact=compact)
            ring = self._ring
            if raw:
                loader.close()
                loader = NativeLoader(plan.files, self.F, self.B, self.fmt, self.drop_remainder,
                                      self.threads, plan.record_shard, raw=True, device_crc=gd == "1")
        src = (_DeviceFeeder(loader, self.F, self.B, torch.device(self.device), self.id_dtype, ring=ring,
                             depth=8 if ring is not None else 4, id_limit=self.id_limit)
               if on_gpu else None)
        k = 0
        try:
            for item in (src if src is not None else loader):
                if self.max_batches is not None and k >= self.max_batches:
                    _release_unread(item)
                    break
                if k < skip:                 # (resume: read past, never trained)
                    _release_unread(item)
                    k += 1
                    continue
                t = item if src is not None else self._to_tensors(*item)
                if store is not None and on_gpu:
                    # the HBM cache keeps ids FIELD-MAJOR ([F, B] storage behind the [B, F] view,
                    # one transpose per batch when the epoch is cached): the run-level sort's
                    # per-field workgroups and the tower gather then read each field contiguously
                    # (profiles/r4c_*: 0.1121 vs 0.1141 ms/step at the 1TB shape) -- the layout
                    # bench.py's resident batches use
                    t = (t[0].t().contiguous().t(),) + tuple(t[1:])
                if store is not None:
                    stored += sum(x.numel() * x.element_size() for x in t)
                    if self.cache_budget is not None and stored > self.cache_budget:
                        # over budget: give the partial cache back, stream every epoch from now on
                        store = None
                        self.cache_overflow = True
                if store is not None:
                    store.append(t)
                if stats:
                    ids = t[0]
                    mn, mx = ids.amin(0), ids.amax(0)
                    self._fmin = mn if self._fmin is None else torch.minimum(self._fmin, mn)
                    self._fmax = mx if self._fmax is None else torch.maximum(self._fmax, mx)
                k += 1
                yield t
        finally:
            if src is not None:
                src.close()                  # (its fill thread reads the loader)
                self.h2d_s = src.h2d_s
                self.h2d_bytes = src.h2d_bytes
                self.fill_take_s, self.fill_issue_s = src.fill_take_s, src.fill_issue_s
            loader.close()
        if stats:                    # (reached only when the epoch was read to its end)
            self._stats_done = True
        if store is not None:
            self._cached = store

    def drop_cache(self):
        """Give the cached epoch back and stream every later epoch (a rank-agreed decision:
        Estimator.agree_cache)."""
        self._cached = None
        self.cache_overflow = True
        self.from_cache = False

    def field_minmax(self):
        """(per-field min ids, per-field max ids) over the first complete epoch as CPU int64
        tensors, or None before one was read."""
        if self._fmin is None or not self._stats_done:
            return None
        return self._fmin.cpu().long(), self._fmax.cpu().long()

    def field_ranges(self, V: int):
        """Per-field id ranges derived from the cached epoch (None before it is cached, or when
        the fields' ids are not disjoint and increasing).  This rank's shard only; the Estimator
        combines every rank's min / max first."""
        mm = self.field_minmax()
        return None if mm is None else derive_field_ranges(mm[0], mm[1], V)

    @property
    def cached_batches(self) -> int:
        return 0 if self._cached is None else len(self._cached)

    def __iter__(self):
        for e in range(self.num_epochs):
            yield from self.iter_epoch(e)
