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
    files = list(files)
    if shuffle:
        random.Random(seed * 1000003 + epoch).shuffle(files)   # identical on every rank
    if n <= 1:
        return ShardPlan(files, (1, 0))
    if policy == "file" and len(files) >= n:
        return ShardPlan(files[i::n], (1, 0))
    return ShardPlan(files, (n, i))


def pipe_root() -> str:
    return os.environ.get("HIPFM_PIPE_ROOT", PIPE_ROOT)


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


class InputPipeline:
    """Epoch-aware batch source (the reference's ``input_fn``, PS:76-133 / HVD:74-133)."""

    def __init__(self, files: Sequence[str], field_size: int, batch_size: int, num_epochs: int = 1,
                 fmt: str = "tfrecord", shard: Tuple[int, int] = (1, 0), policy: str = "file",
                 seed: int = 0, shuffle_files: bool = True, threads: int = 4, cache: bool = False,
                 device=None, drop_remainder: bool = True, pipe_channel: Optional[str] = None,
                 id_dtype=torch.int64):
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
        self._cached: Optional[List[Tuple[torch.Tensor, ...]]] = None
        self.max_batches: Optional[int] = None   # equal-steps enforcement across ranks

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
            t = tuple(x.to(self.device, non_blocking=True) for x in t)
        return t

    def iter_epoch(self, epoch: int, skip: int = 0) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
        """Batches of one epoch; ``skip`` drops the first batches (resume mid-epoch: they are
        read past, never decoded to tensors or trained on).  ``max_batches`` counts the skipped
        ones too (it is the epoch's length)."""
        if self.cache and self._cached is not None:
            end = self.max_batches if self.max_batches else len(self._cached)
            yield from self._cached[skip:end]
            return
        plan = self.epoch_plan(epoch)
        loader = NativeLoader(plan.files, self.F, self.B, self.fmt, self.drop_remainder,
                              self.threads, plan.record_shard)
        store = [] if (self.cache and skip == 0) else None
        k = 0
        try:
            for lab, ids, vals in loader:
                if self.max_batches is not None and k >= self.max_batches:
                    break
                if k < skip:
                    k += 1
                    continue
                t = self._to_tensors(lab, ids, vals)
                if store is not None:
                    store.append(t)
                k += 1
                yield t
        finally:
            loader.close()
        if store is not None:
            self._cached = store

    def __iter__(self):
        for e in range(self.num_epochs):
            yield from self.iter_epoch(e)
