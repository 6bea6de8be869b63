"""Data parallelism over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Replaces the reference's two distribution paths:

* P2 Horovod synchronous DP (HVD:149,262,295,355-372): ``hvd.init`` -> ``init_distributed``
  (torchrun-style env, one process per GPU, ``127.0.0.1`` rendezvous), DistributedOptimizer's
  tensor-fusion all-reduce -> ONE flat dense-gradient bucket (latency-bound at these sizes, so a
  single bucket).  By default it travels in the step's last grouped collective with the sparse
  gradient rows (all-gathered, summed in rank order by the owner launch: parallel/sharded.py G2);
  HIPFM_SH_OVERLAP=1 instead all-reduces it on the main stream while the sparse backward runs on
  a graph branch.  ``BroadcastGlobalVariablesHook`` -> deterministic identical init on every rank
  (+ ``broadcast_dense`` for resumed state).
* P1/P4 Parameter Server + variable partitioning (PS:414-442, DOC p.32): the embedding table
  is ROW-SHARDED over ranks (owner = id % N, local row = id // N) with synchronous updates:
    forward : unique ids -> all-to-all ids to owners -> owners gather rows -> all-to-all rows back
    backward: reduce-by-key row grads -> all-to-all grads to owners -> owner dedup + row update
  xGMI is a full mesh of point-to-point links, so all-to-all uses all 7 peer links at once,
  where a ring all-gather of the Horovod IndexedSlices is per-link bound.
* ``replicated`` mode keeps a full table per rank (Horovod parity): the unique (id, row-grad)
  pairs of every rank are all-gathered in fixed-capacity blocks (not the reference's B*F+V
  rows) and reduced in rank order, identically on every rank (parallel/replicated.py).
Every multi-rank step runs on the native RCCL engine (csrc/kernels/comm.hip); the host-
synchronous torch.distributed exchange of earlier rounds survives only as a CPU test oracle
(tests/sharded_oracle.py).  HIPFM_SAME_DEVICE=1 maps every rank to device 0 and swaps the RCCL
engine for the same-device transport (parallel/loopback.py): the N-GPU job's exact processes and
step, rehearsed on one GPU.

Gradient averaging: the head kernel scales dlogit by 1/(B*N), so SUM all-reduces average.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import kernels as KN
from ..utils.knobs import flag, knob


def same_device() -> bool:
    """HIPFM_SAME_DEVICE=1: every rank of this node runs on device 0 (one-GPU rehearsal of the
    N-GPU job: gloo process group + the same-device collective engine, parallel/loopback.py)."""
    return flag("HIPFM_SAME_DEVICE")


def local_device_index() -> int:
    """The HIP device of this rank: LOCAL_RANK (one process per GPU), or 0 under same_device()."""
    return 0 if same_device() else int(os.environ.get("LOCAL_RANK", "0"))


def _device_cu_count(default: int = 256) -> int:
    """CUs of GPU 0 from the KFD topology (no HIP call: usable before any process touches the GPU)."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in sorted(os.listdir(root), key=lambda x: int(x) if x.isdigit() else 0):
            props = {}
            with open(os.path.join(root, node, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
            simd, per = int(props.get("simd_count", "0")), int(props.get("simd_per_cu", "0") or 0)
            if simd > 0 and per > 0:
                return simd // per
    except (OSError, ValueError):
        pass
    return default


def same_device_env(local_rank: int, local_world: int) -> dict:
    """Environment of one rank under HIPFM_SAME_DEVICE=1: a disjoint slice of the GPU's CUs
    (ROC_GLOBAL_CU_MASK, applied by the HIP runtime to every queue the process creates).  Ranks
    sharing every CU can starve each other's in-launch hand-offs -- a workgroup spinning on an
    earlier workgroup of its own launch that another process's spinning workgroups keep from being
    dispatched (the 8-rank rehearsal's sparse look-back timed out that way); with disjoint CUs each
    rank is a smaller GPU of its own, as one process per GPU is.  Empty unless the mode is on."""
    if not same_device() or local_world <= 1 or knob("HIPFM_SAME_DEVICE_CU_SPLIT") != "1":
        return {}
    n = _device_cu_count()
    per = n // local_world
    lo = local_rank * per
    mask = ((1 << per) - 1) << lo
    return {"ROC_GLOBAL_CU_MASK": hex(mask)}


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600):
    """Initialize the default process group from torchrun-style env (RANK, WORLD_SIZE, ...)."""
    if dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ.setdefault("RANK", "0")               # single-process runs (tests, --force_exchange)
    os.environ.setdefault("WORLD_SIZE", "1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if same_device():
        backend = "gloo"         # RCCL refuses two ranks on one device; gloo carries setup only
    kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", local_device_index())
    dist.init_process_group(**kw)


def agree_max(value: int, group=None) -> int:
    """The MAX of an int over the ranks of ``group`` (identical on every rank; gloo or RCCL)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return int(value)
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def exchange_capacity(id_batches, world: int, sharded: bool, slack: float = 1.05, pad: int = 256,
                      group=None) -> int:
    """Capacity of the fixed-size exchange, measured on every batch this rank will route and
    agreed across ranks (MAX): unique ids per owner (row-sharded all-to-all blocks) or unique
    ids per batch (replicated all-gather blocks).  Used by bench.py and the Estimator."""
    ids = list(id_batches)
    if sharded:
        from .sharded import estimate_capacity
        local = estimate_capacity(ids, world, slack=slack, pad=pad)
    else:
        from .replicated import estimate_unique_capacity
        local = estimate_unique_capacity(ids, slack=slack, pad=pad)
    return agree_max(local, group)


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


class Comm:
    """Collective engine used by NativeDeepFM for one process group: the native RCCL communicator
    (RcclEngine) whenever the group's backend is RCCL and the step exchanges (N > 1 or
    ``force_exchange``).  A NativeDeepFM refuses a multi-rank comm without it."""

    def __init__(self, sharded: bool = True, group=None, force_exchange: bool = False,
                 native: Optional[bool] = None, capacity: Optional[int] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        # force_exchange: run the multi-rank code path even on a 1-rank group (tests on 1 GPU)
        self.force_exchange = bool(force_exchange)
        self.sharded = bool(sharded) and (self.world_size > 1 or self.force_exchange)
        # native RCCL engine (csrc/kernels/comm.hip): fixed-capacity all-to-alls + the dense
        # gradient exchange, issued as grouped operations on the step's main stream -> no host
        # sync, graph-capturable step.  ONE communicator carries every collective of the step
        # in a fixed order (parallel/sharded.py module docstring: deadlock freedom)
        loop = same_device() and torch.cuda.is_available()
        if native is None:
            native = ((dist.get_backend(group) == "nccl" or loop)
                      and (self.world_size > 1 or self.force_exchange))
        self.engine = None
        if capacity is not None and self.world_size > 1:
            # every rank must use the SAME block size in the fixed-capacity exchanges: take the
            # max of the per-rank estimates (each rank measured its own batches)
            capacity = agree_max(capacity, group)
        self.capacity = capacity
        if native and loop:
            from .loopback import LoopbackEngine
            self.engine = LoopbackEngine(group)
        elif native:
            from .sharded import RcclEngine
            self.engine = RcclEngine(group)
        self.graph_safe = True

    @property
    def bytes_sent(self) -> int:
        return self.engine.bytes_sent if self.engine is not None else 0

    def allreduce_scalar(self, x: torch.Tensor) -> torch.Tensor:
        t = x.detach().clone().reshape(1).double() if x.dim() == 0 else x.clone()
        dist.all_reduce(t, group=self.group)
        return t.reshape(())

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        dist.broadcast(t, src=src, group=self.group)

    def barrier(self):
        dist.barrier(group=self.group)

    def close(self):
        """Destroy the native RCCL communicators (before the process group goes away).  Not for
        communicators captured into HIP graphs: ncclCommDestroy then blocks (ROCm 7)."""
        if self.engine is not None:
            self.engine.close()
