"""Same-device collective engine: N rank PROCESSES on one GPU (HIPFM_SAME_DEVICE=1).

RCCL refuses two ranks on one device, so before this engine the production multi-rank step
(row-sharded exchange, dense gradient exchange, run-level routing, graphs of whole runs) could only
execute as threads in one process (tests/test_gpu_shard.py MeshEngine) or on a 1-rank RCCL group.
``LoopbackEngine`` has the RCCL engine's interface (``group(ops)``: all-to-all / all-gather / f32
sum all-reduce issued as one unit on the caller's stream) over IPC-mapped device staging buffers
and a shared-memory barrier run as a host node (csrc/kernels/loopback.hip has the protocol).  It
is capturable, so ``bench.py --gpus N`` and ``launch.py --nproc_per_node N`` under
HIPFM_SAME_DEVICE=1 run every rank's real step -- graphs included -- on the one GPU of a
development box.  The all-reduce sums in rank order (bitwise equal to the rank-ordered gather).

The process group is gloo in this mode (the RCCL backend would hit the same duplicate-device
check); it only carries setup traffic (handles, capacities, eval histograms).
"""
from __future__ import annotations

import ctypes as C
import os
import uuid

import torch
import torch.distributed as dist

from ..ops import _lib as LIB
from ..ops import kernels as KN
from ..utils.knobs import knob


def _stage_bytes(kind: int, nbytes: int, world: int) -> int:
    """Staging bytes of one op (loopback.hip op_stage_bytes)."""
    b = nbytes * world if kind == KN.COMM_A2A else nbytes
    return (b + 255) // 256 * 256


def group_stage_bytes(ops, world: int) -> int:
    return sum(_stage_bytes(k, nb, world) for k, _, _, nb in ops if nb)


class LoopbackError(RuntimeError):
    """The same-device transport's barrier timed out (this rank or a peer): the step is invalid."""


class LoopbackEngine:
    """Grouped collectives between the ranks of ``group`` that share ONE device."""

    def __init__(self, group=None, timeout_ms: int = None):
        self.pg = group                 # (process group: setup traffic only)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.bytes_sent = 0
        self.half = 0
        L = LIB.get_lib()
        self._L = L
        timeout_ms = int(timeout_ms or knob("HIPFM_LB_TIMEOUT_MS"))
        name = [f"/dev/shm/hipfm_lb_{uuid.uuid4().hex}" if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=0, group=group)
        path = name[0]
        h = C.c_void_p()
        if self.rank == 0:
            LIB.check(L.hfm_lb_create(C.byref(h), self.world, 0, path.encode(), 1, timeout_ms), "lb_create")
        dist.barrier(group=group)
        if self.rank != 0:
            LIB.check(L.hfm_lb_create(C.byref(h), self.world, self.rank, path.encode(), 0, timeout_ms),
                      "lb_create")
        dist.barrier(group=group)
        if self.rank == 0:
            os.unlink(path)             # every rank mapped it: nothing is left behind in /dev/shm
        self.handle = int(h.value)

    def reserve(self, nbytes: int):
        """Staging halves of at least ``nbytes`` (collective: every rank calls it at the same point
        of its host program with the same size, outside any graph capture).  Grows only."""
        nbytes = int(nbytes)
        if nbytes <= self.half:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"loopback transport: a group needs {nbytes} B of staging (have "
                               f"{self.half}) inside a graph capture; reserve it before capturing")
        L = self._L
        hb = int(L.hfm_lb_ipc_handle_bytes())
        buf = (C.c_char * hb)()
        LIB.check(L.hfm_lb_alloc_stage(self.handle, nbytes, buf), "lb_alloc_stage")
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(buf), group=self.pg)
        allh = (C.c_char * (hb * self.world)).from_buffer_copy(b"".join(handles))
        LIB.check(L.hfm_lb_open_peers(self.handle, allh), "lb_open_peers")
        self.half = int(L.hfm_lb_stage_half_kb(self.handle)) << 10

    def group(self, ops):
        """(kind, send, recv, bytes) collectives as one unit on the current stream."""
        need = group_stage_bytes(ops, self.world)
        if need > self.half:
            self.reserve(max(need + need // 4, 16 << 20))
        for kind, _, _, nb in ops:
            self.bytes_sent += nb if kind == KN.COMM_ALLREDUCE else nb * self.world
        from ..ops._lib import CommOp
        arr = (CommOp * max(1, len(ops)))()
        for i, (kind, send, recv, nbytes) in enumerate(ops):
            assert send.is_contiguous() and recv.is_contiguous()
            arr[i].kind, arr[i].send, arr[i].recv, arr[i].bytes = int(kind), send.data_ptr(), recv.data_ptr(), int(nbytes)
        LIB.check(self._L.hfm_lb_group(self.handle, arr, len(ops), LIB.stream_handle()), "lb_group")

    def error(self) -> int:
        return int(self._L.hfm_lb_error(self.handle)) if self.handle else 0

    def check(self):
        e = self.error()
        if e:
            raise LoopbackError("same-device transport: a collective barrier timed out "
                                f"({'this rank' if e == 1 else 'a peer rank'}); the steps since are invalid")

    def close(self):
        if self.handle:
            self._L.hfm_lb_destroy(self.handle)
            self.handle = 0
