"""Data parallelism over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Replaces the reference's two distribution paths:

* P2 Horovod synchronous DP (HVD:149,262,295,355-372): ``hvd.init`` -> ``init_distributed``
  (torchrun-style env, one process per GPU, ``127.0.0.1`` rendezvous), DistributedOptimizer's
  tensor-fusion all-reduce -> ONE flat dense-gradient bucket (0.68 MB at the notebook config:
  latency-bound, so a single bucket) launched asynchronously right after the MLP backward and
  overlapped with the whole sparse backward (sort / reduce / exchange / row update) on RCCL's
  stream; ``BroadcastGlobalVariablesHook`` -> deterministic identical init on every rank
  (+ ``broadcast_dense`` for resumed state).
* P1/P4 Parameter Server + variable partitioning (PS:414-442, DOC p.32): the embedding table
  is ROW-SHARDED over ranks (owner = id % N, local row = id // N) with synchronous updates:
    forward : unique ids -> all-to-all ids to owners -> owners gather rows -> all-to-all rows back
    backward: reduce-by-key row grads -> all-to-all grads to owners -> owner dedup + row update
  xGMI is a full mesh of point-to-point links, so all-to-all uses all 7 peer links at once,
  where a ring all-gather of the Horovod IndexedSlices is per-link bound.
* ``replicated`` mode keeps a full table per rank (Horovod parity): the unique (id, row-grad)
  pairs of every rank are all-gathered in fixed-capacity blocks (not the reference's B*F+V
  rows) and reduced in rank order, identically on every rank (parallel/replicated.py; the
  torch.distributed ``replicated_exchange`` below is the host-synchronous fallback).

Gradient averaging: the head kernel scales dlogit by 1/(B*N), so SUM all-reduces average.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import kernels as KN
from .embedding import Router
from ..utils.knobs import knob


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
    kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
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
    """Collective engine used by NativeDeepFM for one process group."""

    def __init__(self, sharded: bool = True, group=None, force_exchange: bool = False,
                 native: Optional[bool] = None, capacity: Optional[int] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        # force_exchange: run the multi-rank code path even on a 1-rank group (tests on 1 GPU)
        self.force_exchange = bool(force_exchange)
        self.sharded = bool(sharded) and (self.world_size > 1 or self.force_exchange)
        self.router = Router(self.world_size, self.rank, group)
        self._bytes = 0
        # native RCCL engine (csrc/kernels/comm.hip): fixed-capacity all-to-alls + the dense
        # gradient exchange, issued as grouped operations on the step's main stream -> no host
        # sync, graph-capturable step.  ONE communicator carries every collective of the step
        # in a fixed order (parallel/sharded.py module docstring: deadlock freedom)
        if native is None:
            native = (dist.get_backend(group) == "nccl" and (self.world_size > 1 or self.force_exchange)
                      and knob("HIPFM_SHARD_EXCHANGE") == "fixed")
        self.engine = None
        if capacity is not None and self.world_size > 1:
            # every rank must use the SAME block size in the fixed-capacity exchanges: take the
            # max of the per-rank estimates (each rank measured its own batches)
            capacity = agree_max(capacity, group)
        self.capacity = capacity
        if native:
            from .sharded import RcclEngine
            self.engine = RcclEngine(group)
        # steps with host-synchronous routing (variable all-to-all splits) cannot be graphed
        self.graph_safe = (self.world_size == 1 and not self.force_exchange) or self.engine is not None

    @property
    def bytes_sent(self) -> int:
        eng = self.engine.bytes_sent if self.engine is not None else 0
        return self._bytes + self.router.bytes_sent + eng

    @bytes_sent.setter
    def bytes_sent(self, v: int):
        self._bytes = v - self.router.bytes_sent

    # ------------------------------------------------------------------ dense
    def allreduce_dense_async(self, g: torch.Tensor):
        self.bytes_sent += g.numel() * 4
        return dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def wait(self, work):
        work.wait()   # stream-ordered: the compute stream waits for RCCL's stream, no host block

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

    # ------------------------------------------------------------------ helpers
    def _a2a_counts(self, send_counts: torch.Tensor) -> List[int]:
        recv = torch.empty_like(send_counts)
        dist.all_to_all_single(recv, send_counts, group=self.group)
        return recv

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        self.bytes_sent += inp.numel() * inp.element_size()
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=self.group)

    # ------------------------------------------------------------------ row-sharded table
    def sharded_forward_gather(self, m, B: int):
        """Route this batch's unique ids to their owners and fetch the rows back.

        Returns (idx, tv_rows, tw_rows): ``idx`` maps every slot to a row of the compact
        [U, K] buffers the FM kernel then gathers from (K1 is unchanged)."""
        N, K = self.world_size, m.K
        n = B * m.F
        dev = m.device
        i32 = dict(dtype=torch.int32, device=dev)
        st = m.__dict__.setdefault("_shard_state", {})
        if st.get("M") != m.M:
            st["inv"] = torch.zeros(m.M * m.F, **i32)
            st["flags"] = torch.zeros(m.M * m.F, **i32)
            st["seg"] = torch.zeros(m.M * m.F, **i32)
            st["uniq"] = torch.zeros(m.M * m.F, **i32)
            st["M"] = m.M
        KN.sort_ids(m.idx, m.sorted_keys, None, m.perm, n, m.end_bit, m.temp)
        KN.unique_inverse(m.sorted_keys, m.perm, n, st["flags"], st["seg"], st["uniq"], st["inv"],
                          m.num_u, m.temp)
        U = int(m.num_u.item())                                   # host sync (routing sizes)
        plan = self.router.route(st["uniq"][:U])

        def serve(loc):
            rows = torch.empty(loc.numel(), K + 1, dtype=torch.float32, device=dev)
            rows[:, :K] = m.tv.index_select(0, loc)
            rows[:, K] = m.tw.index_select(0, loc)
            return rows
        rows_u = self.router.fetch_rows(plan, serve)
        st.update(U=U, plan=plan)
        st["tv_rows"] = rows_u[:, :K].contiguous()
        st["tw_rows"] = rows_u[:, K].contiguous()
        return st["inv"], st["tv_rows"], st["tw_rows"]

    def sharded_backward(self, m, B: int, idx, tv):
        st = m._shard_state
        n = B * m.F
        K = m.K
        gr = KN.grad_row_floats(K)
        m._segment_reduce(n, compact=True)
        KN.seg_apply(K, KN.SEG_WRITE_UG, 0, m.seg_args(n, compact=True, vsrc=tv, vsrc_compact=True), n)
        ids, recv = self.router.push_grads(st["plan"], m.UG[: st["U"]])
        return self._owner_reduce(m, ids, recv)

    def _owner_reduce(self, m, keys: torch.Tensor, rows: torch.Tensor):
        """Deduplicate received (global id, grad row) pairs on the owner (sort + reduce)."""
        R = keys.numel()
        dev = m.device
        if R == 0:
            m.num_u.zero_()
            return m.ukeys, m.UG, m.num_u, 0
        i32 = dict(dtype=torch.int32, device=dev)
        sk = torch.empty(R, **i32)
        perm = torch.empty(R, **i32)
        tmp = torch.empty(R, **i32)
        tb = max(KN.radix_temp_bytes(R), KN.rbk_temp_bytes(m.K, R))
        temp = torch.empty(tb + 256, dtype=torch.uint8, device=dev)
        KN.sort_ids(keys, sk, None, perm, R, m.end_bit, temp)
        rows_sorted = rows.index_select(0, perm.long())
        uk = torch.empty(R, **i32)
        ug = torch.empty_like(rows_sorted)
        num = torch.empty(1, **i32)
        KN.reduce_by_key(m.K, sk, rows_sorted, uk, ug, num, R, temp)
        m._owner_keep = (uk, ug, num, temp)   # keep alive until the update kernels ran
        return uk, ug, num, R

    # ------------------------------------------------------------------ replicated table
    def replicated_exchange(self, m, n: int):
        """All-gather every rank's unique (id, grad row) pairs and reduce them identically."""
        N = self.world_size
        dev = m.device
        cnt = m.num_u.to(torch.int64)
        cnts = [torch.empty_like(cnt) for _ in range(N)]
        dist.all_gather(cnts, cnt, group=self.group)
        c = [int(x.item()) for x in cnts]
        mx = max(c) if c else 0
        gr = m.UG.shape[1]
        keys = torch.full((N, mx), 0, dtype=torch.int32, device=dev)
        rows = torch.zeros(N, mx, gr, dtype=torch.float32, device=dev)
        my = c[self.rank]
        kk = torch.zeros(mx, dtype=torch.int32, device=dev)
        rr = torch.zeros(mx, gr, dtype=torch.float32, device=dev)
        kk[:my] = m.ukeys[:my]
        rr[:my] = m.UG[:my]
        self.bytes_sent += kk.numel() * 4 + rr.numel() * 4
        dist.all_gather_into_tensor(keys, kk, group=self.group)
        dist.all_gather_into_tensor(rows, rr, group=self.group)
        allk = torch.cat([keys[r, : c[r]] for r in range(N)])
        allr = torch.cat([rows[r, : c[r]] for r in range(N)])
        return self._owner_reduce(m, allk.contiguous(), allr.contiguous())
