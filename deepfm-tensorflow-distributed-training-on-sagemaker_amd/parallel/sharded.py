"""Sync-free row-sharded embedding exchange (fixed per-peer capacity) for the MI355X executor.

The reference pulls embedding rows from parameter servers and pushes gradients back every step
(PS:414-442; variable partitioning, DOC p.32).  Here the table is row-sharded over the ranks
(owner = id % N, local row = id // N) and every exchange is an RCCL all-to-all of N equal blocks
of ``capacity`` entries, issued from the native engine (csrc/kernels/comm.hip) on the compute
stream.  No split size ever crosses to the host, so the whole multi-GPU step — sort, bucketing,
three all-to-alls, forward, backward, owner update and the dense all-reduce — is captured into
one HIP graph per resident batch, exactly like the single-GPU step (csrc/kernels/shard.hip has
the protocol).

Capacity: the unique ids a rank sends to one owner must fit ``capacity``.  ``estimate_capacity``
measures sample batches; a bucket that overflows sets an error word that the model checks
(``NativeDeepFM.check_errors``) and raises on — rows are never silently dropped.
"""
from __future__ import annotations

import math
from typing import Iterable, Optional

import torch

from ..ops import kernels as KN
from ..ops._lib import ShApplyArgs


def estimate_capacity(id_batches: Iterable[torch.Tensor], world: int, slack: float = 1.25,
                      pad: int = 256) -> int:
    """Per-peer capacity from sample batches: max over batches and owners of the number of
    unique ids one rank sends to one owner, times ``slack``, plus ``pad``, rounded to 64."""
    mx = 0
    for ids in id_batches:
        u = torch.unique(ids.reshape(-1).long())
        mx = max(mx, int(torch.bincount(u % world, minlength=world).max().item()))
    return int(math.ceil((mx * slack + pad) / 64.0) * 64)


def default_capacity(n_slots: int, world: int) -> int:
    """Capacity without calibration: 1.5x the mean slots per owner (bounded by all slots)."""
    return int(min(n_slots, math.ceil((1.5 * n_slots / world + 1024) / 64.0) * 64))


class RcclEngine:
    """Native RCCL communicator (comm.hip), bootstrapped over the launcher's process group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = KN.comm_unique_id() if self.rank == 0 else None
        obj = [uid]
        dist.broadcast_object_list(obj, src=0, group=group)
        self.handle = KN.comm_init(self.world, self.rank, obj[0])
        self.bytes_sent = 0

    def alltoall(self, send: torch.Tensor, recv: torch.Tensor, bytes_per_peer: int):
        self.bytes_sent += bytes_per_peer * self.world
        KN.comm_alltoall(self.handle, send, recv, bytes_per_peer)

    def allreduce_(self, t: torch.Tensor):
        self.bytes_sent += t.numel() * 4
        KN.comm_allreduce_(self.handle, t)

    def close(self):
        if self.handle:
            KN.comm_destroy(self.handle)
            self.handle = 0


class FixedCapacityExchange:
    """Buffers + step pieces of the row-sharded exchange for one NativeDeepFM (one rank)."""

    def __init__(self, m, engine, capacity: Optional[int] = None, tags: Optional[torch.Tensor] = None):
        self.m, self.eng = m, engine
        self.N, self.rank = engine.world, engine.rank
        dev = m.device
        K, n = m.K, m.M * m.F
        self.C = int(capacity) if capacity else default_capacity(n, self.N)
        self.C = (self.C + 63) // 64 * 64
        self.RW = K + 4                      # exchanged row: {v[K], w, 0, 0, 0} / {g_v, g_w, 0, 0, 0}
        T = self.N * self.C
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.send_ids = torch.full((T,), -1, **i32)
        self.recv_ids = torch.full((T,), -1, **i32)
        self.upos = torch.zeros(n, **i32)
        self.cnt_tmp = torch.zeros(KN.sh_count_blocks(n) * self.N, **i32)
        self.send_cnt = torch.zeros(self.N, **i32)
        self.err = torch.zeros(1, **i32)
        self.slot_row = torch.zeros(n, **i32)
        self.rows_out = torch.zeros(T, self.RW, **f32)
        self.rows_in = torch.zeros(T, self.RW, **f32)
        self.send_g = torch.zeros(T, self.RW, **f32)
        self.recv_g = torch.zeros(T, self.RW, **f32)
        # owner-side request tags: [local rows][N] of {step + 1, slot} (64-bit)
        self.tags = tags if tags is not None else torch.zeros(m.R * self.N, dtype=torch.int64, device=dev)

    # ------------------------------------------------------------------ forward
    def forward(self, B: int):
        """Sort + dedup the slot ids, fetch the unique rows from their owners.  Returns the
        per-slot row index and the (tv, tw) views of the received rows for fm_fwd."""
        m = self.m
        n = B * m.F
        m._sort_slots(B)
        KN.segments(m.sorted_keys, n, m.seg_flags, m.sid_incl, m.ukeys, m.seg_start, m.num_u, m.temp)
        KN.sh_bucket(m.ukeys, m.num_u, n, self.N, self.C, self.cnt_tmp, self.send_ids, self.upos,
                     self.send_cnt, self.err)
        self.eng.alltoall(self.send_ids, self.recv_ids, self.C * 4)
        KN.sh_serve(m.K, self.recv_ids, self.N * self.C, self.N, m.tv, m.tw, self.rows_out)
        self.eng.alltoall(self.rows_out, self.rows_in, self.C * self.RW * 4)
        KN.sh_slot_rows(m.perm, m.sid_incl, self.upos, n, self.slot_row)
        return self.slot_row, self.rows_in[:, : m.K], self.rows_in[:, m.K]

    # ------------------------------------------------------------------ backward
    def backward(self, B: int):
        """Per-unique gradient rows -> owners -> rank-ordered sum + row update on the owner."""
        m = self.m
        n = B * m.F
        A = m.sf_args(n)
        A.tv, A.tw = self.rows_in.data_ptr(), self.rows_in.data_ptr() + 4 * m.K
        A.ldv = A.ldw = self.RW
        A.sid, A.upos, A.gout = m.sid_incl.data_ptr(), self.upos.data_ptr(), self.send_g.data_ptr()
        KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
        self.eng.alltoall(self.send_g, self.recv_g, self.C * self.RW * 4)
        S = ShApplyArgs()
        S.recv_ids, S.total, S.N, S.C = self.recv_ids.data_ptr(), self.N * self.C, self.N, self.C
        S.mode = 0 if m.sparse_update == "lazy" else 1
        S.recv_g, S.tags = self.recv_g.data_ptr(), self.tags.data_ptr()
        S.tv, S.tw = m.tv.data_ptr(), m.tw.data_ptr()
        S.s0v, S.s1v, S.s0w, S.s1w = (t.data_ptr() if t.numel() else 0 for t in m.sv)
        S.ldv, S.ldw = KN._ld(m.tv, m.tw)
        if m.sparse_update == "tf1_dense":
            S.Gv, S.Gw = m.Gv.data_ptr(), m.Gw.data_ptr()
        S.h = m.h_sparse
        S.step = m.step.data_ptr()
        KN.sh_owner_apply(m.K, m.opt_id, S)
        if m.sparse_update == "tf1_dense":
            KN.dense_sweep(m.K, m.opt_id, m.R, m.tv, m.tw, m.Gv, m.Gw, m.sv, m.h_sparse, m.step)

    def error(self) -> int:
        return int(self.err.item())
