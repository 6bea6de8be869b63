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
import os
from typing import Iterable, Optional

import torch

from ..ops import kernels as KN
from ..ops._lib import ShApplyArgs, ShTable
from ..utils.knobs import flag

# routing in two launches (sh_route) instead of segments + bucket (7 launches); same outputs
_ROUTE2 = flag("HIPFM_SH_ROUTE2")
# lazy rows: the NEXT batch's rows are served on the side stream during this step (after its
# routing); this step's owner update patches the rows it changes, so the serve launch leaves
# the critical path
_SERVE_AHEAD = flag("HIPFM_SH_SERVE_AHEAD")


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

    def allgather(self, send: torch.Tensor, recv: torch.Tensor, bytes_per_rank: int):
        self.bytes_sent += bytes_per_rank * self.world
        KN.comm_allgather(self.handle, send, recv, bytes_per_rank)

    def alltoall_allgather(self, send, recv, bytes_per_peer: int, gsend, grecv, gbytes_per_rank: int):
        self.bytes_sent += (bytes_per_peer + gbytes_per_rank) * self.world
        KN.comm_alltoall_allgather(self.handle, send, recv, bytes_per_peer, gsend, grecv, gbytes_per_rank)

    def allreduce_(self, t: torch.Tensor):
        self.bytes_sent += t.numel() * 4
        KN.comm_allreduce_(self.handle, t)

    def close(self):
        if self.handle:
            KN.comm_destroy(self.handle)
            self.handle = 0


class _RouteSet:
    """Routing state of one batch: sorted slots, unique ids, owner buckets, received requests.
    Depends only on the batch ids (not on the table), so the next batch's set can be built while
    the current batch trains."""

    def __init__(self, m, n: int, N: int, C: int, temp_bytes: int):
        dev = m.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.sorted_keys = torch.zeros(n, **i32)
        self.perm = torch.zeros(n, **i32)
        self.seg_flags = torch.zeros(n, **i32)
        self.sid_incl = torch.zeros(n, **i32)
        self.ukeys = torch.zeros(n, **i32)
        self.seg_start = torch.zeros(n + 1, **i32)
        self.num_u = torch.zeros(1, **i32)
        self.temp = torch.zeros(temp_bytes, dtype=torch.uint8, device=dev)
        self.upos = torch.zeros(n, **i32)
        self.cnt_tmp = torch.zeros(KN.sh_count_blocks(n) * N, **i32)
        self.tcnt = torch.zeros(KN.sh_route_tiles(n) * (N + 1), **i32)
        self.send_ids = torch.full((N * C,), -1, **i32)
        self.recv_ids = torch.full((N * C,), -1, **i32)
        self.send_cnt = torch.zeros(N, **i32)
        self.gathered = None     # [N, N*C] all-gathered requests (side-stream routing)
        self.slot_row = torch.zeros(n, **i32)
        self.recv = (self.recv_ids.data_ptr(), 0)   # (requests address, row stride) for the owner
        self.key = None          # host: (ids data_ptr, B) routed into this set
        # owner side: served rows and the request table (csrc/kernels/shard.hip) of this set's
        # batch -- per set, because the next batch's rows are served (and its requests stamped)
        # while the current batch's update still reads its own table.  The table has a power of
        # two >= 2x the N*C request slots; keys and per-requester positions carry step stamps --
        # sized by the exchange, not by the table (a direct [R_local][N] tag array is 7 GB per
        # rank at the 1TB shape)
        T = N * C
        self.rows_out = torch.zeros(T, m.K + 4, dtype=torch.float32, device=dev)
        slots = 1
        while slots < 2 * T:
            slots *= 2
        self.req_key = torch.zeros(slots, dtype=torch.int64, device=dev)
        self.req_pos = torch.zeros(slots * N, dtype=torch.int64, device=dev)
        self.table = ShTable(self.req_key.data_ptr(), self.req_pos.data_ptr(), slots - 1, 0)
        self.ahead = False       # host: rows_out holds this batch's rows, served ahead


class FixedCapacityExchange:
    """Buffers + step pieces of the row-sharded exchange for one NativeDeepFM (one rank).

    Two routing sets alternate: with ``next`` known (resident / prefetched batches), the routing
    of batch i+1 (sort, dedup, owner buckets, id all-to-all, slot->row map) runs on a side stream
    during step i — the sparse-input-dist pipelining of production DLRM trainers — so the
    critical path of a step keeps only the row fetch, the compute and the gradient exchange."""

    def __init__(self, m, engine, capacity: Optional[int] = None, engine_route=None):
        self.m, self.eng = m, engine
        self.eng_route = engine_route     # created on the first prefetching step (plan())
        self.N, self.rank = engine.world, engine.rank
        dev = m.device
        K, n = m.K, m.M * m.F
        self.C = int(capacity) if capacity else default_capacity(n, self.N)
        self.C = (self.C + 63) // 64 * 64
        self.RW = K + 4                      # exchanged row: {v[K], w, 0, 0, 0} / {g_v, g_w, 0, 0, 0}
        T = self.N * self.C
        f32 = dict(dtype=torch.float32, device=dev)
        self.sets = [_RouteSet(m, n, self.N, self.C, m.temp.numel()) for _ in range(2)]
        for rs in self.sets:
            rs.gathered = torch.zeros(self.N * self.N * self.C, dtype=torch.int32, device=dev)
        self.cur = 0
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.rows_in = torch.zeros(T, self.RW, **f32)
        self.send_g = torch.zeros(T, self.RW, **f32)
        self.recv_g = torch.zeros(T, self.RW, **f32)
        self._side = None
        self._joined = False
        self._next_ids, self._next_fm = None, False
        self._fork_at = None
        self._fork_plan = None
        self.dense_recv = None               # [N][P] all-gathered dense gradients (fused exchange)

    # ------------------------------------------------------------------ host-side plan
    def plan(self, ids: torch.Tensor, B: int, nxt: Optional[torch.Tensor], resident: bool = True):
        """Routing decisions for one step (part of the graph key): (set index, route the current
        batch inline?, next ids or None, rows already served ahead?, serve the next batch's rows
        ahead?).  Only resident batches (fixed device buffers) can have been prefetched: staged
        buffers change content under the same address."""
        c = self.cur
        key = (ids.data_ptr(), B)
        inline = (not resident) or self.sets[c].key != key
        ahead = (not inline) and self.sets[c].ahead
        if nxt is not None and self.eng_route is None:
            get = getattr(self.m.comm, "route_engine", None)
            self.eng_route = get() if get is not None else self.eng
        serve_next = nxt is not None and _SERVE_AHEAD and self.m.sparse_update == "lazy"
        return (c, inline, None if nxt is None else (nxt.data_ptr(), nxt.numel() // self.m.F), ahead,
                serve_next)

    def commit(self, plan, ids: torch.Tensor, B: int, resident: bool = True):
        """Consecutive steps always use alternate routing sets (prefetched or not): a step's
        routing kernels never overwrite buffers the previous step's backward still reads, even
        when graph replays run back to back.  A routing set is reused ONLY for the batch the
        caller declared as next (``next_ids``): a set is never matched again by address alone,
        since a freshly allocated batch can get the address of an earlier one back from the
        caching allocator."""
        c, _, nk, _, serve_next = plan
        self.sets[c].key = None
        self.sets[c].ahead = False
        self.sets[1 - c].key = nk
        self.sets[1 - c].ahead = nk is not None and serve_next
        self.cur = 1 - c

    def drop_served(self):
        """Parameters changed outside a step (load / broadcast): rows served ahead are stale, so
        the next step serves its rows itself (its prefetched routing stays valid)."""
        for rs in self.sets:
            rs.ahead = False

    # ------------------------------------------------------------------ pieces
    def route(self, rs: _RouteSet, ids: torch.Tensor, B: int, eng, gather: bool = False, fm: bool = False):
        """Sort + dedup the slot ids, bucket the unique ids by owner, send the requests.
        ``gather``: requests travel by all-gather (every rank's [N, C] block; this rank keeps
        column ``rank``) instead of all-to-all — RCCL's all-to-all cannot be captured on a forked
        side stream (segfault at graph instantiation on ROCm 7), its collectives can."""
        m = self.m
        n = B * m.F
        if m.uses_field_sort(B):
            m._fsort(ids, B, rs.sorted_keys, rs.perm, field_major=fm)
        else:
            KN.sort_ids(ids, rs.sorted_keys, None, rs.perm, n, m.end_bit, rs.temp)
        if _ROUTE2:
            KN.sh_route(rs.sorted_keys, n, self.N, self.C, rs.tcnt, rs.sid_incl, rs.send_ids, rs.upos,
                        rs.send_cnt, rs.num_u, self.err)
        else:
            KN.segments(rs.sorted_keys, n, rs.seg_flags, rs.sid_incl, rs.ukeys, rs.seg_start, rs.num_u,
                        rs.temp)
            KN.sh_bucket(rs.ukeys, rs.num_u, n, self.N, self.C, rs.cnt_tmp, rs.send_ids, rs.upos,
                         rs.send_cnt, self.err)
        if gather:
            if rs.gathered is None:
                rs.gathered = torch.zeros(self.N * self.N * self.C, dtype=torch.int32, device=m.device)
            eng.allgather(rs.send_ids, rs.gathered, self.N * self.C * 4)
            # the owner kernels read this rank's column of the gathered requests in place
            rs.recv = (rs.gathered.data_ptr() + 4 * self.rank * self.C, self.N * self.C)
        else:
            eng.alltoall(rs.send_ids, rs.recv_ids, self.C * 4)
            rs.recv = (rs.recv_ids.data_ptr(), 0)
        KN.sh_slot_rows(rs.perm, rs.sid_incl, rs.upos, n, rs.slot_row)

    def begin(self, plan, B: int, fork: str = "start"):
        """Start of a step: route the current batch if it was not prefetched, then fork the
        routing of the next batch onto a side stream -- here (``fork="start"``), right after the
        row fetch is enqueued (``"fetch"``), or when the caller calls ``fork_next`` (graph
        branches are dispatched in capture order: a branch enqueued first delays the main
        stream's first kernels)."""
        m = self.m
        c, inline, nk = plan[:3]
        if inline:
            self.route(self.sets[c], m.idx, B, self.eng, fm=m._idx_fm)
        self._joined = False
        self._fork_at = fork if nk is not None else None
        self._fork_plan = plan
        if self._fork_at == "start":
            self.fork_next()

    def fork_next(self):
        """Enqueue the next batch's routing on the side stream (once per step)."""
        if self._fork_at is None:
            return
        self._fork_at = None
        m = self.m
        c, _, nk, _, serve_next = self._fork_plan
        main = torch.cuda.current_stream(m.device)
        if self._side is None:
            self._side = torch.cuda.Stream(m.device)
        self._side.wait_stream(main)
        nxt_ids = self._next_ids
        rs = self.sets[1 - c]
        with torch.cuda.stream(self._side):
            self.route(rs, nxt_ids, nk[1], self.eng_route, gather=True, fm=self._next_fm)
            if serve_next:
                # the next batch's rows as of now (stamped step + 2); this step's owner update
                # patches the rows it changes (it joins this branch first)
                KN.sh_serve(m.K, rs.recv[0], self.N * self.C, self.N, m.tv, m.tw, rs.rows_out, C=self.C,
                            step=m.step, table=rs.table, rstride=rs.recv[1], ahead=True)

    def _join_side(self, plan):
        if plan[2] is not None and not self._joined:
            torch.cuda.current_stream(self.m.device).wait_stream(self._side)
            self._joined = True

    def end(self, plan):
        self.fork_next()                     # (not forked yet: e.g. no tower in this step)
        self._join_side(plan)

    def fetch(self, plan, train: bool = True):
        """Owners serve the requested rows (after the previous step's updates), rows come back.
        Training steps stamp the owner-side request tags here (read by the update at the end of
        the step); eval / predict fetches leave them alone."""
        m = self.m
        rs = self.sets[plan[0]]
        if train:
            if not plan[3]:                  # (else served during the previous step)
                KN.sh_serve(m.K, rs.recv[0], self.N * self.C, self.N, m.tv, m.tw, rs.rows_out,
                            C=self.C, step=m.step, table=rs.table, rstride=rs.recv[1])
        else:
            KN.sh_serve(m.K, rs.recv[0], self.N * self.C, self.N, m.tv, m.tw, rs.rows_out, C=self.C,
                        rstride=rs.recv[1])
        self.eng.alltoall(rs.rows_out, self.rows_in, self.C * self.RW * 4)
        if train and self._fork_at == "fetch":
            self.fork_next()
        return rs.slot_row, self.rows_in[:, : m.K], self.rows_in[:, m.K]

    def backward(self, plan, B: int, dense=None, join=None, wgfin=None):
        """Per-unique gradient rows -> owners -> rank-ordered sum + row update on the owner.
        ``dense`` (ShDenseArgs, lazy rows): the dense optimizer runs in the owner update's launch,
        after ``join()`` made the main stream wait for the dense gradient all-reduce.
        ``wgfin`` (WgFinArgs): the fused tower's dense gradient is computed inside the sparse
        backward's launch and all-gathered right after the gradient rows' all-to-all (no
        all-reduce, no comm stream); the owner launch sums the N rank gradients in rank order."""
        m = self.m
        rs = self.sets[plan[0]]
        n = B * m.F
        A = m.sf_args(n)
        A.sorted_keys, A.perm = rs.sorted_keys.data_ptr(), rs.perm.data_ptr()
        A.tv, A.tw = self.rows_in.data_ptr(), self.rows_in.data_ptr() + 4 * m.K
        A.ldv = A.ldw = self.RW
        A.sid, A.upos, A.gout = rs.sid_incl.data_ptr(), rs.upos.data_ptr(), self.send_g.data_ptr()
        if wgfin is not None:
            KN.sparse_wgfin_x(m.K, A, wgfin)
        else:
            KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
        if wgfin is not None:
            if self.dense_recv is None:
                self.dense_recv = torch.zeros(self.N * m.P, dtype=torch.float32, device=m.device)
            if hasattr(self.eng, "alltoall_allgather"):      # one aggregated RCCL operation
                self.eng.alltoall_allgather(self.send_g, self.recv_g, self.C * self.RW * 4, m.g[: m.P],
                                            self.dense_recv, m.P * 4)
            else:
                self.eng.alltoall(self.send_g, self.recv_g, self.C * self.RW * 4)
                self.eng.allgather(m.g[: m.P], self.dense_recv, m.P * 4)
            dense.g, dense.nsum = self.dense_recv.data_ptr(), self.N
        else:
            self.eng.alltoall(self.send_g, self.recv_g, self.C * self.RW * 4)
        S = ShApplyArgs()
        S.recv_ids, S.total, S.N, S.C = rs.recv[0], self.N * self.C, self.N, self.C
        S.rstride = rs.recv[1]
        S.mode = 0 if m.sparse_update == "lazy" else 1      # tags were stamped by fetch()
        S.recv_g, S.table = self.recv_g.data_ptr(), rs.table
        S.tv, S.tw = m.tv.data_ptr(), m.tw.data_ptr()
        S.s0v, S.s1v, S.s0w, S.s1w = (t.data_ptr() if t.numel() else 0 for t in m.sv)
        S.ldv, S.ldw = KN._ld(m.tv, m.tw)
        if m.sparse_update == "tf1_dense":
            S.Gv, S.Gw = m.Gv.data_ptr(), m.Gw.data_ptr()
        S.h = m.h_sparse
        S.step = m.step.data_ptr()
        if plan[2] is not None and plan[4] and m.sparse_update == "lazy":
            # the next batch's rows were served ahead: join that branch, patch what changes
            nxt = self.sets[1 - plan[0]]
            self._join_side(plan)
            S.next, S.next_rows = nxt.table, nxt.rows_out.data_ptr()
        if dense is not None:
            if join is not None:
                join()
            KN.sh_apply_dense(m.K, m.opt_id, S, dense)
            return
        KN.sh_owner_apply(m.K, m.opt_id, S)
        if m.sparse_update == "tf1_dense":
            KN.dense_sweep(m.K, m.opt_id, m.R, m.tv, m.tw, m.Gv, m.Gw, m.sv, m.h_sparse, m.step)

    def reset_table(self):
        """The tables' stamps are step numbers: clear them when the step counter is rewritten."""
        for rs in self.sets:
            rs.req_key.zero_()
            rs.req_pos.zero_()
        self.drop_served()

    def error(self) -> int:
        return int(self.err.item())
