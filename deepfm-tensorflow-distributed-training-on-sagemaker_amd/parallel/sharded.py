"""Sync-free row-sharded embedding exchange (fixed per-peer capacity) for the MI355X executor.

The reference pulls embedding rows from parameter servers and pushes gradients back every step
(PS:414-442; variable partitioning, DOC p.32).  Here the table is row-sharded over the ranks
(owner = id % N, local row = id // N) and every exchange is an RCCL all-to-all of N equal blocks
of ``capacity`` entries, issued from the native engine (csrc/kernels/comm.hip) on the compute
stream.  No split size ever crosses to the host, so the whole multi-GPU step — sort, bucketing,
the all-to-alls, forward, backward, owner update and the dense gradient exchange — is captured
into one HIP graph per resident batch, exactly like the single-GPU step (csrc/kernels/shard.hip
has the protocol).

Collective order (deadlock freedom by construction).  Every collective of a step goes through
ONE communicator, as a grouped RCCL operation on the step's MAIN stream, at fixed points:

    [inline routing only]  G0 = {ids all-to-all of this batch}
    fetch                  G1 = {rows all-to-all of this batch [, ids all-to-all of the NEXT
                                 batch when it was routed during the previous step]}
    end of the backward    G2 = {gradient rows all-to-all, dense gradient all-gather (or
                                 all-reduce) [, ids all-to-all of the NEXT batch when it is
                                 routed during this step]}

Routing KERNELS (sort, owner buckets, slot map) of upcoming batches run on a side stream; their
id exchanges join G1 / G2 on the main stream.  So each rank issues the same sequence of groups
on one communicator in one stream order -- never two operations that could wait on each other
across ranks -- whatever order the graph's branches reach the hardware queues in (``_issue``
refuses a collective off the main stream).  tests/test_gpu_shard.py records the sequence per
emulated rank and checks it is identical.

Pipeline depth.  Three routing sets rotate.  With the next TWO batches known (resident pool,
cached epoch), batch i+2 is routed during step i, its ids travel in step i+1's G1, and its rows
are then SERVED AHEAD on a side stream during step i+1 (the owner update of step i+1 patches the
rows it changes; lazy rows only) -- the serve leaves the critical path.  With only the next batch
known, it is routed during the step and its ids travel in G2 (depth 1); rows are served at the
start of their own step.

Run-level routing.  A multi-step graph over resident batches instead routes EVERY batch of the
run at its start (``route_run``: batched sort + routing launches and ONE grouped ids all-to-all,
G0 of the run) into one routing set per step; each step then only serves its rows inline, G1
(rows) and G2 (gradients + dense) -- one queue, no side branch, no cross-queue join (each join
of a branch costs the step ~10 us on MI355X, profiles/r3c_fx_kernels.md).  The collective
sequence is still fixed by the host plan alone: identical on every rank.

Capacity: the unique ids a rank sends to one owner must fit ``capacity``.  ``estimate_capacity``
measures sample batches; a bucket that overflows sets an error word that the model checks
(``NativeDeepFM.check_errors``) and raises on — rows are never silently dropped.
"""
from __future__ import annotations

import math
import os
from typing import Iterable, NamedTuple, Optional

import torch

from ..ops import kernels as KN
from ..ops._lib import ShApplyArgs, ShTable
from ..utils.knobs import flag, knob

# routing in two launches (sh_route) instead of segments + bucket (7 launches); same outputs
_ROUTE2 = flag("HIPFM_SH_ROUTE2")
# run-routed steps: the next step's rows are served by extra workgroups of the sparse backward's
# launch when it is the fused sfwg_x launch (profiles/r4h_px_serve_in_sfwg_kernels.md), else by
# workgroups of the tower's launch


_DENSE_XCHG = knob("HIPFM_DENSE_XCHG")


def dense_allreduce(world: int) -> bool:
    """The fused exchange's dense gradient: all-reduced (ring: 2 (N-1)/N x P floats per rank) or
    all-gathered and summed in rank order by the owner launch (N x P floats received, no RCCL
    reduction, in place: the default -- bitwise the same sum on every rank count's emulation and
    on hardware).  ``allreduce`` / ``auto`` (all-reduce from 4 ranks) are opt-in: RCCL's ring sum
    reassociates the rank gradients, and neither has been compared with the rank-ordered sum on
    an N >= 4 node yet."""
    return _DENSE_XCHG == "allreduce" or (_DENSE_XCHG == "auto" and world >= 4)


def overlap_branch(owner, device) -> "torch.cuda.Stream":
    """The graph branch an exchange runs its sparse backward on while the main stream carries the
    dense all-reduce (HIPFM_SH_OVERLAP); one per exchange object, created on first use."""
    st = getattr(owner, "_ovl_stream", None)
    if st is None:
        st = owner._ovl_stream = torch.cuda.Stream(device)
    return st


def reserve_staging(engine, nbytes: int):
    """Collective on transports with staging buffers (parallel/loopback.py), a no-op on RCCL:
    every rank calls it at the same host point with the same size, before any capture needs it."""
    r = getattr(engine, "reserve", None)
    if r is not None:
        r(nbytes)


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

    def group(self, ops):
        """(kind, send, recv, bytes) collectives as one grouped RCCL operation (KN.comm_group)."""
        for kind, _, _, nb in ops:
            self.bytes_sent += nb if kind == KN.COMM_ALLREDUCE else nb * self.world
        KN.comm_group(self.handle, ops)

    def close(self):
        if self.handle:
            KN.comm_destroy(self.handle)
            self.handle = 0


_ROUTED, _XCHG, _SERVED = "routed", "xchg", "served"


class _RouteSet:
    """Routing state of one batch: sorted slots, unique ids, owner buckets, received requests,
    the owner-side request table and served rows.  Depends only on the batch ids (not on the
    table) up to the serve, so upcoming batches' sets are built while the current batch trains."""

    def __init__(self, m, n: int, N: int, C: int, temp_bytes: int, RW: int):
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
        self.slot_row = torch.zeros(n, **i32)
        self.inv = None                            # run sets: inverse sort perm (sorted gradient rows)
        self.recv_ptr = self.recv_ids.data_ptr()   # requests as the owner kernels read them
        self.rstride = 0                           # (run sets: a column of the packed run buffer)
        self.slot_ld = 0                           # slot_row layout: 0 row-major, else [F][slot_ld]
        self.key = None          # host: (ids data_ptr, B) of the batch in this set
        self.stage = None        # host: _ROUTED (kernels done) / _XCHG (ids exchanged) / _SERVED
        # owner side: the request table (csrc/kernels/shard.hip) of this set's batch and its
        # served rows.  The table has a power of two >= 2x the N*C request slots; keys and per-
        # requester positions carry step stamps -- sized by the exchange, not by the table (a
        # direct [R_local][N] tag array is 7 GB per rank at the 1TB shape)
        T = N * C
        self.rows_out = torch.zeros(T, RW, dtype=torch.float32, device=dev)
        slots = 1
        while slots < 2 * T:
            slots *= 2
        self.req_key = torch.zeros(slots, dtype=torch.int64, device=dev)
        self.req_pos = torch.zeros(slots * N, dtype=torch.int64, device=dev)
        self.table = ShTable(self.req_key.data_ptr(), self.req_pos.data_ptr(), slots - 1, 0)


class CollectiveOrderError(RuntimeError):
    """A collective of the row-sharded step was about to be issued off the step's main stream."""


class ShPlan(NamedTuple):
    """Host-side routing decisions of one step (part of the captured graph's key)."""
    c: int                       # routing set of this batch (run mode: index into run_sets)
    route: bool                  # run this batch's routing kernels inline
    ids: bool                    # exchange this batch's ids inline (G0)
    serve: bool                  # serve this batch's rows at the start of the step
    n1: Optional[tuple]          # (ids address, B) of the next batch
    n1_mode: Optional[str]       # "xchg": routed earlier, ids in G1 (+ serve ahead); "route": now, ids in G2
    serve_ahead: bool            # serve the next batch's rows during this step
    n2: Optional[tuple]          # (ids address, B) of the batch after: routed during this step
    run: bool = False            # run-level routing: set c of run_sets, routed + ids exchanged at
                                 # the start of the run (route_run)


class FixedCapacityExchange:
    """Buffers + step pieces of the row-sharded exchange for one NativeDeepFM (one rank).  See
    the module docstring for the collective order and the pipeline depth."""

    NSETS = 3

    def __init__(self, m, engine, capacity: Optional[int] = None):
        self.m, self.eng = m, engine
        self.N, self.rank = engine.world, engine.rank
        dev = m.device
        K, n = m.K, m.M * m.F
        self.C = int(capacity) if capacity else default_capacity(n, self.N)
        self.C = (self.C + 63) // 64 * 64
        # exchanged rows (csrc/kernels/shard_table.h sh_row_words): served rows {v as bf16, w, 0}
        # (K/2 + 2 words; the fused gather tower reads bf16 v) or {v[K], w, 0, 0, 0} (K + 4 words);
        # gradient rows {g_v[K], g_w} (K + 1 words)
        self.rbf16 = m.exchange_rows == "bf16" and m.fused and m.gather_fused
        self.RWS = K // 2 + 2 if self.rbf16 else K + 4
        self.RWG = K + 1
        T = self.N * self.C
        f32 = dict(dtype=torch.float32, device=dev)
        self.sets = [_RouteSet(m, n, self.N, self.C, m.temp.numel(), self.RWS) for _ in range(self.NSETS)]
        self.cur = 0
        self.err = m.err_words[2:3]          # capacity overflow (the model's error words)
        self.rows_in = torch.zeros(T, self.RWS, **f32)
        self.send_g = torch.zeros(T, self.RWG, **f32)
        self.recv_g = torch.zeros(T, self.RWG, **f32)
        self._side = None
        self._serve_stream = None
        self._main = None
        self._joined = True
        self._served_ev = None
        self._next = (None, False, None, False)     # (n1 ids, n1 field-major, n2 ids, n2 fm)
        self._fork_at = None
        self._plan = None
        self.dense_recv = None               # [N][P] all-gathered dense gradients (fused exchange)
        self.trace = None                    # list: record every issued group (tests)
        self.run_sets = []                   # run-level routing: one set per step of the run
        self._run_descs = {}
        self._run_ids = None                 # packed [2][N][G][C] ids of a run (send, recv)
        self._run_retired = []               # superseded packed ids buffers (captured graphs read them)
        self.gather_ld = 0                   # slot_row layout of the last fetch (tower idx_ld)
        self.tower_serve = None              # ShServeArgs the next tower launch serves (run mode)
        self.x_serve = None                  # ... or the next sparse backward launch (sfwg_x)
        # staging of a transport that needs it (the same-device engine): the largest group of a
        # step -- G1 rows + ids, or G2 gradient rows + dense gradient + ids
        reserve_staging(engine, 4 * T * (max(self.RWS, self.RWG) + 1) + 8 * m.P + (64 << 10))

    # ------------------------------------------------------------------ host-side plan
    def plan(self, ids: torch.Tensor, B: int, nxt: Optional[torch.Tensor], resident: bool = True,
             nxt2: Optional[torch.Tensor] = None) -> ShPlan:
        """Routing decisions for one step.  Only resident batches (fixed device buffers) can have
        been prefetched: staged buffers change content under the same address."""
        c = self.cur
        key = (ids.data_ptr(), B)
        sc = self.sets[c]
        match = resident and sc.key == key
        route = not (match and sc.stage in (_ROUTED, _XCHG, _SERVED))
        ids_x = not (match and sc.stage in (_XCHG, _SERVED))
        serve = not (match and sc.stage == _SERVED)
        n1 = n2 = n1_mode = None
        ahead = False
        if nxt is not None:
            n1 = (nxt.data_ptr(), nxt.numel() // self.m.F)
            s1 = self.sets[(c + 1) % self.NSETS]
            n1_mode = "xchg" if (s1.key == n1 and s1.stage == _ROUTED) else "route"
            ahead = n1_mode == "xchg" and self.m.sparse_update == "lazy"
            if nxt2 is not None:
                n2 = (nxt2.data_ptr(), nxt2.numel() // self.m.F)
        return ShPlan(c, route, ids_x, serve, n1, n1_mode, ahead, n2)

    # ------------------------------------------------------------------ run-level routing
    def route_run(self, batches):
        """Run-level routing (a multi-step graph's start): the field sort, routing kernels and id
        exchange of EVERY batch of the run -- 2 + 3 launches and ONE grouped all-to-all on the main
        stream -- so each step of the run (``run_plan``) serves its rows, fetches them and pushes
        its gradients with no side branch and no cross-queue join.  ``batches``: [(ids [B*F] as
        the step binds them, B, field-major)], all of one B; needs the per-field sort."""
        sets, n, sort_plan, d = self.route_run_prepare(batches)
        G = len(sets)
        m = self.m
        self._main = torch.cuda.current_stream(m.device)
        m._fsort.run_sort(sort_plan)
        KN.sh_route_run(d, G, n, self.N, self.C, self.err, G * self.C, m.F, sets[0].slot_ld)
        send, recv = self._run_ids[0], self._run_ids[1]
        # G0 of the whole run: ONE all-to-all of the packed [N][G][C] ids (16 grouped all-to-alls
        # of [N][C] cost 92 us on the 1-rank proxy, RCCL's per-operation cost)
        self._issue([(KN.COMM_A2A, send, recv, G * self.C * 4)])
        self._main = None

    def route_run_prepare(self, batches):
        """Host side of ``route_run`` (allocations and device plans; call it before a capture)."""
        m = self.m
        G = len(batches)
        B = batches[0][1]
        n = B * m.F
        while len(self.run_sets) < G:
            self.run_sets.append(_RouteSet(m, m.M * m.F, self.N, self.C, m.temp.numel(), self.RWS))
        sets = self.run_sets[:G]
        grow = m.grow is not None and m.grow_sorted
        for rs in sets:
            if grow and rs.inv is None:
                rs.inv = torch.zeros(m.M * m.F, dtype=torch.int32, device=m.device)
        sort_plan = m._fsort.run_plan([(ids, b, fm, rs.sorted_keys, rs.perm, rs.inv if grow else None)
                                       for (ids, b, fm), rs in zip(batches, sets)])
        T = self.N * G * self.C
        reserve_staging(self.eng, 4 * T + (64 << 10))       # G0 of the run (packed ids all-to-all)
        if self._run_ids is None or self._run_ids.shape[1] < T:
            # a larger run: a new packed ids buffer.  The old one and the descriptors built on it
            # stay alive (graphs captured from earlier runs still read them: never freed under a
            # captured graph, which would let a replay fault on reused memory)
            if self._run_ids is not None:
                self._run_retired.append(self._run_ids)
            self._run_ids = torch.full((2, T), -1, dtype=torch.int32, device=m.device)
        ld = m.M if (m.fused and m.gather_fused) else 0     # field-major slot maps for the tower
        for g, rs in enumerate(sets):
            rs.recv_ptr = self._run_ids[1].data_ptr() + 4 * g * self.C
            rs.rstride = G * self.C
            rs.slot_ld = ld
        key = (G, n, self._run_ids.data_ptr())
        d = self._run_descs.get(key)
        if d is None:
            from ..ops._lib import ShRouteBatch
            descs = []
            for g, rs in enumerate(sets):
                r = ShRouteBatch()
                r.sk, r.perm, r.tcnt, r.sid_incl = (rs.sorted_keys.data_ptr(), rs.perm.data_ptr(),
                                                    rs.tcnt.data_ptr(), rs.sid_incl.data_ptr())
                r.send_ids = self._run_ids[0].data_ptr() + 4 * g * self.C
                r.upos, r.send_cnt = rs.upos.data_ptr(), rs.send_cnt.data_ptr()
                r.num_u, r.slot_row = rs.num_u.data_ptr(), rs.slot_row.data_ptr()
                descs.append(r)
            d = KN.struct_array_to_device(descs, m.device)
            self._run_descs[key] = d
        return sets, n, sort_plan, d

    def run_plan(self, j: int, G: int) -> ShPlan:
        """Step j of a G-step run routed by ``route_run``: G1 (rows) and G2 (gradients) only --
        nothing routed, no ids exchanged, nothing forked.  The run's first step serves its rows
        at its start; every step then serves the NEXT step's rows inside its own tower launch
        (``tower_serve``; lazy rows, fused gather tower: its owner update patches what it
        changes), so later steps start at their row all-to-all."""
        ahead = self.m.sparse_update == "lazy" and self.m.fused and self.m.gather_fused
        return ShPlan(j, False, False, j == 0 or not ahead, None, None, ahead and j + 1 < G, None, True)

    def _serve_args(self, rs: "_RouteSet", ahead: bool):
        from ..ops._lib import ShServeArgs
        m = self.m
        a = ShServeArgs()
        a.recv_ids, a.total, a.N, a.C, a.rstride = rs.recv_ptr, self.N * self.C, self.N, self.C, rs.rstride
        a.tv, a.tw = m.tv.data_ptr(), m.tw.data_ptr()
        a.ldv, a.ldw = KN._ld(m.tv, m.tw)
        a.rows, a.step, a.T = rs.rows_out.data_ptr(), m.step.data_ptr(), rs.table
        a.stamp_off, a.vbf16, a.rbf16 = (2 if ahead else 1), KN._bf(m.tv), int(self.rbf16)
        return a

    def _rs(self, plan: ShPlan) -> _RouteSet:
        return self.run_sets[plan.c] if plan.run else self.sets[plan.c]

    def commit(self, plan: ShPlan, ids: torch.Tensor = None, B: int = 0, resident: bool = True):
        """Consecutive steps rotate through the routing sets (prefetched or not), so a step's
        routing kernels never overwrite buffers an earlier step's backward still reads, even when
        graph replays run back to back.  A set is reused ONLY for the batch a caller declared as
        upcoming: never matched again by address alone (a fresh batch can get the address of an
        earlier one back from the caching allocator)."""
        if plan.run:                     # the rotating sets hold nothing for the next step
            self.invalidate()
            return
        c = plan.c
        self.sets[c].key = self.sets[c].stage = None
        s1, s2 = self.sets[(c + 1) % self.NSETS], self.sets[(c + 2) % self.NSETS]
        if plan.n1 is not None:
            s1.key, s1.stage = plan.n1, (_SERVED if plan.serve_ahead else _XCHG)
        else:
            s1.key = s1.stage = None
        if plan.n2 is not None:
            s2.key, s2.stage = plan.n2, _ROUTED
        else:
            s2.key = s2.stage = None
        self.cur = (c + 1) % self.NSETS

    def invalidate(self):
        """Forget every prefetched set (after an out-of-band use of the exchange, e.g. predict).
        A set served ahead holds request-table stamps of the NEXT step number for a batch that may
        now not be stepped: its table is cleared, or a different batch routed through it at that
        step would find stale requesters stamped current (wrong gradient sums on the owner).
        (Not inside a capture: a run graph's own steps move the step number past those stamps.)"""
        capturing = self.m.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        self.tower_serve = self.x_serve = None
        for rs in self.sets:
            if rs.stage == _SERVED and not capturing:
                rs.req_key.zero_()
                rs.req_pos.zero_()
            rs.key = rs.stage = None

    def drop_served(self):
        """Parameters changed outside a step (load / broadcast): rows served ahead are stale, so
        the next step serves its rows itself (its routing and exchanged ids stay valid)."""
        for rs in self.sets:
            if rs.stage == _SERVED:
                rs.stage = _XCHG

    # ------------------------------------------------------------------ collectives
    def _issue(self, ops):
        """Every collective of the step, as one group on the MAIN stream (the stream ``begin``
        ran on) -- the fixed issue order the module docstring argues deadlock freedom from."""
        cur = torch.cuda.current_stream(self.m.device) if self.m.device.type == "cuda" else None
        if self._main is not None and cur is not None and cur != self._main:
            raise CollectiveOrderError("row-sharded exchange: collective issued off the step's main "
                                       "stream (every collective must keep the fixed main-stream order)")
        if self.trace is not None:
            self.trace.append(tuple((k, int(nb)) for k, _, _, nb in ops))
        self.eng.group(ops)

    # ------------------------------------------------------------------ pieces
    def route_kernels(self, rs: _RouteSet, ids: torch.Tensor, B: int, fm: bool = False):
        """Sort + dedup the slot ids, bucket the unique ids by owner, slot -> received-row map
        (kernels only; the ids' all-to-all is issued by the caller on the main stream)."""
        m = self.m
        n = B * m.F
        if m.uses_field_sort(B):
            m._fsort(ids, B, rs.sorted_keys, rs.perm, field_major=fm)
        else:
            KN.sort_ids(ids, rs.sorted_keys, None, rs.perm, n, m.end_bit, rs.temp, limit=m.V,
                        err=m.err_words[3:4])
        if _ROUTE2:
            KN.sh_route(rs.sorted_keys, n, self.N, self.C, rs.tcnt, rs.sid_incl, rs.send_ids, rs.upos,
                        rs.send_cnt, rs.num_u, self.err)
        else:
            KN.segments(rs.sorted_keys, n, rs.seg_flags, rs.sid_incl, rs.ukeys, rs.seg_start, rs.num_u,
                        rs.temp)
            KN.sh_bucket(rs.ukeys, rs.num_u, n, self.N, self.C, rs.cnt_tmp, rs.send_ids, rs.upos,
                         rs.send_cnt, self.err)
        KN.sh_slot_rows(rs.perm, rs.sid_incl, rs.upos, n, rs.slot_row)

    def _ids_op(self, rs: _RouteSet):
        return (KN.COMM_A2A, rs.send_ids, rs.recv_ids, self.C * 4)

    def _set(self, plan: ShPlan, k: int) -> _RouteSet:
        return self.sets[(plan.c + k) % self.NSETS]

    def begin(self, plan: ShPlan, B: int, fork: str = "start"):
        """Start of a step (on its main stream): route the current batch if it was not prefetched
        (kernels, G0), then fork the routing kernels of the upcoming batches onto a side stream --
        here (``fork="start"``), after the row fetch (``"fetch"``), or when the caller calls
        ``fork_next`` (graph branches are dispatched in capture order)."""
        m = self.m
        self._main = torch.cuda.current_stream(m.device)
        self._plan = plan
        rs = self._rs(plan)
        if plan.route:
            self.route_kernels(rs, m.idx, B, fm=m._idx_fm)
        if plan.ids:
            self._issue([self._ids_op(rs)])                           # G0
        side_work = plan.n1_mode == "route" or plan.n2 is not None
        self._joined = not side_work
        self._fork_at = fork if side_work else None
        self._served_ev = None
        if self._fork_at == "start":
            self.fork_next()

    def fork_next(self):
        """Enqueue the upcoming batches' routing kernels on the side stream (once per step)."""
        if self._fork_at is None:
            return
        self._fork_at = None
        m, plan = self.m, self._plan
        n1_ids, n1_fm, n2_ids, n2_fm = self._next
        if self._side is None:
            self._side = torch.cuda.Stream(m.device)
        self._side.wait_stream(self._main)
        with torch.cuda.stream(self._side):
            if plan.n1_mode == "route":
                self.route_kernels(self._set(plan, 1), n1_ids, plan.n1[1], fm=n1_fm)
            if plan.n2 is not None:
                self.route_kernels(self._set(plan, 2), n2_ids, plan.n2[1], fm=n2_fm)

    def _join_side(self):
        if not self._joined:
            self.fork_next()
            self._main.wait_stream(self._side)
            self._joined = True

    def end(self, plan):
        self._join_side()
        self._main = None

    def fetch(self, plan: ShPlan, train: bool = True):
        """Owners serve the requested rows (after the previous step's updates) unless they were
        served ahead, rows come back (G1, with the next batch's ids when routed earlier; its rows
        are then served ahead on a side stream).  Training steps stamp the owner-side request
        tags with the serve (read by the update at the end of the step); eval / predict fetches
        leave them alone."""
        m = self.m
        rs = self._rs(plan)
        if plan.serve:
            if train:
                KN.sh_serve(m.K, rs.recv_ptr, self.N * self.C, self.N, m.tv, m.tw, rs.rows_out,
                            C=self.C, step=m.step, table=rs.table, rstride=rs.rstride, rbf16=self.rbf16,
                            rflag=m._xflags)
            else:
                KN.sh_serve(m.K, rs.recv_ptr, self.N * self.C, self.N, m.tv, m.tw, rs.rows_out, C=self.C,
                            rstride=rs.rstride, rbf16=self.rbf16)
        ops = [(KN.COMM_A2A, rs.rows_out, self.rows_in, self.C * self.RWS * 4)]
        if train and plan.n1_mode == "xchg":
            ops.append(self._ids_op(self._set(plan, 1)))
        self._issue(ops)                                                 # G1
        if train and plan.serve_ahead and plan.run:
            # the next run step's rows, served by extra workgroups of this step's sparse backward
            # launch (or of its tower launch)
            sv = self._serve_args(self.run_sets[plan.c + 1], ahead=True)
            if m._sp.xfuse:
                self.x_serve = sv
            else:
                self.tower_serve = sv
        elif train and plan.serve_ahead:
            # the next batch's rows as of now (stamped step + 2); this step's owner update
            # patches the rows it changes (it waits for this branch first)
            nx = self._set(plan, 1)
            if self._serve_stream is None:
                self._serve_stream = torch.cuda.Stream(m.device)
            self._serve_stream.wait_stream(self._main)
            with torch.cuda.stream(self._serve_stream):
                KN.sh_serve(m.K, nx.recv_ids, self.N * self.C, self.N, m.tv, m.tw, nx.rows_out, C=self.C,
                            step=m.step, table=nx.table, ahead=True, rbf16=self.rbf16)
                self._served_ev = torch.cuda.Event()
                self._served_ev.record(self._serve_stream)
        if train and self._fork_at == "fetch":
            self.fork_next()
        self.gather_ld = rs.slot_ld
        return (rs.slot_row,) + self.row_views()

    def row_views(self):
        """(v, w) views of the received rows as the tower's gather reads them (a bf16 v view of the
        compact rows: row stride RWS words, KN._bf true)."""
        K = self.m.K
        if self.rbf16:
            return self.rows_in.view(torch.bfloat16)[:, :K], self.rows_in[:, K // 2]
        return self.rows_in[:, :K], self.rows_in[:, K]

    def backward(self, plan: ShPlan, B: int, dense=None, join=None, wgfin=None, dense_ar=None,
                 overlap=None):
        """Per-unique gradient rows -> owners -> rank-ordered sum + row update on the owner.
        ``wgfin`` (WgFinArgs): the fused tower's dense gradient is computed inside the sparse
        backward's launch and all-gathered with the gradient rows (the owner launch sums the N
        rank gradients in rank order); else ``dense_ar`` (the flat dense gradient) is all-reduced
        in the same group, after ``join()`` made the main stream wait for its producer.
        ``dense`` (ShDenseArgs, lazy rows): the dense optimizer runs in the owner update's launch.
        The next batch's ids, when routed during this step, travel in the same group (G2).
        ``overlap`` (HIPFM_SH_OVERLAP; the callable that enqueues the dense gradient): the sparse
        backward forks onto a graph branch right after the tower, the main stream computes the dense
        gradient (``overlap()``) and all-reduces ``dense_ar`` (G2a) beside it, and the gradient rows
        follow after the join (G2b) -- two groups, still issued on the main stream in a host-fixed
        order."""
        m = self.m
        rs = self._rs(plan)
        n = B * m.F
        A = m.sf_args(n)
        A.sorted_keys, A.perm = rs.sorted_keys.data_ptr(), rs.perm.data_ptr()
        A.tv = self.rows_in.data_ptr()
        A.tw = A.tv + 4 * (m.K // 2 if self.rbf16 else m.K)
        A.ldv = A.ldw = self.RWS
        A.vbf16 = int(self.rbf16)            # (MODE 2 reads v from the received rows)
        A.sid, A.upos, A.gout = rs.sid_incl.data_ptr(), rs.upos.data_ptr(), self.send_g.data_ptr()
        if overlap is not None:
            if dense_ar is None or wgfin is not None:
                raise RuntimeError("overlapped exchange: the dense gradient is all-reduced on its own")
            side = overlap_branch(self, m.device)
            side.wait_stream(self._main)
            with torch.cuda.stream(side):
                KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
            overlap()                        # the dense gradient (wgfin launch) on the main stream
            if join is not None:
                join()
            self._issue([(KN.COMM_ALLREDUCE, dense_ar, dense_ar, dense_ar.numel() * 4)])   # G2a
            self._main.wait_stream(side)
            dense_ar = None
        elif wgfin is not None:
            sv, self.x_serve = self.x_serve, None
            KN.sparse_wgfin_x(m.K, A, wgfin, serve=sv)
        else:
            KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
        if join is not None and overlap is None:
            join()
        ops = [(KN.COMM_A2A, self.send_g, self.recv_g, self.C * self.RWG * 4)]
        if wgfin is not None and dense_allreduce(self.N):
            ops.append((KN.COMM_ALLREDUCE, m.g[: m.P], m.g[: m.P], m.P * 4))   # dense.g: m.g, nsum 0
        elif wgfin is not None:
            if self.dense_recv is None:      # (m.g is this rank's slot of it: an in-place gather)
                self.dense_recv = m.g_gather
            ops.append((KN.COMM_ALLGATHER, m.g[: m.P], self.dense_recv, m.P * 4))
            dense.g, dense.nsum = self.dense_recv.data_ptr(), self.N
        elif dense_ar is not None:
            ops.append((KN.COMM_ALLREDUCE, dense_ar, dense_ar, dense_ar.numel() * 4))
        if plan.n1_mode == "route":
            self._join_side()                # the next batch's buckets are built
            ops.append(self._ids_op(self._set(plan, 1)))
        self._issue(ops)                                                 # G2
        S = ShApplyArgs()
        S.recv_ids, S.total, S.N, S.C = rs.recv_ptr, self.N * self.C, self.N, self.C
        S.rstride = rs.rstride
        # lazy owner update (lazy rows, or the tf1_dense split form: the flagged requested rows;
        # the sweep workgroups take every other row) or the tf1_dense gradient scatter; the tags
        # were stamped by the serve
        S.mode = 0 if (m.sparse_update == "lazy" or m.tf1_xsplit) else 1
        S.recv_g, S.table = self.recv_g.data_ptr(), rs.table
        S.tv, S.tw = m.tv.data_ptr(), m.tw.data_ptr()
        S.s0v, S.s1v, S.s0w, S.s1w = (t.data_ptr() if t.numel() else 0 for t in m.sv)
        S.ldv, S.ldw = KN._ld(m.tv, m.tw)
        if m.sparse_update == "tf1_dense":
            S.Gv, S.Gw = m.Gv.data_ptr(), m.Gw.data_ptr()
        S.h = m.h_sparse
        S.step = m.step.data_ptr()
        S.vbf16 = 1 if m.emb_bf16 else 0
        S.rbf16 = int(self.rbf16)
        if plan.run and plan.serve_ahead:
            # the next run step's rows were served in this step's tower launch: patch what changes
            nx = self.run_sets[plan.c + 1]
            S.next, S.next_rows = nx.table, nx.rows_out.data_ptr()
        elif self._served_ev is not None:
            # the next batch's rows were served ahead: wait for them, patch what changes
            self._main.wait_event(self._served_ev)
            nx = self._set(plan, 1)
            S.next, S.next_rows = nx.table, nx.rows_out.data_ptr()
        if m.tf1_xsplit:
            if dense is None:
                raise RuntimeError("tf1_dense split form: the sweep rides in the owner + dense launch")
            m.sweep_fields(S)
        if dense is not None:
            KN.sh_apply_dense(m.K, m.opt_id, S, dense)
            return
        KN.sh_owner_apply(m.K, m.opt_id, S)
        if m.sparse_update == "tf1_dense":
            KN.dense_sweep(m.K, m.opt_id, m.R, m.tv, m.tw, m.Gv, m.Gw, m.sv, m.h_sparse, m.step)

    def step_bytes(self, run_steps: int = 1) -> dict:
        """Modelled traffic of one training step per rank: ``sent`` = bytes this rank sends to OTHER
        ranks (rows G1 + gradient rows G2 + dense gradient all-gather + its share of the run's ids
        all-to-all), ``moved`` = bytes its collectives deliver including its own block (what a
        1-rank proxy copies).  Fixed-capacity blocks: independent of the batch's contents."""
        N, C, P = self.N, self.C, self.m.P
        per_peer = C * (self.RWS + self.RWG) * 4 + C * 4 / max(1, run_steps) * (1 if run_steps else 0)
        if dense_allreduce(N):           # ring all-reduce: 2 (N - 1) / N of the buffer out
            ds, dm = 2 * (N - 1) * P * 4 / N, 2 * P * 4
        else:                            # all-gather: the own block to every other rank
            ds, dm = (N - 1) * P * 4, N * P * 4
        return {"sent": int((N - 1) * per_peer + ds), "moved": int(N * per_peer + dm)}

    def reset_table(self):
        """The tables' stamps are step numbers: clear them when the step counter is rewritten."""
        for rs in self.sets + self.run_sets:
            rs.req_key.zero_()
            rs.req_pos.zero_()
        self.drop_served()

    def error(self) -> int:
        return int(self.err.item())
