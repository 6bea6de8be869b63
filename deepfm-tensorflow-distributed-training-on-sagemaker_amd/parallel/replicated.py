"""Replicated-table data parallelism (Horovod parity, BASELINE config #3) as a captured step.

The reference's Horovod path keeps a full table per rank; ``DistributedOptimizer`` averages the
dense gradients with an all-reduce and all-gathers the embedding ``IndexedSlices`` -- every
slot's row gradient plus the whole-table L2 term, ``B*F + V`` rows per rank (HVD:262; SURVEY
§2.6 X2-X4).  Here each rank sends only its UNIQUE ids and their summed row gradients, in a
fixed-capacity block, so no size ever crosses to the host and the whole step is one HIP graph:

  local   : slot sort (the single-GPU side-stream / prefetched sort) -> sh_route with ONE bucket
            (unique ids in id order, per-slot unique index, capacity overflow flag) -> the fused
            sparse backward in exchange mode writes one gradient row per unique id (V read from
            the local table by id) -- and, with the fused tower, the dense gradient in the same
            launch
  exchange: ONE grouped RCCL operation on the main stream: all-gather of the [C] ids and the
            [C, K+1] gradient rows (+ the dense gradients: all-gather, summed in rank order by
            the update launch; or all-reduce).  Run-sorted steps (multi-step graphs): every
            step's ids are routed and all-gathered once at the run start, each step's requests
            are tagged by extra workgroups of its sparse launch, and its group carries the
            gradient rows (+ dense) only
  update  : every rank runs the owner-update kernel of the row-sharded path over all N ranks'
            blocks with ``rdiv = 1`` (local row = id): the lowest rank holding an id sums all
            ranks' rows IN RANK ORDER and applies the optimizer (lazy), or scatters into the
            tf1_dense gradient for the full-table sweep.  Identical arithmetic on every rank keeps
            the replicas bitwise identical; no atomics, deterministic.

The L2 term of the whole-table loss is applied inside the update (lazy: touched rows; tf1_dense:
the sweep), identically on every rank, so it never travels.  LR x N and the 1/(B*N) gradient
scale follow HVD:149 / the head kernel.
"""
from __future__ import annotations

import math
from typing import Iterable, Optional

import torch

from ..ops import kernels as KN
from ..ops._lib import ShApplyArgs, ShTable
from .sharded import dense_allreduce, overlap_branch


def estimate_unique_capacity(id_batches: Iterable[torch.Tensor], slack: float = 1.05, pad: int = 256) -> int:
    """Per-rank capacity of the replicated exchange: max unique ids of a batch, times ``slack``,
    plus ``pad``, rounded to 64."""
    mx = 0
    for ids in id_batches:
        mx = max(mx, int(torch.unique(ids.reshape(-1)).numel()))
    return int(math.ceil((mx * slack + pad) / 64.0) * 64)


class ReplicatedExchange:
    """Buffers + the backward/exchange/update piece of the replicated-table step (one rank)."""

    RUN_CAP0 = 32        # steps the packed run-ids buffers are first sized for (grown on demand)

    def __init__(self, m, engine, capacity: Optional[int] = None):
        self.m, self.eng = m, engine
        self.N, self.rank = engine.world, engine.rank
        dev = m.device
        n = m.M * m.F
        self.C = min(n, int(capacity)) if capacity else n
        self.C = (self.C + 63) // 64 * 64
        self.RW = m.K + 1                     # gradient rows {g_v[K], g_w} (shard_table.h sh_grad_words)
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.send_ids = torch.full((self.C,), -1, **i32)
        self.upos = torch.zeros(n, **i32)
        self.tcnt = torch.zeros(KN.sh_route_tiles(n) * 2, **i32)
        self.send_cnt = torch.zeros(1, **i32)
        self.num_u = torch.zeros(1, **i32)
        T = self.N * self.C
        self.g_ids = torch.full((T,), -1, **i32)
        self.g_rows = torch.zeros(T, self.RW, **f32)
        # the sparse launch writes this rank's gradient rows straight into its block of the
        # gathered rows: an in-place all-gather (no 1-rank self-copy, no local copy at N ranks)
        self.send_g = self.g_rows[self.rank * self.C:(self.rank + 1) * self.C]
        slots = 1
        while slots < 2 * T:
            slots *= 2
        self.req_key = torch.zeros(slots, dtype=torch.int64, device=dev)
        self.req_pos = torch.zeros(slots * self.N, dtype=torch.int64, device=dev)
        self.table = ShTable(self.req_key.data_ptr(), self.req_pos.data_ptr(), slots - 1, 0)
        self.err = m.err_words[2:3]           # capacity overflow (the model's error words)
        self.dense_recv = None
        self.trace = None
        self._main = None
        self.run_sets = []               # run-level routing: (sid_incl, upos, send_ids, ...) per step
        self._run_descs = {}
        self._run_j = None               # the step of the run being enqueued (runner)
        # run-level routing: every step's unique ids packed [G][C] (run_sets' send_ids are views),
        # all-gathered ONCE at the run start into [N][G][C]; each step's requests are then tagged
        # by extra workgroups of its own sparse launch (sfwg_x; else of its tower launch), off the
        # owner update's chain, and the step's exchange carries gradient rows (+ dense) only
        self.run_ids = None
        self.g_run_ids = None
        self._run_G = 0
        self._retired = []               # buffers of earlier run layouts (captured graphs use them)
        self._tagged = False
        from .sharded import reserve_staging
        reserve_staging(engine, 4 * self.C * (self.RW + 1) + 8 * m.P + (64 << 10))

    def _issue(self, ops):
        if self.trace is not None:
            self.trace.append(tuple((k, int(nb)) for k, _, _, nb in ops))
        self.eng.group(ops)

    # ------------------------------------------------------------------ run-level routing
    def route_run_prepare(self, G: int, n: int, sets):
        """Allocations and device descriptors for routing every batch of a G-step run sorted at
        its start (``sets``: the runner's (sorted keys, perm, inverse) per step).  Not in a capture."""
        m = self.m
        i32 = dict(dtype=torch.int32, device=m.device)
        if self.run_ids is None or self.run_ids.shape[0] < G:
            if self.run_ids is not None:
                # graphs captured from shorter runs keep using these buffers and the device
                # descriptors that point at them: retired, never freed
                self._retired.append((self.run_ids, self.g_run_ids, [dict(r) for r in self.run_sets],
                                      self._run_descs))
                self._run_descs = {}
            cap = max(G, self.RUN_CAP0)
            self.run_ids = torch.full((cap, self.C), -1, **i32)
            self.g_run_ids = torch.full((self.N * cap * self.C,), -1, **i32)
            for j, rs in enumerate(self.run_sets):
                rs["send_ids"] = self.run_ids[j]
        from .sharded import reserve_staging
        reserve_staging(self.eng, 4 * self.run_ids.shape[0] * self.C + (64 << 10))   # G0 of the run
        while len(self.run_sets) < G:
            self.run_sets.append(dict(sid=torch.zeros(m.M * m.F, **i32), upos=torch.zeros(m.M * m.F, **i32),
                                      send_ids=self.run_ids[len(self.run_sets)], send_cnt=torch.zeros(1, **i32),
                                      num_u=torch.zeros(1, **i32),
                                      tcnt=torch.zeros(KN.sh_route_tiles(m.M * m.F) * 2, **i32)))
        if getattr(self, "_slot_sink", None) is None or self._slot_sink.numel() < m.M * m.F:
            self._slot_sink = torch.zeros(m.M * m.F, **i32)   # (slot maps: unused by this exchange)
        key = (G, n) + tuple(s[0].data_ptr() for s in sets[:G])
        d = self._run_descs.get(key)
        if d is None:
            from ..ops._lib import ShRouteBatch
            descs = []
            for (sk, perm, _), rs in zip(sets[:G], self.run_sets[:G]):
                r = ShRouteBatch()
                r.sk, r.perm, r.tcnt, r.sid_incl = sk.data_ptr(), perm.data_ptr(), rs["tcnt"].data_ptr(), rs["sid"].data_ptr()
                r.send_ids, r.upos = rs["send_ids"].data_ptr(), rs["upos"].data_ptr()
                r.send_cnt, r.num_u, r.slot_row = rs["send_cnt"].data_ptr(), rs["num_u"].data_ptr(), self._slot_sink.data_ptr()
                descs.append(r)
            d = KN.struct_array_to_device(descs, m.device)
            self._run_descs[key] = d
        return d

    def route_run(self, d, G: int, n: int):
        """Unique rows + gradient-row positions of every batch of the run (three launches), then
        one all-gather of the run's ids (G0)."""
        KN.sh_route_run(d, G, n, 1, self.C, self.err, self.C, self.m.F, 0, slot_rows=False)
        self._run_G = G
        self._issue([(KN.COMM_ALLGATHER, self.run_ids[:G], self.g_run_ids[: self.N * G * self.C], G * self.C * 4)])

    def _run_recv(self):
        """(ids pointer, rstride) of the current run step's gathered requests ([N][G][C])."""
        G, C = self._run_G, self.C
        return self.g_run_ids.data_ptr() + 4 * self._run_j * C, G * C

    def tower_tags(self):
        """Tag-only ShServeArgs for the tower launch of the current run step (when its sparse
        backward is not the fused sfwg_x launch, which takes them itself): workgroups after the
        tower's blocks record this step's requests in the table, so the owner update needs no tag
        launch."""
        if self.m._sp.xfuse:
            return None
        a = self._tag_args()
        self._tagged = a is not None
        return a

    def _tag_args(self):
        """ShServeArgs with rows == null (tag only) of the current run step's gathered requests
        (tf1_dense split form: also flagging them for the owner launch's sweep); None outside a
        run step."""
        m = self.m
        if self._run_j is None or not (m.sparse_update == "lazy" or m.tf1_xsplit):
            return None
        from ..ops._lib import ShServeArgs
        a = ShServeArgs()
        a.recv_ids, a.rstride = self._run_recv()
        a.total, a.N, a.C = self.N * self.C, self.N, self.C
        a.rows, a.step, a.T = 0, m.step.data_ptr(), self.table
        a.stamp_off, a.rdiv = 1, 1
        if m.tf1_xsplit:
            a.rflag = m._xflags.data_ptr()
        return a

    def backward(self, B: int, dense=None, join=None, wgfin=None, dense_ar=None, overlap=None):
        """Sorted slots (m.sorted_keys / m.perm) -> unique gradient rows -> all-gather -> rank-
        ordered update of every rank's replica.  ``wgfin`` / ``dense`` / ``join`` / ``dense_ar`` as
        in ``FixedCapacityExchange.backward``."""
        m = self.m
        n = B * m.F
        if self._run_j is not None:      # routed at the run's start (route_run)
            rs = self.run_sets[self._run_j]
            sid, upos, send_ids = rs["sid"], rs["upos"], rs["send_ids"]
        else:
            sid, upos, send_ids = m.sid_incl, self.upos, self.send_ids
            KN.sh_route(m.sorted_keys, n, 1, self.C, self.tcnt, sid, send_ids, upos,
                        self.send_cnt, self.num_u, self.err)
        A = m.sf_args(n)
        A.sid, A.upos, A.gout = sid.data_ptr(), upos.data_ptr(), self.send_g.data_ptr()
        A.v_by_key = 1                      # V rows from the local replica, by id
        if overlap is not None:             # (HIPFM_SH_OVERLAP: see FixedCapacityExchange.backward)
            if dense_ar is None or wgfin is not None:
                raise RuntimeError("overlapped exchange: the dense gradient is all-reduced on its own")
            main = torch.cuda.current_stream(m.device)
            side = overlap_branch(self, m.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
            overlap()                        # the dense gradient (wgfin launch) on the main stream
            if join is not None:
                join()
            self._issue([(KN.COMM_ALLREDUCE, dense_ar, dense_ar, dense_ar.numel() * 4)])   # G2a
            main.wait_stream(side)
            dense_ar = None
        elif wgfin is not None:
            # run steps: this step's requests tagged by the launch's last workgroups (dispatched
            # into the CUs the sparse tiles' tail leaves idle)
            tags = self._tag_args()
            KN.sparse_wgfin_x(m.K, A, wgfin, serve=tags)
            self._tagged = self._tagged or tags is not None
        else:
            KN.sparse_fused(m.K, KN.SF_EXCHANGE, m.opt_id, A)
        if join is not None and overlap is None:
            join()
        tagged, self._tagged = self._tagged, False
        if self._run_j is not None:     # ids gathered at the run start
            recv_ids, rstride = self._run_recv()
            ops = [(KN.COMM_ALLGATHER, self.send_g, self.g_rows, self.C * self.RW * 4)]
        else:
            recv_ids, rstride = self.g_ids.data_ptr(), 0
            ops = [(KN.COMM_ALLGATHER, send_ids, self.g_ids, self.C * 4),
                   (KN.COMM_ALLGATHER, self.send_g, self.g_rows, self.C * self.RW * 4)]
        if wgfin is not None and dense_allreduce(self.N):
            ops.append((KN.COMM_ALLREDUCE, m.g[: m.P], m.g[: m.P], m.P * 4))   # dense.g: m.g, nsum 0
        elif wgfin is not None:
            if self.dense_recv is None:      # (m.g is this rank's slot of it: an in-place gather)
                self.dense_recv = m.g_gather
            ops.append((KN.COMM_ALLGATHER, m.g[: m.P], self.dense_recv, m.P * 4))
            dense.g, dense.nsum = self.dense_recv.data_ptr(), self.N
        elif dense_ar is not None:
            ops.append((KN.COMM_ALLREDUCE, dense_ar, dense_ar, dense_ar.numel() * 4))
        self._issue(ops)
        S = ShApplyArgs()
        S.recv_ids, S.total, S.N, S.C = recv_ids, self.N * self.C, self.N, self.C
        S.rstride, S.rdiv = rstride, 1
        # the requests' tags: stamped by the tower launch's workgroups (run steps), else by a tag
        # launch ahead of the update (mode bit 2)
        S.mode = (0 if (m.sparse_update == "lazy" or m.tf1_xsplit) else 1) | (0 if tagged else 2)
        S.recv_g, S.table = self.g_rows.data_ptr(), self.table
        S.tv, S.tw = m.tv.data_ptr(), m.tw.data_ptr()
        S.s0v, S.s1v, S.s0w, S.s1w = (t.data_ptr() if t.numel() else 0 for t in m.sv)
        S.ldv, S.ldw = KN._ld(m.tv, m.tw)
        if m.sparse_update == "tf1_dense":
            S.Gv, S.Gw = m.Gv.data_ptr(), m.Gw.data_ptr()
        S.h = m.h_sparse
        S.step = m.step.data_ptr()
        S.vbf16 = 1 if m.emb_bf16 else 0
        if m.tf1_xsplit:                    # flags from the tag kernel, l2-only sweep of the rest
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
        """Modelled traffic of one step per rank (see FixedCapacityExchange.step_bytes): this rank's
        ids + gradient-row block + dense gradient, all-gathered to the N - 1 other ranks (the ids
        once per run, the run's share per step)."""
        N, P = self.N, self.m.P
        blk = self.C * 4 + self.C * self.RW * 4
        if dense_allreduce(N):
            ds, dm = 2 * (N - 1) * P * 4 / N, 2 * P * 4
        else:
            ds, dm = (N - 1) * P * 4, N * P * 4
        return {"sent": int((N - 1) * blk + ds), "moved": int(N * blk + dm)}

    def reset_table(self):
        self.req_key.zero_()
        self.req_pos.zero_()
