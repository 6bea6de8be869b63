"""NativeDeepFM: the MI355X executor of one DeepFM training / inference step.

No autograd and no per-op dispatch: the step is a fixed sequence of hand-written gfx950
kernels over pre-allocated HBM buffers (so it can be captured once into a HIP graph and
replayed), with the backward written out explicitly:

  K1 fm_fwd        gather fm_w/fm_v rows, y_w, y_v, S = sum_f E, E and E^T (bf16)     fm.hip
  K6 gemm(FWD)     per deep layer: relu(X W^T + b) * dropout -> H, H^T            mlp.hip
  K7 head          y_d, y, sigmoid, BCE, dlogit, dZ_L, partial sums               mlp.hip
  K6 gemm(F32)     per layer: wgrad slabs (split over the batch)                  mlp.hip
  K6 gemm(DGRAD)   per layer: dZ_{i-1} = (dZ_i W_i) masked by H_{i-1} > 0         mlp.hip
  finalize         slab sums + bias row-sums -> flat dense gradient               mlp.hip
  K3 sort          radix sort of the batch ids (hipCUB)                           sparse.hip
  K2 fm_bwd        per-slot embedding row gradients in sorted order               fm.hip
  K3 reduce        reduce-by-key -> one gradient row per unique id                sparse.hip
  [sparse exchange: allgather (replicated table) or all-to-all (row-sharded)]
  K4 sparse optim  lazy row update, or tf1_dense scatter + full-table sweep        optim.hip
  K5 dense optim   flat Adam/... over MLP params + fm_bias, refreshes bf16 W, W^T   optim.hip

Numerics contract (tests/test_gpu_kernels.py): fp32 tables and optimizer state, bf16 MLP
operands with fp32 accumulation, matching models/reference.py (the TF1 transcription).
Reference parity cites: model_fn HVD:141-287, optimizer HVD:252-263, LR scaling HVD:149.
"""
from __future__ import annotations

import contextlib
import gc
import math
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..ops import kernels as KN
from .runner import GraphRunnerMixin, graph_capture  # noqa: F401  (graph_capture: re-exported)
from .state import NativeStateMixin
from . import layers as LP
from .layers import LayerPathMixin, _lds_tile_ok, _pick_splitk, _pick_tile  # noqa: F401  (re-exported)
from .step_plan import IDLE, ModeSpec, StepKnobs, StepPlan, plan_step, sfwg_possible, sweep_merges
from ..ops._lib import (TW_MAXL, BnArgs, EpiArgs, FinOpt, HeadArgs, TowerArgs, W8Job, WgFinArgs, WgFinJob,
                        WgJob, RowSumJob, SegApplyArgs, SfArgs, ShadowSeg, SlabJob)
from ..utils.rng import keep_threshold
from .reference import glorot_std, init_params, pad32
from ..utils.knobs import flag, knob


# Execution-mode switches (each one is a supported, tested mode; rejected experiments are gone)
_SORT_MODE = knob("HIPFM_SORT")                # auto | global
_SORT_SIDE_STREAM = flag("HIPFM_SORT_SIDE_STREAM")
_SPARSE_IMPL = knob("HIPFM_SPARSE")             # fused | seg
_SHARD_PIPELINE = flag("HIPFM_SHARD_PIPELINE")
_TOWER_GATHER = flag("HIPFM_TOWER_GATHER")   # FM gather fused into the tower
# weight gradients + split-K combine + bias/head reductions + dense optimizer in one launch
_WGFIN = flag("HIPFM_WGFIN")
# weight segments from this size up get their transposed bf16 shadow from a tiled pass
_SHADOW_T_MIN = 1 << 18
# single GPU, lazy rows: wgfin inside the sparse backward's launch (sparse_fused.hip sfwg_kernel)
_SFWG = flag("HIPFM_SFWG")
# one GPU, multi-step graphs: the run's batches sorted up front (fsort_run.h) instead of each
# next batch on a side branch of the step before
_RUN_SORT = flag("HIPFM_RUN_SORT")
# row-sharded lazy step: dense optimizer inside the owner update's launch
_SH_APPLY_DENSE = flag("HIPFM_SH_APPLY_DENSE")
# multi-rank lazy step: the dense all-reduce overlapped with the sparse backward (graph branch)
_SH_OVERLAP = flag("HIPFM_SH_OVERLAP")
# run-sorted single-GPU steps: the tower writes sorted per-slot gradient rows (0: the sparse launch
# gathers vals / dlogit / S / dX0 per slot)
_GROW = knob("HIPFM_GROW")     # 0 off | 1 rows at their sorted positions | 2 rows in slot order
# tf1_dense on one GPU: split sweep concurrent with the step (0: scatter + full-table sweep)
_TF1_SPLIT = flag("HIPFM_TF1_SPLIT")
_XROWS = knob("HIPFM_XROWS")
_DX0_SPLIT = knob("HIPFM_DX0_SPLIT")      # auto | 1 | 0 (tower.hip tower_dx0_kernel)
_L0_SPLIT = knob("HIPFM_L0_SPLIT")        # auto | 0 (tower.hip tower_l0s_kernel)
_SWEEP_MODE = knob("HIPFM_SWEEP_MODE")      # auto | merged | branch
_SWEEP_MBLK = 2048   # merged-mode sweep workgroups: 512 0.191, 1024 0.179, 2048 0.156, 3072 0.156, 6144 0.172 ms
_SWEEP_WG = 256      # branch sweep workgroups: 128: 0.178, 256: 0.160, 512: 0.179 ms


def step_knobs() -> StepKnobs:
    """The step planner's knob snapshot (read at call time: tests switch these module values)."""
    return StepKnobs(sort_side_stream=_SORT_SIDE_STREAM, sparse_impl=_SPARSE_IMPL,
                     wgfin=_WGFIN, sfwg=_SFWG, sh_apply_dense=_SH_APPLY_DENSE,
                     sweep_mode=_SWEEP_MODE, run_sort=_RUN_SORT,
                     shard_pipeline=_SHARD_PIPELINE, sh_overlap=_SH_OVERLAP)


def check_field_ranges(ranges, F: int, V: int) -> List[Tuple[int, int]]:
    """Validate per-field id ranges [lo, hi): one per field, non-empty, disjoint and increasing
    in field order, inside [0, V).  Returns them as a list of int pairs."""
    out = [(int(lo), int(hi)) for lo, hi in ranges]
    if len(out) != F:
        raise ValueError(f"field_ranges: expected {F} ranges, got {len(out)}")
    prev = 0
    for f, (lo, hi) in enumerate(out):
        if lo < prev or hi <= lo or hi > V:
            raise ValueError(f"field_ranges: field {f} range [{lo}, {hi}) is not disjoint/increasing "
                             f"inside [0, {V})")
        prev = hi
    return out


def field_ranges_from_sizes(sizes: Sequence[int]) -> List[Tuple[int, int]]:
    """Consecutive per-field vocabularies starting at id 0 (the usual CTR id layout)."""
    out, lo = [], 0
    for n in sizes:
        out.append((lo, lo + int(n)))
        lo += int(n)
    return out


_OPT_SLOTS = {"Adam": 2, "ftrl": 2, "Adagrad": 1, "Momentum": 1, "GD": 0}
_TABLE_LAYOUT = knob("HIPFM_TABLE_LAYOUT")     # record | split


def table_record_floats(K: int, optimizer: str, bf16: bool = False) -> int:
    """Floats per embedding-row record in the interleaved table layout:
        [ v (K) | w, w_slot0, w_slot1, pad | v_slot0 (K) | v_slot1 (K) ]  rounded up to 64 B
    (<= 16 floats) or to whole 128-B lines.  A lazy row update then reads and writes one record
    (K = 8 with Adam: exactly one 128-B line) instead of one row in each of six tables, and the
    forward gather finds v and w in the same 64-B sector.  ``bf16`` (mixed-precision embeddings):
    v and its slots are bf16 (K/2 floats each), w and its slots stay fp32 -- K = 8 with Adam is one
    64-B record, K = 32 with Adam 256 B (the Criteo-1TB table at K = 32: 226 GB, one MI355X)."""
    kv = K // 2 if bf16 else K
    x = kv + 4 + _OPT_SLOTS[optimizer] * kv
    return (x + 15) // 16 * 16 if x <= 16 else (x + 31) // 32 * 32


def _align(n: int, a: int = 64) -> int:
    return (n + a - 1) // a * a


@dataclass
class DenseSeg:
    name: str
    off: int
    shape: tuple        # native layout shape
    tf_shape: tuple     # TF checkpoint shape


class NativeDeepFM(GraphRunnerMixin, NativeStateMixin, LayerPathMixin):
    """DeepFM on one GPU (one rank).  ``comm`` (parallel.dist.Comm) adds data parallelism."""

    def __init__(self, feature_size: int, field_size: int, embedding_size: int = 32,
                 deep_layers=(256, 128, 64), keep_probs=(0.5, 0.5, 0.5), l2_reg: float = 1e-4,
                 learning_rate: float = 5e-4, optimizer: str = "Adam", loss_type: str = "log_loss",
                 sparse_update: str = "tf1_dense", seed: int = 1234, batch_size: int = 1024,
                 device="cuda", comm=None, init: bool = True, batch_norm: bool = False,
                 batch_norm_decay: float = 0.9, adam_epsilon: float = 1e-8,
                 adagrad_init: float = 1e-8, fused: Optional[bool] = None,
                 field_ranges: Optional[Sequence[Tuple[int, int]]] = None, mlp_dtype: str = "bf16",
                 emb_dtype: str = "fp32", exchange_rows: Optional[str] = None):
        self.batch_norm = bool(batch_norm)
        # row-sharded exchange: the served rows carry v as bf16 (the compute dtype; owners keep fp32
        # master rows and optimizer state) or fp32 (bitwise the one-GPU step's reads)
        self.exchange_rows = exchange_rows or _XROWS
        if self.exchange_rows not in ("bf16", "fp32"):
            raise ValueError(f"exchange_rows must be bf16 or fp32, got {self.exchange_rows!r}")
        self.bn_decay = float(batch_norm_decay)
        if mlp_dtype not in ("bf16", "fp8"):
            raise ValueError(f"mlp_dtype must be bf16 or fp8, got {mlp_dtype!r}")
        # fp8: the deep tower's forward GEMMs take OCP e4m3 operands (per-row / per-channel
        # power-of-two scales, fp32 accumulation); backward and master weights stay bf16 / fp32
        self.fp8 = mlp_dtype == "fp8"
        # mixed-precision embeddings (BASELINE config #5): fm_v rows and their optimizer slots
        # stored bf16 (stochastically rounded, counter-based: reproducible), fm_w and every
        # computation fp32 -- half the table bytes and traffic of the gather and the row update
        if emb_dtype not in ("fp32", "bf16"):
            raise ValueError(f"emb_dtype must be fp32 or bf16, got {emb_dtype!r}")
        self.emb_bf16 = emb_dtype == "bf16"
        if self.emb_bf16 and (sparse_update != "lazy" or _TABLE_LAYOUT != "record"):
            raise ValueError("emb_dtype=bf16 needs sparse_update=lazy and the record table layout")
        self.bn_eps = 1e-3          # tf.contrib.layers.batch_norm default epsilon (PS:289)
        self.V, self.F, self.K = int(feature_size), int(field_size), int(embedding_size)
        if self.K not in (4, 8, 16, 32, 64):
            raise ValueError("embedding_size must be one of 4, 8, 16, 32, 64 on the native path")
        self.layers = [int(x) for x in deep_layers]
        self.keep = [float(x) for x in keep_probs]
        self.l2 = float(l2_reg)
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.lr = float(learning_rate) * self.world          # HVD:149
        self.optimizer = optimizer
        self.adagrad_init = float(adagrad_init)
        self.opt_id = KN.OPT_IDS[optimizer]
        self.loss_type = loss_type
        self.sparse_update = sparse_update
        self.seed = int(seed)
        self.device = torch.device(device)
        self.sharded = comm is not None and comm.sharded
        # multi-rank code path (also forced on a 1-rank group by tests: comm.force_exchange)
        self.exchange = comm is not None and (self.world > 1 or getattr(comm, "force_exchange", False))
        if self.exchange and getattr(comm, "engine", None) is None:
            raise ValueError("a multi-rank NativeDeepFM needs the native RCCL engine (parallel.dist.Comm "
                             "on an RCCL process group)")
        # local rows of the embedding tables (row-sharded: id -> rank id % N, row id // N)
        self.R = (self.V + self.world - 1) // self.world if self.sharded else self.V
        self.row_div = self.world if self.sharded else 1
        self.end_bit = max(1, int(math.ceil(math.log2(max(2, self.V)))))
        # per-field id ranges [lo, hi) (disjoint, increasing): enable the one-launch per-field
        # LDS sort of the slot ids (csrc/kernels/field_sort.hip) instead of the global sort
        self.field_ranges = None
        if field_ranges is not None:
            self.field_ranges = check_field_ranges(field_ranges, self.F, self.V)

        # ---- dense parameter layout (flat fp32 buffer = one all-reduce bucket) ----
        F, K = self.F, self.K
        self.d0 = F * K
        self.K0p = pad32(self.d0)
        self.Np = [pad32(L) for L in self.layers]
        # a per-layer (unfused) tower with a wide first layer pads its input to 128 columns: the
        # layer-0 weight-gradient and dX0 GEMMs then tile on the LDS-staged 128 x 128 tile (at
        # K0p = 320 they ran on the 64 x 64 register tile: 0.75 of a 5.4 ms 4096x3 step,
        # profiles/r6tw_tower4096_kernels.md); the padding columns stay exactly zero
        if self._per_layer_tower(fused) and self.Np[0] >= 1024:
            self.K0p = (self.d0 + 127) // 128 * 128
        self.Kp = [self.K0p] + self.Np[:-1]
        segs: List[DenseSeg] = []
        off = 0

        def add(name, shape, tf_shape):
            nonlocal off
            segs.append(DenseSeg(name, off, shape, tf_shape))
            off = _align(off + int(torch.Size(shape).numel()))
        add("fm_bias", (1,), (1,))
        din = self.d0
        for i, L in enumerate(self.layers):
            add(f"Deep-part/mlp{i}/weights", (self.Np[i], self.Kp[i]), (din, L))
            add(f"Deep-part/mlp{i}/biases", (self.Np[i],), (L,))
            if self.batch_norm:     # trainable BN params live in the flat (all-reduced) buffer
                add(f"Deep-part/bn_{i}/beta", (self.Np[i],), (L,))
                add(f"Deep-part/bn_{i}/gamma", (self.Np[i],), (L,))
            din = L
        add("Deep-part/deep_out/weights", (self.Np[-1],), (din, 1))
        add("Deep-part/deep_out/biases", (1,), (1,))
        self.dense_segs: "OrderedDict[str, DenseSeg]" = OrderedDict((s.name, s) for s in segs)
        self.P = off

        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # embedding tables: fm_v [R, K], fm_w [R] and their optimizer slots are strided views of
        # one [R, RS] record buffer (table_record_floats); HIPFM_TABLE_LAYOUT=split keeps six
        # separate contiguous tables (A/B)
        self.record = _TABLE_LAYOUT == "record"
        self._kv = K // 2 if self.emb_bf16 else K          # floats of the v part of a record
        if self.record:
            self.rec_stride = table_record_floats(K, optimizer, self.emb_bf16)
            self.rec = torch.zeros(self.R, self.rec_stride, **f32)
            self.tv = self.rec.view(torch.bfloat16)[:, :K] if self.emb_bf16 else self.rec[:, :K]
            self.tw = self.rec[:, self._kv]
        else:
            self.rec = None
            self.tv = torch.zeros(self.R, K, **f32)
            self.tw = torch.zeros(self.R, **f32)
        self.p = torch.zeros(self.P, **f32)
        # multi-rank fused exchange: the dense gradients are all-gathered IN PLACE (RCCL then
        # skips the own block's copy -- a 5.3 us copy kernel per step on the 1-rank proxy,
        # profiles/r4i_px_kernels.md): this rank's gradient buffer is its slot of the gather buffer
        if self.exchange:
            self.g_gather = torch.zeros(self.world * self.P, **f32)
            self.g = self.g_gather[self.rank * self.P:(self.rank + 1) * self.P]
        else:
            self.g_gather = None
            self.g = torch.zeros(self.P, **f32)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        self._done_ctr = torch.zeros(1, dtype=torch.int32, device=dev)   # dense_opt block counter
        self._host_step = 0
        # BN moving statistics: non-trainable, outside the optimizer/all-reduce buffer
        # (rank-local, like the reference's per-worker batch_norm updates)
        self.bn_moving = torch.zeros(2 * sum(self.Np) if self.batch_norm else 0, **f32)
        self.bn_mm, self.bn_mv = [], []
        if self.batch_norm:
            o = 0
            for n in self.Np:
                self.bn_mm.append(self.bn_moving[o:o + n])
                self.bn_mv.append(self.bn_moving[o + n:o + 2 * n])
                o += 2 * n
            for t in self.bn_mv:
                t.fill_(1.0)
        self._alloc_slots()
        # tf1_dense on one GPU (record layout, fused sparse kernel): the split form -- batch rows
        # take their full update in the sparse kernel's lazy mode, every other row gets the
        # l2-only update from a sweep that runs concurrently with the step (optim.hip
        # tf1_sweep_kernel).  Byte flags per row per sorted-slot set mark the batch's rows.
        self.tf1_split = (self.sparse_update == "tf1_dense" and self.record and not self.exchange and
                          not self.sharded and
                          _TF1_SPLIT and K in (4, 8, 16, 32) and _SPARSE_IMPL == "fused" and
                          _SORT_SIDE_STREAM)
        self.lazy_rows = self.sparse_update == "lazy" or self.tf1_split   # sparse kernel mode
        if self.tf1_split:
            self._row_flags = [torch.zeros(self.R, dtype=torch.uint8, device=dev) for _ in range(2)]
            self._stamp_n = [0, 0]          # keys whose flags are set in set c, not yet swept
            self.sw_step = torch.zeros(1, dtype=torch.int64, device=dev)
            self._sw_done = torch.zeros(1, dtype=torch.int32, device=dev)
            self._sweep_stream = None
        elif self.sparse_update == "tf1_dense":
            self.Gv = torch.zeros(self.R, K, **f32)
            self.Gw = torch.zeros(self.R, **f32)
        self.W16, self.WT16 = [], []
        shadow = []
        for i in range(len(self.layers)):
            s = self.dense_segs[f"Deep-part/mlp{i}/weights"]
            w16 = torch.zeros(self.Np[i], self.Kp[i], dtype=torch.bfloat16, device=dev)
            wt16 = torch.zeros(self.Kp[i], self.Np[i], dtype=torch.bfloat16, device=dev)
            self.W16.append(w16)
            self.WT16.append(wt16)
            shadow.append(ShadowSeg(s.off, self.Np[i], self.Kp[i], w16.data_ptr(), wt16.data_ptr()))
        self._shadow_dev = KN.struct_array_to_device(shadow, dev)
        self._nshadow = len(shadow)
        # single-GPU dense optimizer (dense_opt / finalize_opt): large segments leave their
        # transposed shadow to one tiled pass after the update (the per-element transposed stores
        # cost 0.5 ms per step at 4096 x 4096 layers)
        big = [sg for sg in shadow if sg.rows * sg.cols >= _SHADOW_T_MIN]
        self._shadow_t = None
        self._shadow_opt = self._shadow_dev
        if big:
            nt = [ShadowSeg(sg.off, sg.rows, sg.cols, sg.w16, 0 if sg.rows * sg.cols >= _SHADOW_T_MIN else sg.wt16)
                  for sg in shadow]
            self._shadow_opt = KN.struct_array_to_device(nt, dev)
            self._shadow_t = (KN.struct_array_to_device(big, dev), len(big),
                              sum(((sg.rows + 63) // 64) * ((sg.cols + 63) // 64) for sg in big))
        self.W8, self.sW, self.W8amax = [], [], []
        if self.fp8:
            jobs, row0 = [], 0
            for i in range(len(self.layers)):
                s = self.dense_segs[f"Deep-part/mlp{i}/weights"]
                w8 = torch.zeros(self.Np[i], self.Kp[i], dtype=torch.uint8, device=dev)
                sw = torch.ones(self.Np[i], dtype=torch.float32, device=dev)
                am = torch.zeros(3, self.Np[i], dtype=torch.int32, device=dev)   # wgfin delayed scaling
                self.W8.append(w8)
                self.sW.append(sw)
                self.W8amax.append(am)
                jobs.append(W8Job(self.p.data_ptr() + 4 * s.off, w8.data_ptr(), sw.data_ptr(),
                                  self.Np[i], self.Kp[i], row0, 0, am.data_ptr()))
                row0 += self.Np[i]
            self._w8_jobs = KN.struct_array_to_device(jobs, dev)
            self._w8_rows = row0
        self.h_sparse = KN.hyper(self.lr, self.l2, eps=adam_epsilon)
        self.h_dense = KN.hyper(self.lr, 0.0, eps=adam_epsilon)
        # device-side error words (sticky; one D2H copy reads them all, see poll_errors):
        #   0 / 1  per-field sort (this / next batch): an id outside its field's range
        #   2      row-sharded exchange: a bucket overflowed its per-peer capacity
        #   3      global slot sort / routing: an id outside [0, V) (clamped, so nothing faults)
        #   4..7   sparse backward hand-off words (sf_sync; [6] = error bits)
        self.err_words = torch.zeros(16, dtype=torch.int32, device=dev)
        self._err_host = torch.zeros(16, dtype=torch.int32, pin_memory=dev.type == "cuda")
        self._err_ev = None
        self._bufs_M = 0
        self._side = None
        self._side_next = None
        self._run_j = None          # run-level sort: this step's index in the run (train_steps)
        self._run_n = 0             # run-level sort / routing: steps in the run being captured
        self._tower_stamp = None    # tf1_dense run step: (keys, n, flags) the tower launch stamps
        self._run_ss = []           # run-level sort: (keys, perm) per step of the run
        self._next_sort_ids = None
        self._next_fm = False      # the declared next batch's ids are field-major
        self._tf1_plan = None      # tf1_dense split sweep: (flag set, inline sort, stale keys)
        self._idx_fm = False       # the bound batch's ids (self.idx) are field-major [F, M]
        self._comm_stream = None
        self.shx = None
        self._shx_plan = None
        self._sp = IDLE            # the plan of the step being enqueued (models/step_plan.py)
        self._last_plan = IDLE
        self._sh_join = None
        self._idsT_B = 0
        self.batch_size = int(batch_size)
        # fused deep tower (csrc/kernels/tower.hip): whole forward + head + dgrad chain in one
        # launch per 32-sample block; batch norm (needs batch-wide statistics between the
        # GEMMs) and towers whose activations do not fit in LDS use the per-layer kernels
        can_fuse = (not self.batch_norm and len(self.layers) <= TW_MAXL and
                    self._tower_lds_bytes() <= 150 * 1024)
        want = (knob("HIPFM_FUSED_TOWER") != "0") if fused is None else bool(fused)
        self.fused = can_fuse and want
        # the FM gather (K1) as the fused tower's prologue: E goes straight into the tower's LDS
        # tile (no fm_fwd launch, no E round trip through HBM)
        self.gather_fused = self.fused and _TOWER_GATHER and self.K in (4, 8, 16, 32)
        if self.gather_fused and self._tower_lds_bytes() > 150 * 1024:
            self.gather_fused = False
        if self.fp8 and not self.fused:
            raise ValueError("mlp_dtype=fp8 runs on the fused tower kernel (no batch norm, "
                             "activations within LDS)")
        if self.emb_bf16 and not self.gather_fused:
            raise ValueError("emb_dtype=bf16 runs on the gather-fused tower (K in 4, 8, 16, 32; no "
                             "batch norm)")
        # sorted gradient rows (run-sorted single-GPU steps): the bf16 gather tower writes every
        # slot's embedding gradient row to its sorted position; the sparse launch streams them
        # dX0 in a launch of its own (tower.hip tower_dx0_kernel, bit-identical): below 4096 rows
        # the tower has < 128 blocks, and each would compute all K0p / 32 dX0 tiles alone
        # (decided once, from the constructed batch: the K = 32 gradient rows depend on it)
        self.dx0_split = self.fused and not self.fp8 and (
            _DX0_SPLIT == "1" or (_DX0_SPLIT == "auto" and self._padM(self.batch_size) < 4096))
        # (K = 32: the dX0 launch writes the rows -- the tower has no LDS left for their scratch)
        self.grow_ok = (self.gather_fused and not self.fp8 and self.F <= 64 and _GROW != "0" and
                        ((self.K in (4, 8, 16) and self._tower_grow_layout()[1] <= 150 * 1024) or
                         (self.K == 32 and self.dx0_split)))
        self.grow_sorted = _GROW == "1"      # (else slot order: the sparse launch gathers through perm)
        # the FM gather + layer 0 over ~8 field slices in a launch of their own (tower.hip
        # tower_l0s_kernel; the batches of the dX0 split: the tower's 32-row blocks are too few
        # to fill the GPU, and each gathered all F fields and reduced all K0p / 32 k-steps alone)
        self.l0s = self.l0_ks = 0
        if (_L0_SPLIT != "0" and self.gather_fused and not self.fp8 and self.K in (4, 8, 16, 32) and
                self.dx0_split):
            T = self.K0p // 32
            ks = max(1, -(-T // 8))
            if -(-T // ks) >= 2:
                self.l0s, self.l0_ks = -(-T // ks), ks
        if init:
            if self.V * self.K <= (1 << 24):
                # small tables: the exact golden initialization (CPU generator, bit-reproducible)
                self.load_tf_params(init_params(self.V, F, K, self.layers, self.batch_norm,
                                                self.seed))
            else:
                # huge tables (Criteo-1TB shape): same distributions, generated in place on the
                # GPU per rank (no host staging, no full-table temporary)
                self.load_tf_params(init_params(self.V, F, K, self.layers, self.batch_norm,
                                                self.seed, tables=False))
                self.init_tables_inplace()
        self._alloc_step_buffers(self._padM(self.batch_size))

    # ------------------------------------------------------------------ allocation
    def init_tables_inplace(self):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed * 7919 + (self.rank if self.sharded else 0))
        with torch.no_grad():
            for t, shape in ((self.tw, (self.V,)), (self.tv, (self.V, self.K))):
                std = glorot_std(shape)
                if t.dtype == torch.float32:
                    torch.nn.init.trunc_normal_(t, 0.0, std, -2 * std, 2 * std, generator=g)
                    continue
                step = 1 << 24              # bf16 rows: drawn in fp32, rounded per row block
                for a in range(0, t.shape[0], step):
                    blk = torch.empty(t[a:a + step].shape, dtype=torch.float32, device=t.device)
                    torch.nn.init.trunc_normal_(blk, 0.0, std, -2 * std, 2 * std, generator=g)
                    t[a:a + step].copy_(blk)

    def _alloc_slots(self):
        f32 = dict(dtype=torch.float32, device=self.device)
        R, K, P = self.R, self.K, self.P
        e = torch.empty(0, **f32)
        o = self.optimizer
        ns = _OPT_SLOTS[o]
        init = {"Adagrad": self.adagrad_init, "ftrl": 0.1}.get(o, 0.0)   # slot-0 initial value
        if self.record:
            rec, kv = self.rec, self._kv
            if self.emb_bf16:
                rb, o = rec.view(torch.bfloat16), 2 * (kv + 4)
                s0v, s1v = rb[:, o: o + K], rb[:, o + K: o + 2 * K]
            else:
                s0v, s1v = rec[:, kv + 4: kv + 4 + K], rec[:, kv + 4 + K: kv + 4 + 2 * K]
            s0w, s1w = rec[:, kv + 1], rec[:, kv + 2]
        else:
            s0v, s1v = torch.zeros(R, K, **f32), torch.zeros(R, K, **f32)
            s0w, s1w = torch.zeros(R, **f32), torch.zeros(R, **f32)
        self.sv = [s0v if ns >= 1 else e, s1v if ns >= 2 else e,
                   s0w if ns >= 1 else e, s1w if ns >= 2 else e]
        self.sd = [torch.zeros(P, **f32) if ns >= 1 else e, torch.zeros(P, **f32) if ns >= 2 else e]
        if init:
            with torch.no_grad():
                for t in (self.sv[0], self.sv[2], self.sd[0]):
                    t.fill_(init)

    def _tower_lds_layout(self):
        """(H tile offsets, dZ tile offsets, bf16 E tile offset, fp8 E tile byte offset, bytes):
        H tiles, then the dZ region -- which also holds the gathered bf16 E tile, dead before the
        first dZ tile is written -- then (fp8 + gather) the fp8 E tile."""
        off, h_off = 0, []
        for n in self.Np:
            h_off.append(off)
            off += 32 * (n + 8)
        dz = 32 * (max(self.Np) + 8)
        gather = getattr(self, "gather_fused", False)
        region = max(2 * dz, 32 * (self.K0p + 8) if gather else 0)
        dz_off = [off, off + dz]
        x_off = off if gather else -1
        nbytes = 2 * (off + region)
        x8_off = -1
        if gather and self.fp8:
            x8_off = (nbytes + 15) // 16 * 16
            nbytes = x8_off + 32 * (self.K0p + 16)
        return h_off, dz_off, x_off, x8_off, nbytes

    def _tower_lds_bytes(self) -> int:
        return self._tower_lds_layout()[4]

    def _per_layer_tower(self, fused) -> bool:
        """The fused-tower decision of the constructor, made before the dense layout exists
        (it depends on the layer widths only: the gather's E tile is checked separately)."""
        lds = 2 * (sum(32 * (n + 8) for n in self.Np) + 2 * 32 * (max(self.Np) + 8))
        can_fuse = not self.batch_norm and len(self.layers) <= TW_MAXL and lds <= 150 * 1024
        want = (knob("HIPFM_FUSED_TOWER") != "0") if fused is None else bool(fused)
        return not (can_fuse and want)

    def _tower_grow_layout(self):
        """(byte offset, total LDS bytes) of the tower's sorted-gradient-row scratch, appended to
        the layout above: x [32][F] f32, S [32][K] f32, inverse perm [32][F] i32, and the 4 wave
        tiles [32][40] bf16 of tower.hip tw_grow_tile -- in the H tiles' region (dead by the dX0
        phase) when it holds them, so the launch stays small enough for 3 workgroups per CU (the
        run-routed step's serve workgroups co-reside with the tower's two per CU)."""
        g_off = (self._tower_lds_bytes() + 15) // 16 * 16
        hbytes = sum(2 * 32 * (n + 8) for n in self.Np)
        wt = 0 if hbytes >= 4 * 32 * 40 * 2 else 4 * 32 * 40 * 2
        return g_off, g_off + 32 * (8 * self.F + 4 * self.K) + wt

    @staticmethod
    def _padM(B: int) -> int:
        return max(128, (B + 127) // 128 * 128)

    def _alloc_step_buffers(self, M: int):
        """Per-step activations/gradients for a (padded) batch of M rows."""
        if M <= self._bufs_M:
            return
        dev = self.device
        F, K, K0p = self.F, self.K, self.K0p
        bf = dict(dtype=torch.bfloat16, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.M = M
        self.idx = torch.zeros(M * F, **i32)
        self.vals = torch.zeros(M * F, **f32)
        self.labels = torch.zeros(M, **f32)
        self.y_fm = torch.zeros(M, **f32)
        self.S = torch.zeros(M, K, **f32)
        self.E = torch.zeros(M, K0p, **bf)
        self.Et = torch.zeros(K0p, M, **bf)
        if self.fp8:
            self.E8 = torch.zeros(M, K0p, dtype=torch.uint8, device=dev)
            self.sE = torch.ones(M, **f32)
        self.H = [torch.zeros(M, n, **bf) for n in self.Np]
        self.Ht = [torch.zeros(n, M, **bf) for n in self.Np]
        self.dZ = [torch.zeros(M, n, **bf) for n in self.Np]
        self.dZt = [torch.zeros(n, M, **bf) for n in self.Np]
        self.dX0 = torch.zeros(M, K0p, **bf)            # layer-1 input gradient (bf16)
        if getattr(self, "l0s", 0):                      # split gather + layer 0: fp32 partials
            self.l0z = torch.zeros(self.l0s, M, self.Np[0], **f32)
            self.l0fm = torch.zeros(self.l0s, M, K + 2, **f32)
        # per-slot gradient rows in sorted order (run-sorted steps, tower.hip tw_grow_tile)
        self.grow = torch.zeros(M * F, K + 2, **f32) if getattr(self, "grow_ok", False) else None   # {a[K], g_w, c}
        self._grow_inv = None
        if self.batch_norm:
            self.Rb = [torch.zeros(M, n, **f32) for n in self.Np]         # relu output (pre-BN)
            self.dH = [torch.zeros(M, n, **f32) for n in self.Np]         # dL/d(layer output)
            self.bn_save = [torch.zeros(6, n, **f32) for n in self.Np]
            self.bn_part = torch.zeros(M // 64, 2 * max(self.Np), **f32)
        self.prob = torch.zeros(M, **f32)
        self.dlogit = torch.zeros(M, **f32)
        # head partial rows: one per 64-sample head workgroup, or per 32-sample tower block
        self.nhead = M // 32 if self.fused else (M + 63) // 64
        self.partial = torch.zeros(self.nhead, self.Np[-1] + 2, **f32)
        self.loss_sum = torch.zeros(1, **f32)
        # wgrad split-K configuration + slabs
        self.wg_cfg = []
        for i in range(len(self.layers)):
            Mg, Ng, Kd = self.Np[i], self.Kp[i], M
            if self.fused:
                s = 32          # per-layer weight-gradient split-K workgroups
                while s > 1 and (M % (32 * s) or M // s < 128):
                    s //= 2
                self.wg_cfg.append((None, s))
                continue
            t = LP._pick_tile(Mg, Ng, row_major_stream=False, Kd=Kd)
            if t not in (KN.TILE_LDS, KN.TILE_PP) and LP._LDS_GEMM and LP._lds_tile_ok(Mg, Ng, Kd, splitk=4):
                t = KN.TILE_LDS     # (few output tiles, but the batch reduction splits 4+ ways)
            bm, bn = KN.TILES[t]
            if t == KN.TILE_PP and LP._WG_DIRECT and (Mg // bm) * (Ng // bn) >= 256:
                # one 256x256 tile per CU already: unsplit, straight into g (the library GEMM by
                # default; the 4096 x 384 layer-0 one stays on the split LDS tile + finalize: 90 +
                # 14 us vs hipBLASLt's 107, profiles/r6tw_blas_kernels.md)
                s = 0
            else:
                s = LP._pick_splitk(Mg, Ng, Kd, t)
            self.wg_cfg.append((t, s))
        self.wg_direct = [s == 0 for (t, s) in self.wg_cfg]
        self.wg_cfg = [(t, max(s, 1)) for (t, s) in self.wg_cfg]
        self.slabs = [torch.zeros(0 if d else s, self.Np[i], self.Kp[i], **f32)
                      for i, ((t, s), d) in enumerate(zip(self.wg_cfg, self.wg_direct))]
        # fp32 product scratch of the library-GEMM forward / dgrad (layers._epi_blas_ok)
        cn = [] if (self.fused or self.batch_norm) else (
            [self.Np[i] for i in range(len(self.layers)) if LP._epi_blas_ok(M, self.Np[i], self.Kp[i])]
            + [self.Np[i - 1] for i in range(1, len(self.layers)) if LP._epi_blas_ok(M, self.Np[i - 1], self.Np[i])])
        self.cbuf = torch.empty(M * max(cn) if cn else 0, **f32)
        # sparse path
        n = M * F
        gr = KN.grad_row_floats(K)
        self.sorted_keys = torch.zeros(n, **i32)
        self.perm = torch.zeros(n, **i32)
        self.G = torch.zeros(n, gr, **f32)          # per-unique partial sums (fused backward)
        self.UG = torch.zeros(n, gr, **f32)
        self.cont = torch.zeros(KN.seg_tiles(K, n) + 1, gr, **f32)
        self.ukeys = torch.zeros(n, **i32)
        self.num_u = torch.zeros(1, **i32)
        self.seg_flags = torch.zeros(n, **i32)
        self.sid_incl = torch.zeros(n, **i32)
        self.seg_start = torch.zeros(n + 1, **i32)
        nt = KN.sparse_fused_tiles(K, n)
        self.sf_ctail = torch.zeros(nt, K + 4, **f32)
        self.sf_lead = torch.zeros(nt, K + 4, **f32)
        self.sf_tinfo = torch.zeros(nt, 4, **i32)
        # in-launch hand-off words of the sparse tile kernel (csrc/kernels/sync.h): per-tile
        # publication flags (tagged with the step index) and error bits; zeroed whenever the
        # step counter is rewritten (_reset_sync)
        self.sf_flags = torch.zeros(nt, **i32)
        self.sf_sync = self.err_words[4:8]
        self.sf_sync.zero_()
        self._fsort = None
        self._fsort_next = None
        # sorted-slot sets: set c holds the sort of the batch this step trains, set 1 - c receives
        # the sort of the NEXT batch, computed on a side stream during this step (single GPU,
        # next batch declared by the caller); the two sets alternate step by step
        if getattr(self, "tf1_split", False) and any(self._stamp_n):
            for f in self._row_flags:
                f.zero_()
            self._stamp_n = [0, 0]
        self._ss = [(self.sorted_keys, self.perm),
                    (torch.zeros(n, **i32), torch.zeros(n, **i32))]
        self._ss_key = [None, None]
        self._ss_cur = 0
        self._sort_plan = None
        self._make_field_sorts()
        tb = max(KN.radix_temp_bytes(n), KN.rbk_temp_bytes(K, n), KN.scan_temp_bytes(n))
        self.temp = torch.zeros(tb + 256, dtype=torch.uint8, device=dev)
        self._build_finalize_jobs()
        if self.fused:
            self._build_wgrad_jobs()
            self._build_wgfin()
        self._bufs_M = M
        self.shx = None
        self._shx_eval = None
        self.rpx = None
        if self.sharded and getattr(self.comm, "engine", None) is not None:
            from ..parallel.sharded import FixedCapacityExchange
            self.shx = FixedCapacityExchange(self, self.comm.engine, self.comm.capacity)
        elif self.exchange and getattr(self.comm, "engine", None) is not None:
            # replicated table (Horovod parity): fixed-capacity all-gather of unique gradient rows
            from ..parallel.replicated import ReplicatedExchange
            self.rpx = ReplicatedExchange(self, self.comm.engine, self.comm.capacity)
        # tf1_dense under the native exchange, split form: the rows requested this step (any rank)
        # take their full update in the lazy owner launch and get a byte flag (set by the serve /
        # tag kernel); every other local row gets its l2-only update from sweep workgroups of the
        # same launch (instead of a [R, K] gradient scatter plus a full-table sweep)
        self.tf1_xsplit = (self.sparse_update == "tf1_dense" and self.record and _TF1_SPLIT and self.fused and
                           (self.shx is not None or self.rpx is not None) and self.K in (4, 8, 16, 32) and
                           not self.emb_bf16 and _SH_APPLY_DENSE and _WGFIN and
                           getattr(self, "_wgfin_ns", 1 << 30) <= KN.SFWG_MAX_NS)
        self._xflags = torch.zeros(self.R, dtype=torch.uint8, device=dev) if self.tf1_xsplit else None
        self._own_in = (self.idx, self.vals, self.labels)
        self._drop_graphs()
        self.max_graphs = 256
        self._graph = None

    def _make_field_sorts(self):
        self._fsort = self._fsort_next = None
        if self.field_ranges is None:
            return
        M, dev = self.M, self.device
        # the sort runs on a side stream next to the step in both cases, and every sort
        # workgroup holds 148 KB of LDS: one workgroup per field on one GPU (0.160 ms/step vs
        # 0.162 / 0.169 / 0.179 with 2 / 4 / 16 per field); 4 per field for the next batch's
        # routing on the sharded step (0.198 ms vs 0.206 with 16; HIPFM_FSORT_PB overrides)
        pb = knob("HIPFM_FSORT_PB")
        self._fsort = KN.FieldSort(self.field_ranges, min(M, KN.field_sort_max_rows()), dev,
                                   max_pb=int(pb) if pb is not None else (2 if self.sharded else 0),
                                   err=self.err_words[0:1])
        if not self.sharded:
            self._fsort_next = KN.FieldSort(self.field_ranges, min(M, KN.field_sort_max_rows()),
                                            dev, max_pb=int(pb) if pb is not None else 0,
                                            err=self.err_words[1:2])

    def exchange_capacity(self) -> Optional[int]:
        """Block capacity of the native fixed-size exchange (None without one)."""
        x = self.shx if self.shx is not None else self.rpx
        return None if x is None else x.C

    def set_exchange_capacity(self, capacity: int):
        """Re-plan the fixed-size exchange with a measured capacity (every rank the same value):
        new exchange buffers, routing sets and request tables; captured graphs are dropped."""
        self.comm.capacity = int(capacity)
        if self.shx is not None:
            from ..parallel.sharded import FixedCapacityExchange
            old = self.shx
            self.shx = FixedCapacityExchange(self, self.comm.engine, self.comm.capacity)
            # the capacity was measured on training batches: evaluation / predict keep the larger
            # exchange (same capacity on every rank: the uncalibrated default)
            if self.shx.C < old.C and getattr(self, "_shx_eval", None) is None:
                old.invalidate()
                self._shx_eval = old
        elif self.rpx is not None:
            from ..parallel.replicated import ReplicatedExchange
            self.rpx = ReplicatedExchange(self, self.comm.engine, self.comm.capacity)
        self._drop_graphs()

    def set_field_ranges(self, ranges):
        """Per-field id ranges found after construction (e.g. derived while caching the first
        epoch): switches the slot sort to the one-launch per-field LDS sort."""
        self.field_ranges = None if ranges is None else check_field_ranges(ranges, self.F, self.V)
        self._make_field_sorts()
        self._ss_key = [None, None]
        self._drop_graphs()

    def _build_wgfin(self):
        """wgfin_kernel configuration (tower.hip): NS workgroup splits of the batch per 32x32
        output tile, 4 waves each; slabs, bias slabs, arrival counters."""
        M, dev = self.M, self.device
        f32 = dict(dtype=torch.float32, device=dev)
        # 4 workgroup splits x 4 waves: same-box A/B 0.1214 (4) / 0.1228 (8) / 0.126 (16) ms/step;
        # fewer at small batches, so every wave keeps >= 8 k-steps of 32 rows: at B = 1024 (the
        # reference workload) 4 splits gave each wave 2 k-steps and 665 workgroups to dispatch ahead
        # of the sparse tiles -- 0.0832-0.0837 (4) / 0.0764-0.0767 (2) / 0.0763-0.0764 (1) ms/step,
        # while B = 16384 keeps 4: 0.1028-0.1037 (4) / 0.1038-0.1042 (2) / 0.131 (1)
        # (profiles/r6_wgfin_splits_ab.log)
        ns = 4          # wgfin workgroups per output tile (8 / 16: equal or slower)
        while ns > 1 and (M % (ns * 4 * 32) or M // (ns * 4 * 32) < 8):
            ns //= 2
        self._wgfin_ns = ns
        self.wf_slabs, self.wf_bslabs, jobs = [], [], []
        tile0 = wg0 = 0
        g0 = self.g.data_ptr()
        for i in range(len(self.layers)):
            Np, Kp = self.Np[i], self.Kp[i]
            sl = torch.zeros(ns, Np, Kp, **f32)
            bsl = torch.zeros(ns, Np, **f32)
            self.wf_slabs.append(sl)
            self.wf_bslabs.append(bsl)
            Xt = self.Et if i == 0 else self.Ht[i - 1]
            j = WgFinJob()
            j.A, j.B, j.slab, j.bslab = self.dZt[i].data_ptr(), Xt.data_ptr(), sl.data_ptr(), bsl.data_ptr()
            j.gw = g0 + 4 * self.dense_segs[f"Deep-part/mlp{i}/weights"].off
            j.gb = g0 + 4 * self.dense_segs[f"Deep-part/mlp{i}/biases"].off
            j.w16, j.wt16 = self.W16[i].data_ptr(), self.WT16[i].data_ptr()
            if self.fp8:      # the optimizer tail also writes the fp8 weights (no w8_quant launch)
                j.w8, j.sdq, j.amax3 = (self.W8[i].data_ptr(), self.sW[i].data_ptr(),
                                        self.W8amax[i].data_ptr())
            j.M, j.N, j.tiles_m, j.tiles_n = Np, Kp, Np // 32, Kp // 32
            j.tile0, j.wg0 = tile0, wg0
            tile0 += j.tiles_m * j.tiles_n
            wg0 += j.tiles_m * j.tiles_n * ns
            jobs.append(j)
        self._wgfin_jobs = KN.struct_array_to_device(jobs, dev)
        self._wgfin_ntiles, self._wgfin_wgs = tile0, wg0
        self.wf_tile_ctr = torch.zeros(max(1, tile0), dtype=torch.int32, device=dev)
        self.wf_done_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        self.sfwg_done = torch.zeros(1, dtype=torch.int32, device=dev)

    def _wgfin_args(self, with_opt: bool) -> WgFinArgs:
        a = WgFinArgs()
        a.jobs, a.njobs = self._wgfin_jobs.data_ptr(), len(self.layers)
        a.ldk, a.ns = self.M, self._wgfin_ns
        a.kchunk = self.M // (a.ns * 4)
        a.tile_wgs = self._wgfin_wgs
        a.tile_ctr, a.done_ctr = self.wf_tile_ctr.data_ptr(), self.wf_done_ctr.data_ptr()
        a.partial, a.nhead, a.L = self.partial.data_ptr(), self.nhead, self.Np[-1]
        g0 = self.g.data_ptr()
        a.g_wout = g0 + 4 * self.dense_segs["Deep-part/deep_out/weights"].off
        a.g_bout = g0 + 4 * self.dense_segs["Deep-part/deep_out/biases"].off
        a.g_fmbias = g0 + 4 * self.dense_segs["fm_bias"].off
        a.loss_sum = self.loss_sum.data_ptr()
        o = FinOpt()
        o.p, o.g, o.s0, o.s1, o.n = (self.p.data_ptr(), g0, self.sd[0].data_ptr() if self.sd[0].numel() else 0,
                                     self.sd[1].data_ptr() if self.sd[1].numel() else 0, self.P)
        o.h = self.h_dense
        o.step = self.step.data_ptr()
        o.segs, o.nseg = self._shadow_dev.data_ptr(), self._nshadow
        a.o = o
        a.opt_on = 1 if with_opt else 0
        return a

    def _dense_grads(self):
        """Weight / bias / head gradients of the fused tower (+ the dense optimizer when this step
        fuses it): one wgfin launch, or wgrad_group + finalize (HIPFM_WGFIN=0)."""
        if _WGFIN:
            KN.wgfin(self.opt_id if self._sp.fuse_opt else -1, self._wgfin_args(self._sp.fuse_opt))
            return
        KN.wgrad_group(self._wg_jobs, self._nwg_jobs, self._wg_tasks)
        self._finalize_grads()

    def _build_wgrad_jobs(self):
        jobs, task0 = [], 0
        M = self.M
        for i in range(len(self.layers)):
            s = self.wg_cfg[i][1]
            Xt = self.Et if i == 0 else self.Ht[i - 1]
            j = WgJob()
            j.A, j.B, j.out = self.dZt[i].data_ptr(), Xt.data_ptr(), self.slabs[i].data_ptr()
            j.lda = j.ldb = M
            j.M, j.N = self.Np[i], self.Kp[i]
            j.tiles_m, j.tiles_n = self.Np[i] // 32, self.Kp[i] // 32
            j.splitk, j.kchunk = s, M // s
            j.task0 = task0
            task0 += j.tiles_m * j.tiles_n * s
            jobs.append(j)
        self._wg_jobs = KN.struct_array_to_device(jobs, self.device)
        self._nwg_jobs = len(jobs)
        self._wg_tasks = task0

    def _tower_args(self, B: int, train: bool, with_labels: bool = True, gather=None, grow: bool = False,
                    grow_inv=None) -> TowerArgs:
        """``gather`` = (idx, tv, tw): the tower's prologue gathers the FM rows itself.
        ``grow``: write per-slot gradient rows -- at their sorted positions (``grow_inv``, the
        batch's inverse sort permutation) or in slot order (``grow_sorted`` off)."""
        a = TowerArgs()
        nl = len(self.layers)
        a.M, a.nvalid, a.nl, a.K0p = self.M, B, nl, self.K0p
        pb = self.p.data_ptr()
        h_off, dz_off, x_off, x8_off, nbytes = self._tower_lds_layout()
        for i in range(nl):
            a.Np[i] = self.Np[i]
            a.W[i] = self.W16[i].data_ptr()
            a.WT[i] = self.WT16[i].data_ptr()
            a.bias[i] = pb + 4 * self.dense_segs[f"Deep-part/mlp{i}/biases"].off
            keep = self.keep[i]
            a.keep_thr[i] = min(keep_threshold(keep), 0xFFFFFFFF)
            a.inv_keep[i] = (1.0 / keep) if keep < 1.0 else 1.0
            a.drop[i] = 1 if keep < 1.0 else 0
            a.Ht[i] = self.Ht[i].data_ptr() if i + 1 < nl else 0    # (H_last^T feeds no GEMM)
            a.dZt[i] = self.dZt[i].data_ptr()
            a.h_off[i] = h_off[i]
        a.dz_off[0], a.dz_off[1] = dz_off
        a.lds_bytes = nbytes
        a.x_off, a.x8_off = x_off, x8_off
        if gather is not None:
            idx, tv, tw = gather
            a.idx, a.vals, a.tv, a.tw = idx.data_ptr(), self.vals.data_ptr(), tv.data_ptr(), tw.data_ptr()
            # field-major bound ids (the sharded step gathers through its row-major slot map)
            a.idx_ld = self.M if (self._idx_fm and idx is self.idx) else 0
            if self.shx is not None and idx is not self.idx:
                a.idx_ld = self.shx.gather_ld           # run-routed slot maps are field-major
            a.ldv, a.ldw = KN._ld(tv, tw)
            a.fm_bias = pb + 4 * self.dense_segs["fm_bias"].off
            a.F = self.F
            a.S = self.S.data_ptr()
            a.Et = self.Et.data_ptr() if train else 0
            a.id_lim = tv.shape[0]
            a.vbf16 = KN._bf(tv)
        else:
            a.E = self.E.data_ptr()
        if self.fp8:
            a.fp8 = 1
            if gather is None:
                a.E8, a.sE = self.E8.data_ptr(), self.sE.data_ptr()
            for i in range(nl):
                a.W8[i], a.sW[i] = self.W8[i].data_ptr(), self.sW[i].data_ptr()
        if train and self.dx0_split:
            a.dx0_split = 1
        if gather is not None and self.l0s and (a.dx0_split or not grow):
            a.l0s, a.l0_ks = self.l0s, self.l0_ks
            a.l0z, a.l0fm = self.l0z.data_ptr(), self.l0fm.data_ptr()
        if grow:
            a.grow, a.inv_ld = self.grow.data_ptr(), B                  # (run-sorted: B == M)
            a.inv = grow_inv.data_ptr() if self.grow_sorted else 0
            if not a.dx0_split:    # (the tower writes the rows: its scratch layout; else the dX0
                a.g_off, a.lds_bytes = self._tower_grow_layout()      # launch reads S from HBM)
                a.S = 0                        # (the sparse launch reads the rows instead)
        a.seed = self.seed & 0xFFFFFFFF
        a.train = 1 if train else 0
        a.square_loss = 1 if self.loss_type == "square_loss" else 0
        a.gscale = 1.0 / (B * self.world)
        a.step = self.step.data_ptr()
        a.w_out = pb + 4 * self.dense_segs["Deep-part/deep_out/weights"].off
        a.b_out = pb + 4 * self.dense_segs["Deep-part/deep_out/biases"].off
        a.y_fm = self.y_fm.data_ptr()
        a.labels = self.labels.data_ptr() if with_labels else 0
        a.dX0 = self.dX0.data_ptr()
        a.prob = self.prob.data_ptr()
        a.dlogit = self.dlogit.data_ptr()
        a.partial = self.partial.data_ptr()
        return a

    def _dense_fwd_bwd(self, B: int, defer_wgrad: bool = False, after_fm=None):
        """Forward, loss head and the whole deep-tower backward (dense grads into self.g, dX0
        for the FM backward).  Returns the (idx, table) pair the sparse backward uses.
        ``defer_wgrad``: stop after the fused tower (the caller runs wgrad + finalize).
        ``after_fm``: hook called once the FM forward is enqueued."""
        if self.fused and self.gather_fused:
            idx, tv, tw = self._fm_inputs(B, train=True)
            ta = self._tower_args(B, train=True, gather=(idx, tv, tw),
                                  grow=self._sp.grow_rows, grow_inv=self._grow_inv)
            if self.shx is not None and self.shx.tower_serve is not None:
                # run-routed step: the next step's rows served by extra tower workgroups
                ta.sv, self.shx.tower_serve = self.shx.tower_serve, None
                ta.serve_wgs = -(-ta.sv.total * (self.K // 4) // 256)
            elif self.rpx is not None and (sv := self.rpx.tower_tags()) is not None:
                # replicated run step: this step's requests tagged by extra tower workgroups
                ta.sv = sv
                ta.serve_wgs = -(-sv.total // 256)         # (one thread per request)
            if self._tower_stamp is not None:
                # tf1_dense run-sorted step: this batch's row flags set by extra tower workgroups
                keys, n, flags = self._tower_stamp
                self._tower_stamp = None
                ta.stamp_keys, ta.stamp_n, ta.stamp_div, ta.stamp_flags = keys.data_ptr(), n, self.row_div, flags.data_ptr()
                ta.stamp_wgs = -(-n // KN.tower_stamp_rows_per_wg())
            KN.tower(ta, KE=self.K)
            if after_fm is not None:
                after_fm()
            if not defer_wgrad:
                self._dense_grads()
            return idx, tv
        if self.fused:
            idx, tv = self._fm_forward(B, train=True)
            if after_fm is not None:
                after_fm()
            KN.tower(self._tower_args(B, train=True))
            if not defer_wgrad:
                self._dense_grads()
            return idx, tv
        idx, tv = self._forward(B, train=True)
        if after_fm is not None:
            after_fm()
        self._head(B, train=True)
        self._mlp_backward(B)
        return idx, tv

    def _reset_sync(self):
        """In-launch hand-off flags carry the step index as their tag: a step counter moved
        backwards (checkpoint restore) must not meet flags of its future."""
        if hasattr(self, "sf_flags"):
            self.sf_flags.zero_()
        if hasattr(self, "sfwg_done"):
            self.sfwg_done.zero_()
        if getattr(self, "shx", None) is not None:
            self.shx.reset_table()
        if getattr(self, "rpx", None) is not None:
            self.rpx.reset_table()
        if getattr(self, "tf1_split", False):
            self.sw_step.copy_(self.step)
            self._sw_done.zero_()

    def refresh_shadows(self):
        """Re-derive the bf16 / fp8 weight copies after parameters changed outside a step (load,
        broadcast); rows served ahead for the next row-sharded step are dropped as well."""
        if getattr(self, "shx", None) is not None:
            self.shx.drop_served()
        KN.shadow_refresh(self.p, self.P, self._shadow_dev, self._nshadow)
        if self.fp8:
            KN.w8_quant(self._w8_jobs, len(self.layers), self._w8_rows)

    # ------------------------------------------------------------------ batch staging
    def stage_batch(self, ids: torch.Tensor, vals: torch.Tensor, labels: Optional[torch.Tensor]):
        """Copy a batch into the static input buffers (device->device when already resident)."""
        self.idx, self.vals, self.labels = self._own_in
        self._idx_fm = False
        B = ids.shape[0]
        M = self._padM(B)
        if M > self._bufs_M:
            self._alloc_step_buffers(M)
        n = B * self.F
        self.idx[:n].copy_(ids.reshape(-1), non_blocking=True)
        self.vals[:n].copy_(vals.reshape(-1), non_blocking=True)
        if n < self.idx.numel():
            self.idx[n:].zero_()
            self.vals[n:].zero_()
        if labels is not None:
            self.labels[:B].copy_(labels.reshape(-1), non_blocking=True)
        return B

    # ------------------------------------------------------------------ forward pieces
    def _fm_inputs(self, B: int, train: bool):
        """(slot -> row index, fm_v rows, fm_w rows) the FM gather reads: the local tables, or the
        rows fetched from their owners (row-sharded)."""
        if self.shx is not None:
            return self.shx.fetch(self._shx_plan, train)
        return self.idx, self.tv, self.tw

    def _fm_forward(self, B: int, train: bool):
        M, F, K = self.M, self.F, self.K
        idx, tv, tw = self._fm_inputs(B, train)
        fm_bias = self.p[self.dense_segs["fm_bias"].off:]
        # the side-stream field sort forked after this launch reads the ids field-major from it
        ib = self._idsT_B if train else 0
        ext = dict(idsT=self._fsort.idsT, Bt=ib) if ib else {}
        if self.fp8:
            KN.fm_fwd(idx, self.vals, tv, tw, fm_bias, M, F, K, self.K0p, self.y_fm, self.S, None,
                      self.Et if train else None, E8=self.E8, sE=self.sE, **ext)
        else:
            KN.fm_fwd(idx, self.vals, tv, tw, fm_bias, M, F, K, self.K0p, self.y_fm, self.S, self.E,
                      self.Et if train else None, **ext)
        return idx, tv

    def seg_args(self, n: int, compact: bool, vsrc=None, vsrc_compact: bool = False) -> SegApplyArgs:
        A = SegApplyArgs()
        A.sorted_keys = self.sorted_keys.data_ptr()
        A.ukeys = self.ukeys.data_ptr()
        A.seg_start = self.seg_start.data_ptr()
        A.num = self.num_u.data_ptr()
        A.n = n
        A.ntiles = KN.seg_tiles(self.K, n)
        A.compact = 1 if compact else 0
        A.row_div = self.row_div
        A.vsrc_compact = 1 if vsrc_compact else 0
        A.vsrc = 0 if vsrc is None else vsrc.data_ptr()
        A.partial = self.G.data_ptr()
        A.cont = self.cont.data_ptr()
        A.UG = self.UG.data_ptr()
        A.tv, A.tw = self.tv.data_ptr(), self.tw.data_ptr()
        A.s0v, A.s1v, A.s0w, A.s1w = (t.data_ptr() if t.numel() else 0 for t in self.sv)
        if self.sparse_update == "tf1_dense" and not self.tf1_split:
            A.Gv, A.Gw = self.Gv.data_ptr(), self.Gw.data_ptr()
        A.h = self.h_sparse
        A.step = self.step.data_ptr()
        A.ldv, A.ldw = KN._ld(self.tv, self.tw)
        return A

    def uses_field_sort(self, B: int) -> bool:
        return (self._fsort is not None and _SORT_MODE != "global" and B <= self._fsort.max_rows)

    def _sort_slots(self, B: int):
        """Stable sort of the B*F slot ids -> (sorted_keys, perm): one per-field LDS launch when
        the field id ranges are known, else the global radix sort."""
        n = B * self.F
        if self.uses_field_sort(B):
            self._fsort(self.idx, B, self.sorted_keys, self.perm, field_major=self._idx_fm)
        else:
            KN.sort_ids(self.idx, self.sorted_keys, None, self.perm, n, self.end_bit, self.temp,
                        limit=self.V, err=self.err_words[3:4])

    def _raise_errors(self, w):
        """Raise on the first set error word of a host copy ``w`` of ``err_words`` (and on a
        poisoned same-device transport, whose error word lives on the host)."""
        eng = getattr(self.comm, "engine", None) if self.comm is not None else None
        if eng is not None and hasattr(eng, "check"):
            eng.check()
        if w[0] or w[1]:
            raise RuntimeError("an id lies outside its field's declared range (field_ranges): "
                               "the per-field sort is invalid for this data")
        if w[3]:
            raise RuntimeError(f"a feature id lies outside [0, feature_size={self.V}) (the step "
                               "clamped it; check the input data)")
        if w[6]:
            raise RuntimeError(f"sparse backward hand-off failed (error bits {w[6]:#x}): a look-back "
                               "timed out or read an inconsistent tile publication")
        if w[2]:
            if getattr(self, "rpx", None) is not None:
                raise RuntimeError(f"replicated exchange: a batch has more than capacity="
                                   f"{self.rpx.C} unique ids (raise the capacity)")
            C = self.shx.C if self.shx is not None else "?"
            raise RuntimeError(f"row-sharded exchange: a rank sent more than capacity={C} "
                               "unique ids to one owner (raise the capacity)")

    def check_errors(self):
        """Raise on device-side errors flagged by earlier steps (one host sync)."""
        self._err_ev = None
        self._raise_errors(self.err_words.tolist())
        temps = [self.temp] + ([rs.temp for rs in self.shx.sets] if self.shx is not None else [])
        if any(KN.sort_error(t) for t in temps):
            raise RuntimeError("the global slot sort's look-back timed out (a tile's predecessor "
                               "never published): the sort order of that step is invalid")

    def poll_errors(self):
        """Asynchronous error check, called after every enqueued step / graph replay: raises on
        the error words copied after an EARLIER call if that copy has landed, then starts a new
        non-blocking copy (one small D2H per call, never a host wait).  A bad step is thus
        reported within a call or two instead of at the next ``log_steps`` sync."""
        if self.device.type != "cuda":
            return
        ev = self._err_ev
        if ev is not None:
            if not ev.query():
                return                   # the previous copy is still in flight: keep it
            self._raise_errors(self._err_host.tolist())
        self._err_host.copy_(self.err_words, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._err_ev = ev

    def sf_args(self, n: int) -> SfArgs:
        A = SfArgs()
        A.sorted_keys, A.perm = self.sorted_keys.data_ptr(), self.perm.data_ptr()
        A.vals, A.dlogit = self.vals.data_ptr(), self.dlogit.data_ptr()
        A.dX0, A.S = self.dX0.data_ptr(), self.S.data_ptr()
        A.n, A.F, A.KP, A.row_div = n, self.F, self.K0p, self.row_div
        A.ctail, A.lead, A.tinfo = self.sf_ctail.data_ptr(), self.sf_lead.data_ptr(), self.sf_tinfo.data_ptr()
        A.tv, A.tw = self.tv.data_ptr(), self.tw.data_ptr()
        A.s0v, A.s1v, A.s0w, A.s1w = (t.data_ptr() if t.numel() else 0 for t in self.sv)
        if self.sparse_update == "tf1_dense" and not self.tf1_split:
            A.Gv, A.Gw = self.Gv.data_ptr(), self.Gw.data_ptr()
        A.h = self.h_sparse
        A.step = self.step.data_ptr()
        A.ldv, A.ldw = KN._ld(self.tv, self.tw)
        A.step_off = 0 if (self._sp.dense_early and not self._sp.sfwg) else 1
        A.flags, A.sync = self.sf_flags.data_ptr(), self.sf_sync.data_ptr()
        A.vbf16 = 1 if self.emb_bf16 else 0
        A.grow = self.grow.data_ptr() if self._sp.grow_rows else 0
        A.grow_perm = 0 if self.grow_sorted else 1
        return A

    def _sparse_backward(self, B: int, idx, tv, presorted: bool = False):
        """Embedding backward.  Single rank: the row update is fused into the reduction
        (returns None).  Multi-rank: returns compact unique-row gradients for the exchange."""
        n = B * self.F
        if self.shx is not None:
            self.shx.backward(self._shx_plan, B,
                              dense=self._sh_dense_args() if self._sp.sh_apply_dense else None,
                              join=self._sh_join,
                              wgfin=self._wgfin_args(False) if self._sp.xfuse else None,
                              dense_ar=self.g if self._sp.exchange_allreduce else None,
                              overlap=self._dense_grads if self._sp.overlap_dense else None)
            return None
        if not presorted:
            self._sort_slots(B)
        if self.rpx is not None:
            self.rpx.backward(B, dense=self._sh_dense_args() if self._sp.sh_apply_dense else None,
                              join=self._sh_join,
                              wgfin=self._wgfin_args(False) if self._sp.xfuse else None,
                              dense_ar=self.g if self._sp.exchange_allreduce else None,
                              overlap=self._dense_grads if self._sp.overlap_dense else None)
            return None
        if self._sp.sfwg:
            KN.sparse_wgfin(self.K, self.opt_id, self.sf_args(n), self._wgfin_args(True), self.sfwg_done,
                            sweep=self._sweep_args() if self._sp.tf1_merged else None)
            return None
        if not self.exchange and _SPARSE_IMPL == "fused":
            KN.sparse_fused(self.K, KN.SF_LAZY if self.lazy_rows else KN.SF_SCATTER,
                            self.opt_id, self.sf_args(n))
            if not self.lazy_rows:
                KN.dense_sweep(self.K, self.opt_id, self.R, self.tv, self.tw, self.Gv, self.Gw,
                               self.sv, self.h_sparse, self.step)
            return None
        if not self.exchange:
            self._segment_reduce(n, compact=False)
            A = self.seg_args(n, compact=False)
            if self.lazy_rows:
                KN.seg_apply(self.K, KN.SEG_LAZY, self.opt_id, A, n)
            else:
                KN.seg_apply(self.K, KN.SEG_SCATTER, 0, A, n)
                KN.dense_sweep(self.K, self.opt_id, self.R, self.tv, self.tw, self.Gv, self.Gw,
                               self.sv, self.h_sparse, self.step)
            return None
        raise RuntimeError("multi-rank step without its native exchange")

    def _segment_reduce(self, n: int, compact: bool):
        """Per-slot gradients + per-tile run sums (K2+K3).  compact: partials indexed by the
        unique index (needs the segment structure), else by head position."""
        sid = None
        if compact:
            KN.segments(self.sorted_keys, n, self.seg_flags, self.sid_incl, self.ukeys,
                        self.seg_start, self.num_u, self.temp)
            sid = self.sid_incl
        KN.fm_bwd_seg(self.K, self.sorted_keys, self.perm, sid, self.vals, self.dlogit, self.dX0,
                      self.S, n, self.F, self.K0p, self.G, self.cont)

    # ------------------------------------------------------------------ public step API
    _knobs = staticmethod(step_knobs)

    def _mode_spec(self) -> ModeSpec:
        return ModeSpec(K=self.K, fused=self.fused, gather_fused=self.gather_fused, sharded=self.sharded,
                        exchange=self.exchange, native_exchange=(self.shx is not None or self.rpx is not None),
                        row_sharded=self.shx is not None, lazy_rows=self.lazy_rows,
                        lazy=self.sparse_update == "lazy", tf1_split=self.tf1_split, fp8=self.fp8,
                        tf1x=getattr(self, "tf1_xsplit", False),
                        wgfin_fits=getattr(self, "_wgfin_ns", 1 << 30) <= KN.SFWG_MAX_NS,
                        fin_covers_all=self._fin_covers_all, grow_ok=self.grow is not None)

    def step_plan(self, B: int) -> StepPlan:
        """The plan (models/step_plan.py) of the step bound by ``_bind_step`` at batch size B."""
        fs = self.uses_field_sort(B)
        return plan_step(self._mode_spec(), step_knobs(), B, self._sort_plan, self._tf1_plan is not None,
                         field_sort=fs, idst_capable=fs and KN.fm_fwd_writes_idsT(self.F, self.K),
                         routed_run=self._shx_plan is not None and self._shx_plan.run)

    # the last step's plan, observable by tests (which dense-optimizer / sweep path ran)
    _tf1_merged = property(lambda self: self._last_plan.tf1_merged)
    _fin_opt_step = property(lambda self: self._last_plan.fuse_opt)
    _sfwg_step = property(lambda self: self._last_plan.sfwg)

    def train_step_enqueue(self, B: int):
        """Enqueue one full training step on the current stream (no host sync), following its
        plan (models/step_plan.py).  Graph branches launch in capture order, so every forked
        branch is enqueued right after the tower: the step's first kernel starts at once."""
        sp = self.step_plan(B)
        main = torch.cuda.current_stream(self.device)
        if sp.grow_rows and self.shx is not None:           # run-routed: the set's inverse perm
            self._grow_inv = self.shx.run_sets[self._shx_plan.c].inv
        if self.shx is not None:
            self._shx_start(B)
        hooks = []          # called once the tower (or FM forward) is enqueued
        plan = self._sort_plan
        if sp.run_sorted:                                   # sorted at the start of the run
            self.sorted_keys, self.perm, self._grow_inv = self._run_ss[plan[3]]
            if self._tf1_plan is not None:
                flags = self._row_flags[self._tf1_plan[0]]
                if sp.tower_stamp:      # stamped by extra workgroups of this step's tower launch
                    self._tower_stamp = (self.sorted_keys, B * self.F, flags)
                else:
                    KN.stamp_rows(self.sorted_keys, B * self.F, self.row_div, flags, 1)
        else:
            self.sorted_keys, self.perm = self._ss[plan[0] if plan is not None else self._ss_cur]
        if sp.prefetch_next:
            # the next batch's sort: a ROOT branch of the step's graph (no dependency on this
            # step's kernels), enqueued after the tower; it overlaps the whole step and is joined
            # only at its end (enqueue point sweep: after the tower 0.1318, after the dense
            # gradients 0.1316, at the end 0.1351, at the start 0.1365 ms/step)
            if self._side_next is None:
                self._side_next = torch.cuda.Stream(self.device)
            self._side_next.wait_stream(main)
            nk_ids, nk_B, nk_fm = self._next_sort_ids, plan[2][1], self._next_fm
            nxt_keys, nxt_perm = self._ss[1 - plan[0]]
            tf1_next = self._row_flags[1 - plan[0]] if self.tf1_split else None

            def sort_next():
                with torch.cuda.stream(self._side_next):
                    self._fsort_next(nk_ids, nk_B, nxt_keys, nxt_perm, field_major=nk_fm)
                    if tf1_next is not None:
                        KN.stamp_rows(nxt_keys, nk_B * self.F, self.row_div, tf1_next, 1)
            hooks = [sort_next]
        if sp.tf1_branch and sp.presorted and not sp.fork_sort:
            # prefetched sort: the sweep is a root branch like the next batch's sort (forked after
            # the tower instead, the graph ran every kernel serially: 0.227 vs 0.160 ms)
            self._sweep_src().wait_stream(main)
            cset = self._tf1_plan[0]
            hooks.append(lambda: self._fork_sweep(None, cset))
        if sp.fork_sort:
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            self._idsT_B = B if sp.sort_idst else 0
            tfp = self._tf1_plan

            def fork_sort():
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    if tfp is not None and tfp[2]:
                        # flags a discarded prefetch set from the keys still in this set
                        KN.stamp_rows(self.sorted_keys, tfp[2], self.row_div, self._row_flags[tfp[0]], 0)
                    if sp.sort_idst:
                        self._fsort.sort_pre(B, self.sorted_keys, self.perm)
                    else:
                        self._sort_slots(B)
                    if tfp is not None:
                        KN.stamp_rows(self.sorted_keys, B * self.F, self.row_div, self._row_flags[tfp[0]], 1)
                if sp.tf1_branch:
                    self._fork_sweep(self._side, tfp[0])
            # (forking after the tower rather than before it: 0.160 -> 0.154 ms/step)
            hooks.insert(0, fork_sort)
        self._sp = sp
        try:
            idx, tv = self._dense_fwd_bwd(B, defer_wgrad=sp.defer_wgrad,
                                          after_fm=(lambda: [h() for h in hooks]) if hooks else None)
        finally:
            self._idsT_B = 0
        if sp.w8_after_fin:
            KN.w8_quant(self._w8_jobs, len(self.layers), self._w8_rows)
        elif sp.dense_early and not sp.fuse_opt:
            self._dense_opt()
        if sp.join_sort:
            main.wait_stream(self._side)
        if sp.dense_branch:
            # weight gradients beside the sparse backward
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(self.device)
            self._comm_stream.wait_stream(main)
            with torch.cuda.stream(self._comm_stream):
                self._dense_grads()
        # native exchange: the dense gradient's producer is joined right before the gradient
        # exchange group (parallel/sharded.py: one communicator, fixed order)
        cs = self._comm_stream if sp.dense_branch else None
        self._sh_join = (lambda: main.wait_stream(cs)) if cs is not None else None
        try:
            self._sparse_backward(B, idx, tv, presorted=sp.presorted)
        finally:
            self._sp, self._last_plan = IDLE, sp
            self._sh_join = None
        if sp.dense_branch:
            main.wait_stream(self._comm_stream)
        if self.shx is not None:
            self.shx.end(self._shx_plan)
        if sp.w8_after_owner:
            KN.w8_quant(self._w8_jobs, len(self.layers), self._w8_rows)
        elif sp.dense_opt_after:
            self._dense_opt()
        if sp.tf1_branch:
            main.wait_stream(self._sweep_stream)
        if sp.prefetch_next:
            # joined at the end of the step: deferring the join to the next step's sparse
            # backward measured 0.155-0.186 vs 0.121 ms/step (the branch lands in the towers' path)
            main.wait_stream(self._side_next)

    def _sweep_args(self):
        from ..ops._lib import SweepArgs
        S = SweepArgs()
        S.rec, S.flags = self.rec.data_ptr(), self._row_flags[self._tf1_plan[0]].data_ptr()
        S.sw_step, S.R, S.ld, S.nblk = self.sw_step.data_ptr(), self.R, self.rec.shape[1], _SWEEP_MBLK
        return S

    def sweep_fields(self, S):
        """tf1_dense split form under the exchange: the owner launch's sweep workgroups (ShApplyArgs)."""
        S.rec, S.rflag = self.rec.data_ptr(), self._xflags.data_ptr()
        S.R, S.rec_ld, S.sweep_blocks = self.R, self.rec.shape[1], _SWEEP_MBLK

    def _sweep_src(self):
        if self._sweep_stream is None:
            # (a low-priority stream measured no better: 0.170 vs 0.160 ms)
            self._sweep_stream = torch.cuda.Stream(self.device)
        return self._sweep_stream

    def _fork_sweep(self, src, c: int):
        """tf1_dense split form: the l2-only update of every row outside this step's batch, on its
        own graph branch (forked from ``src`` once set c's flags are written; joined at the end)."""
        if src is not None:
            self._sweep_src().wait_stream(src)
        with torch.cuda.stream(self._sweep_stream):
            KN.tf1_sweep(self.K, self.opt_id, self.rec, self._row_flags[c], self.h_sparse,
                         self.sw_step, self._sw_done, max_wg=_SWEEP_WG)

    def _sh_dense_args(self):
        from ..ops._lib import ShDenseArgs
        d = ShDenseArgs()
        d.p, d.g = self.p.data_ptr(), self.g.data_ptr()
        d.s0 = self.sd[0].data_ptr() if self.sd[0].numel() else 0
        d.s1 = self.sd[1].data_ptr() if self.sd[1].numel() else 0
        d.n, d.h = self.P, self.h_dense
        d.segs, d.nseg = self._shadow_dev.data_ptr(), self._nshadow
        d.blocks = max(1, min(1024, (self.P + 255) // 256))
        d.done = self._done_ctr.data_ptr()
        return d

    def _dense_opt(self):
        """Dense optimizer over the flat buffer (+ bf16 / fp8 weight shadows); advances the step."""
        KN.dense_opt(self.opt_id, self.p, self.g, self.sd[0], self.sd[1], self.P, self.h_dense,
                     self.step, self._shadow_opt, self._nshadow, done_ctr=self._done_ctr)
        if self._shadow_t is not None:
            KN.shadow_transpose(*self._shadow_t)
        if self.fp8:
            KN.w8_quant(self._w8_jobs, len(self.layers), self._w8_rows)

    def _shx_start(self, B: int):
        """Row-sharded step start: routing plan (inline unless prefetched by the previous step)
        and the fork of the next batch's routing."""
        if self._shx_plan is None:
            self._shx_plan = self.shx.plan(self.idx, B, None, resident=False)
        self.shx.begin(self._shx_plan, B, fork="start")

    def compute_grads(self, ids, vals, labels):
        """Forward + backward WITHOUT any update (tests / debugging): returns the flat dense
        gradient and the compact unique-row embedding gradients (ukeys, UG, U)."""
        if self.sharded:
            raise NotImplementedError("compute_grads is single-rank / replicated only")
        B = self.stage_batch(ids, vals, labels)
        self._dense_fwd_bwd(B)
        n = B * self.F
        self._sort_slots(B)
        self._segment_reduce(n, compact=True)
        KN.seg_apply(self.K, KN.SEG_WRITE_UG, 0, self.seg_args(n, compact=True), n)
        U = int(self.num_u.item())
        return self.g.clone(), self.ukeys[:U].clone(), self.UG[:U].clone()

    def loss_value(self, B: int, include_l2: bool = False) -> float:
        """Mean data loss of the last step (+ l2 terms over the whole tables if asked)."""
        v = float(self.loss_sum.item()) / B
        self.check_errors()
        if include_l2:
            v += self.l2_value()
        return v

    def l2_value(self) -> float:
        s = KN.sumsq(self.tv) + KN.sumsq(self.tw)
        if self.comm is not None and self.sharded and self.world > 1:
            s = self.comm.allreduce_scalar(s)
        return float(self.l2 * 0.5 * s)

    @property
    def forward_collective(self) -> bool:
        """Forward passes (evaluate / predict) issue collectives (the row-sharded table's id and
        row all-to-alls): every rank has to join each one, batch for batch."""
        return self.shx is not None and self.world > 1

    def predict_enqueue(self, B: int, with_labels: bool = False):
        if self.shx is not None:           # row-sharded: route this batch inline, then fetch
            # evaluation / predict batches go through the full-capacity exchange when the training
            # one was calibrated on the training epoch (an eval batch may have more unique ids)
            train_x = self.shx
            x = self._shx_eval if getattr(self, "_shx_eval", None) is not None else train_x
            self.shx = x
            try:
                self._shx_plan = x.plan(self.idx, B, None, resident=False)
                x.begin(self._shx_plan, B)
                self._predict_body(B, with_labels)
                x.commit(self._shx_plan, self.idx, B, resident=False)
                x.invalidate()        # (it used a set a prefetched batch may have been in)
            finally:
                self.shx = train_x
                self._shx_plan = None
            if x is not train_x:
                train_x.invalidate()
            return
        self._predict_body(B, with_labels)

    def join_forward(self):
        """A rank without a batch left joins the other ranks' forward collectives with a dummy
        one-row batch whose outputs nobody reads (distributed evaluation / predict over shards of
        unequal length)."""
        d = getattr(self, "_dummy_in", None)
        if d is None or d[2] != self.field_ranges:
            # one valid id per field: the first id of its declared range (the per-field sort
            # flags an id outside it)
            lo = [r[0] for r in self.field_ranges] if self.field_ranges is not None else [0] * self.F
            d = (torch.tensor([lo], dtype=torch.int32, device=self.device),
                 torch.zeros(1, self.F, dtype=torch.float32, device=self.device), self.field_ranges)
            self._dummy_in = d
        B = self.stage_batch(d[0], d[1], None)
        self.predict_enqueue(B, with_labels=False)

    def _predict_body(self, B: int, with_labels: bool):
        if self.fused and self.gather_fused:
            g = self._fm_inputs(B, train=False)
            KN.tower(self._tower_args(B, train=False, with_labels=with_labels, gather=g), KE=self.K)
            return
        if self.fused:
            self._fm_forward(B, train=False)
            KN.tower(self._tower_args(B, train=False, with_labels=with_labels))
            return
        self._forward(B, train=False)
        self._head(B, train=False, with_labels=with_labels)

    def predict(self, ids, vals) -> torch.Tensor:
        B = self.stage_batch(ids, vals, None)
        self.predict_enqueue(B, with_labels=False)
        return self.prob[:B].clone()

    def eval_batch(self, ids, vals, labels, hist: torch.Tensor):
        """Forward + accumulate the 200-threshold AUC histogram and the loss sum."""
        B = self.stage_batch(ids, vals, labels)
        self.predict_enqueue(B, with_labels=True)
        KN.auc_hist(self.prob, self.labels, B, hist)
        self.eval_loss_sum = self.partial[:, -1].sum()     # sum of per-sample data loss (device)
        return B
