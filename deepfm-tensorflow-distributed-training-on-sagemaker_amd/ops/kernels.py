"""Thin typed wrappers over the kernel library (one function per C entry point).

All wrappers launch on torch's current HIP stream and never synchronize, so sequences of
them can be captured into a HIP graph (``torch.cuda.CUDAGraph``).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import torch

from . import _lib
from ._lib import (BnArgs, EpiArgs, HeadArgs, TowerArgs, W8Job, WgJob, OptHyper, RowSumJob, SegApplyArgs, SfArgs, ShApplyArgs, ShadowSeg, SlabJob, check,
                   ptr, stream_handle)

EPI_F32, EPI_FWD, EPI_DGRAD, EPI_FWD_EVAL, EPI_RELU_F32 = 0, 1, 2, 3, 4
OPT_IDS = {"Adam": 0, "Adagrad": 1, "Momentum": 2, "ftrl": 3, "GD": 4}

# tile ids of hfm_gemm_nt: (rows per block, cols per block)
TILES = {0: (64, 64), 1: (128, 32), 2: (32, 128), 3: (32, 32), 4: (32, 64), 5: (32, 160),
         6: (32, 320), 7: (32, 256), 8: (128, 128), 9: (256, 256), 10: (256, 256), 11: (256, 256),
         12: (256, 256), 13: (256, 256)}
TILE_LDS = 8          # 128 x 128 LDS-staged workgroup tile (mlp.hip gemm_lds_kernel): k-chunks of 64
TILE_PP = 10          # 256 x 256 ping-pong tile, spread LDS-DMA staging (mlp.hip gemm_pp_kernel<., 1>)


def L():
    return _lib.get_lib()


def _ld(tv, tw):
    """Row strides (in floats) of a v table [R, K] and a w table [R] (plain or record views; a
    bf16 v table -- mixed-precision embeddings -- is a view of the fp32 record)."""
    ldv = tv.stride(0) if tv.dim() == 2 else tv.shape[-1]
    ldv = ldv * tv.element_size() // 4
    ldw = tw.stride(0) if tw.dim() == 1 else 1
    return ldv, ldw


def _bf(t) -> int:
    return 1 if t.dtype == torch.bfloat16 else 0


def fm_fwd(idx, vals, tv, tw, bias, B, F, K, KP, y_fm, S, E, Et, E8=None, sE=None, idsT=None,
           Bt=0):
    """FM forward (y_fm, S) + the MLP input: E (bf16 [B, KP]) and/or E8 (OCP fp8 e4m3 rows,
    per-row dequant factors sE) for the fp8 tower; Et (bf16 [KP, B]) for the weight gradient.
    ``idsT`` (int32 [F * Bt], optional): the first Bt samples' ids written field-major for
    ``FieldSort.sort_pre`` (row-tile variant only, see ``fm_fwd_writes_idsT``)."""
    assert tv.stride(-1) == 1
    if E8 is not None:
        assert E8.dtype == torch.uint8 and E8.is_contiguous() and sE is not None
    if idsT is not None:
        assert fm_fwd_writes_idsT(F, K) and 0 < Bt <= B and idsT.numel() >= F * Bt
    check(L().hfm_fm_fwd(ptr(idx), ptr(vals), ptr(tv), ptr(tw), ptr(bias), B, F, K, KP, ptr(y_fm),
                         ptr(S), ptr(E), ptr(Et), ptr(E8), ptr(sE), *_ld(tv, tw), ptr(idsT), int(Bt),
                         stream_handle()),
          "fm_fwd")


def fm_fwd_writes_idsT(F: int, K: int) -> bool:
    """Whether fm_fwd takes the row-tile variant (csrc/kernels/fm.hip launch_fm_fwd), the one
    that can also write the field-major id copy."""
    sb = 256 // K
    return (sb * (F * K + 1) + 2 * sb * F + sb) * 4 <= 120 * 1024


def fm_bwd_sorted(perm, idx, vals, tv, dlogit, dX0, S, n, F, K, KP, G):
    check(L().hfm_fm_bwd_sorted(ptr(perm), ptr(idx), ptr(vals), ptr(tv), ptr(dlogit), ptr(dX0),
                                ptr(S), n, F, K, KP, ptr(G), stream_handle()), "fm_bwd_sorted")


def grad_row_floats(K: int) -> int:
    return K + 4


def sort_temp_bytes(n: int, end_bit: int) -> int:
    b = C.c_size_t(0)
    check(L().hfm_sort_pairs_temp_bytes(n, end_bit, C.byref(b)), "sort_temp")
    return b.value


def rbk_temp_bytes(K: int, n: int) -> int:
    b = C.c_size_t(0)
    check(L().hfm_reduce_by_key_temp_bytes(K, n, C.byref(b)), "rbk_temp")
    return b.value


def scan_temp_bytes(n: int) -> int:
    b = C.c_size_t(0)
    check(L().hfm_scan_temp_bytes(n, C.byref(b)), "scan_temp")
    return b.value


def radix_temp_bytes(n: int) -> int:
    """Workspace bytes for ``sort_ids`` (covers both sort implementations)."""
    b = C.c_size_t(0)
    check(L().hfm_radix_sort_temp_bytes(n, C.byref(b)), "radix_temp")
    b2 = C.c_size_t(0)
    check(L().hfm_onesweep_temp_bytes(n, C.byref(b2)), "onesweep_temp")
    return max(b.value, b2.value)


def cub_sort_ids(keys_in, keys_out, vals_tmp, perm_out, n, end_bit, temp):
    """hipCUB SortPairs (reference implementation for tests / A-B timing)."""
    check(L().hfm_sort_ids(ptr(keys_in), ptr(keys_out), ptr(vals_tmp), ptr(perm_out), n, end_bit,
                           ptr(temp), temp.numel(), stream_handle()), "cub_sort_ids")


def lsd_sort_ids(keys_in, keys_out, perm_out, n, end_bit, temp):
    """Classic 3-kernel-per-pass LSD radix sort (A/B reference for the onesweep sort)."""
    check(L().hfm_radix_sort_ids(ptr(keys_in), ptr(keys_out), ptr(perm_out), n, end_bit, ptr(temp),
                                 temp.numel(), stream_handle()), "radix_sort_ids")


def onesweep_sort_ids(keys_in, keys_out, perm_out, n, end_bit, temp, limit: int = 0, err=None):
    """Onesweep radix sort (global histogram + one decoupled-look-back pass per 8 bits).
    ``limit`` > 0 (the table's rows): keys outside [0, limit) are sorted as limit - 1 and set the
    int32 word ``err``, so a bad id never indexes a table out of bounds downstream."""
    assert limit == 0 or err is not None
    check(L().hfm_onesweep_sort_ids(ptr(keys_in), ptr(keys_out), ptr(perm_out), n, end_bit,
                                    ptr(temp), temp.numel(), int(limit), ptr(err), stream_handle()),
          "onesweep_sort_ids")


def sort_ids(keys_in, keys_out, vals_tmp, perm_out, n, end_bit, temp, limit: int = 0, err=None):
    """Stable sort of slot ids -> (sorted keys, slot permutation) (csrc/kernels/radix_sort.hip):
    the onesweep sort (A/B in tools/bench_sort.py, graph-timed: onesweep 56 us vs the LSD sort
    101 us at n = 640K, 30 bits; ``lsd_sort_ids`` stays for that tool).  ``temp`` must hold
    radix_temp_bytes(n) bytes; ``vals_tmp`` is unused.  ``limit`` / ``err``: id-range guard of
    the onesweep sort (see ``onesweep_sort_ids``)."""
    onesweep_sort_ids(keys_in, keys_out, perm_out, n, end_bit, temp, limit, err)


def fs2_chunk_rows() -> int:
    """Rows per chunk of the run-level sort (fsort_run.h FS2_MAXB)."""
    return int(L().hfm_fs2_chunk_rows())


def field_sort_max_rows() -> int:
    """Largest batch the per-field LDS sort handles (csrc/kernels/field_sort.hip): row chunks of
    ``field_sort_chunk_rows()`` are sorted per workgroup, then merged."""
    return int(L().hfm_field_sort_max_rows())


def field_sort_chunk_rows() -> int:
    return int(L().hfm_field_sort_chunk_rows())


class FieldSort:
    """Per-field MSD-partitioned LDS sort of the B*F slot ids (csrc/kernels/field_sort.hip) for
    disjoint, increasing per-field id ranges [lo, hi): output identical to ``sort_ids`` on the
    same slots.  ``err`` (int32 [1]) turns non-zero when an id lies outside its field's range.
    Batches above ``field_sort_chunk_rows()`` are sorted in row chunks and merged (the work list
    is built for ``max_rows``; a smaller batch skips the workgroups of chunks it does not have)."""

    def __init__(self, ranges, max_rows: int, device, max_pb: int = 0, err=None):
        """``max_pb``: each field is split into up to 2^max_pb workgroups (MSD partitions): 4 when
        the sort is on the critical path, 0 (one workgroup per field) when it overlaps other work."""
        import math
        max_pb = min(int(max_pb), int(L().hfm_field_sort_max_pb()))
        assert max_rows <= field_sort_max_rows()
        self.chunk = field_sort_chunk_rows()
        fr, self._fwork = [], []
        for f, (lo, hi) in enumerate(ranges):
            bits = int(math.ceil(math.log2(hi - lo))) if hi - lo > 1 else 0
            pb = min(bits, max_pb)
            fr.append((int(lo), int(hi), bits, pb))
            self._fwork.append(1 << pb)
        self.F = len(fr)
        self.fr = torch.tensor(fr, dtype=torch.int32).reshape(-1).to(device)
        self.device = device
        self._work = {}
        for b in range(1, max(1, max_rows) + 1, self.chunk):    # all built now, never during capture
            self.work(b)
        self.idsT = torch.zeros(self.F * max(1, max_rows), dtype=torch.int32, device=device)
        big = max_rows > self.chunk
        self.rk = torch.zeros(self.F * max_rows if big else 1, dtype=torch.int32, device=device)
        self.rp = torch.zeros_like(self.rk)
        # error word: a caller's (e.g. a view of the model's error words) or its own
        self.err = err if err is not None else torch.zeros(1, dtype=torch.int32, device=device)
        self.max_rows = max_rows

    def work(self, B: int):
        """(work list on the device, its length) for a batch of B rows: {field, partition, chunk}."""
        nc = max(1, -(-B // self.chunk))
        w = self._work.get(nc)
        if w is None:                                    # (only from __init__)
            items = [(f, p, c) for f, n in enumerate(self._fwork) for c in range(nc) for p in range(n)]
            w = (torch.tensor(items, dtype=torch.int32).reshape(-1).to(self.device), len(items))
            self._work[nc] = w
        return w

    def __call__(self, ids, B: int, keys_out, perm_out, field_major: bool = False):
        """``ids``: row-major [B, F] slots (transposed first), or with ``field_major`` the [F, B]
        layout the sort reads (no transpose launch)."""
        assert B <= self.max_rows and ids.numel() >= B * self.F
        if field_major:
            return self._sort(ids, B, keys_out, perm_out)
        work, nwork = self.work(B)
        check(L().hfm_field_sort(ptr(ids), B, self.F, ptr(self.fr), ptr(work), nwork,
                                 ptr(self.idsT), ptr(self.rk), ptr(self.rp), ptr(keys_out), ptr(perm_out),
                                 ptr(self.err), stream_handle()), "field_sort")

    def run_plan(self, batches):
        """Device plan of the run-level sort (fsort_run.h) of ``batches`` = [(ids, B, field_major,
        keys_out, perm_out)]: one FsJob per batch (own chunk-run scratch), the sort items (batch,
        field, 16K-row chunk; big fields first) and the merge items (B > 16K only).  Built on the host before any
        capture and cached under the buffers' addresses."""
        batches = [tuple(b) + (None,) * (6 - len(b)) for b in batches]      # (..., inv_out or None)
        key = tuple((ptr(i), int(B), bool(fm), ptr(k), ptr(p), ptr(v)) for i, B, fm, k, p, v in batches)
        cache = self.__dict__.setdefault("_run_plans", {})
        hit = cache.get(key)
        if hit is not None:
            return hit
        ch, wpr = fs2_chunk_rows(), int(L().hfm_fs2_merge_wgs_per_run())
        fr = self.fr.view(-1, 4).cpu()
        G = len(batches)
        n = self.F * self.max_rows
        rs = self.__dict__.get("_run_scratch")
        if rs is None or rs.shape[0] < G:
            # a larger run: new scratch for plans built from now on.  Cached plans are NOT dropped:
            # graphs captured from them still read their FsJob arrays and scratch (each plan
            # holds its own in ``keep``), and freeing those let a replay fault on reused memory
            rs = torch.zeros(G, 2, n, dtype=torch.int32, device=self.device)
            self._run_scratch = rs
        jobs, items, mitems, keep = [], [], [], [rs]
        for g, (ids, B, fm, kout, pout, iout) in enumerate(batches):
            assert B <= min(self.max_rows, 8 * ch) and ids.numel() >= B * self.F
            nc = max(1, -(-B // ch))
            wl = [(f, c) for f in range(self.F) for c in range(nc)]
            wl.sort(key=lambda t: -int(fr[t[0], 2]))                 # big fields first
            mf = [f for f in range(self.F) if int(fr[f, 2]) > 0] if nc > 1 else []
            work = torch.tensor(wl, dtype=torch.int32).reshape(-1).to(self.device)
            mft = torch.tensor(mf or [0], dtype=torch.int32).to(self.device)
            keep += [work, mft]
            j = _lib.FsJob()
            j.ids, j.ld = ptr(ids), (B if fm else 0)                    # field-major: [F, B]
            j.B, j.F, j.fr, j.work, j.nwork = B, self.F, ptr(self.fr), ptr(work), len(wl)
            j.rk, j.rp = ptr(rs[g, 0]), ptr(rs[g, 1])
            j.keys, j.perm, j.err = ptr(kout), ptr(pout), ptr(self.err)
            j.inv = ptr(iout)
            j.mfields, j.nmf, j.mwpf = ptr(mft), len(mf), wpr * nc
            jobs.append(j)
            items.append([(g, it) for it in range(len(wl))])
            mitems.append([(g, mw) for mw in range(len(mf) * wpr * nc)])
        # interleave the batches: item k of every batch, then item k + 1 (big fields first overall)
        flat = [t[k] for k in range(max(len(t) for t in items)) for t in items if k < len(t)]
        mflat = [t[k] for k in range(max(len(t) for t in mitems)) for t in mitems if k < len(t)]
        jobs_dev = struct_array_to_device(jobs, self.device)
        it_dev = torch.tensor(flat, dtype=torch.int32).reshape(-1).to(self.device)
        mit_dev = torch.tensor(mflat or [(0, 0)], dtype=torch.int32).reshape(-1).to(self.device)
        plan = (jobs_dev, it_dev, len(flat), mit_dev, len(mflat), keep)
        cache[key] = plan
        return plan

    def run_sort(self, plan):
        """Enqueue the run-level sort of ``run_plan``'s batches (two launches)."""
        jobs_dev, it_dev, nit, mit_dev, nmit, _ = plan
        check(L().hfm_field_sort_run(ptr(jobs_dev), ptr(it_dev), nit, ptr(mit_dev), nmit, stream_handle()),
              "field_sort_run")

    def sort_pre(self, B: int, keys_out, perm_out):
        """The sort alone, from ``self.idsT`` already filled field-major ([F, B]) by fm_fwd."""
        self._sort(self.idsT, B, keys_out, perm_out)

    def _sort(self, idsT, B: int, keys_out, perm_out):
        assert B <= self.max_rows
        work, nwork = self.work(B)
        check(L().hfm_field_sort_pre(ptr(idsT), B, self.F, ptr(self.fr), ptr(work), nwork,
                                     ptr(self.rk), ptr(self.rp), ptr(keys_out), ptr(perm_out),
                                     ptr(self.err), stream_handle()), "field_sort_pre")


def sort_error(temp) -> int:
    """1 if the last onesweep sort in ``temp`` timed out in its look-back (device read: syncs)."""
    off = L().hfm_onesweep_error_offset()
    return int(temp[off: off + 4].view(torch.int32).item())


def reduce_by_key(K, sorted_keys, G, ukeys, UG, num, n, temp):
    check(L().hfm_reduce_by_key(K, ptr(sorted_keys), ptr(G), ptr(ukeys), ptr(UG), ptr(num), n,
                                ptr(temp), temp.numel(), stream_handle()), "reduce_by_key")


def unique_inverse(sorted_keys, perm, n, flags_tmp, seg_tmp, uniq, inverse, num, temp):
    check(L().hfm_unique_inverse(ptr(sorted_keys), ptr(perm), n, ptr(flags_tmp), ptr(seg_tmp),
                                 ptr(uniq), ptr(inverse), ptr(num), ptr(temp), temp.numel(),
                                 stream_handle()), "unique_inverse")


def gather_i32(src, perm, n, out):
    check(L().hfm_gather_i32(ptr(src), ptr(perm), n, ptr(out), stream_handle()), "gather_i32")


def expand_vals(vc, nc: int, mask: int, F: int, rows: int, out):
    """Compact streamed values [rows, nc] (fields of ``mask``) -> ``out`` [rows, F], 1.0 in the
    fields not shipped (data/native_io.py next_into_compact)."""
    assert out.dtype == torch.float32 and out.numel() >= rows * F and vc.numel() >= rows * nc
    check(L().hfm_expand_vals(ptr(vc), nc, mask, F, rows, ptr(out), stream_handle()), "expand_vals")


def seg_tiles(K: int, n: int) -> int:
    return L().hfm_seg_tiles(K, n)


def segments(sorted_keys, n, flags_tmp, sid_incl, ukeys, seg_start, num, temp):
    """Segment structure of a sorted id list: ukeys[U], seg_start[U+1], num=[U] (device)."""
    check(L().hfm_segments(ptr(sorted_keys), n, ptr(flags_tmp), ptr(sid_incl), ptr(ukeys),
                           ptr(seg_start), ptr(num), ptr(temp), temp.numel(), stream_handle()),
          "segments")


def fm_bwd_seg(K, sorted_keys, perm, sid_incl, vals, dlogit, dX0, S, n, F, KP, partial, cont):
    """Per-slot gradients + in-tile run sums.  sid_incl=None -> position-indexed partials."""
    check(L().hfm_fm_bwd_seg(K, ptr(sorted_keys), ptr(perm), ptr(sid_incl), ptr(vals), ptr(dlogit),
                             ptr(dX0), ptr(S), n, F, KP, ptr(partial), ptr(cont), stream_handle()),
          "fm_bwd_seg")


SEG_LAZY, SEG_SCATTER, SEG_WRITE_UG = 0, 1, 2


SF_LAZY, SF_SCATTER, SF_EXCHANGE = 0, 1, 2


def sparse_fused_tiles(K: int, n: int) -> int:
    return int(L().hfm_sparse_fused_tiles(K, n))


def sparse_fused(K, mode, opt, args: SfArgs):
    """Fused embedding backward + row optimizer (lazy) or tf1_dense scatter over sorted slots
    (csrc/kernels/sparse_fused.hip): one tile kernel + one carry kernel."""
    check(L().hfm_sparse_fused(K, mode, opt, C.byref(args), stream_handle()), "sparse_fused")


SFWG_MAX_NS = 4          # sparse_fused.hip SFWG_MAXNS: wgfin splits the merged launch supports


def sparse_wgfin_x(K, args: SfArgs, wf: "WgFinArgs", serve=None):
    """Row-sharded step: gradient rows for the owner exchange + wgfin gradients (no optimizer)
    in one launch (sparse_fused.hip sfwg_x_kernel); ``serve`` (ShServeArgs): the next run step's
    rows served by extra workgroups of the same launch."""
    check(L().hfm_sparse_wgfin_x(K, C.byref(args), C.byref(wf), C.byref(serve) if serve is not None else None,
                                 stream_handle()), "sparse_wgfin_x")


def sparse_wgfin(K, opt, args: SfArgs, wf: "WgFinArgs", done, sweep=None):
    """Lazy sparse backward + the fused tower's wgfin work (weight gradients, split-K combine,
    dense optimizer) in ONE launch (sparse_fused.hip sfwg_kernel); ``done``: int32 [1] arrival
    counter (zero between launches); the launch advances the step counter.  ``sweep``
    (``_lib.SweepArgs``, tf1_dense split form): extra workgroups give every row outside the batch
    its l2-only update."""
    check(L().hfm_sparse_wgfin(K, opt, C.byref(args), C.byref(wf), ptr(done),
                               C.byref(sweep) if sweep is not None else None, stream_handle()),
          "sparse_wgfin")


def seg_apply(K, mode, opt, args: SegApplyArgs, max_groups):
    check(L().hfm_seg_apply(K, mode, opt, C.byref(args), max_groups, stream_handle()), "seg_apply")


def hyper(lr: float, l2: float, b1=0.9, b2=0.999, eps=1e-8, momentum=0.95) -> OptHyper:
    return OptHyper(lr, l2, b1, b2, eps, momentum)


def sparse_rows_update(K, opt, ukeys, UG, num, max_n, row_div, tv, tw, slots, h: OptHyper, step):
    s0v, s1v, s0w, s1w = slots
    check(L().hfm_sparse_rows_update(K, opt, ptr(ukeys), ptr(UG), ptr(num), max_n, row_div, ptr(tv),
                                     ptr(tw), ptr(s0v), ptr(s1v), ptr(s0w), ptr(s1w), C.byref(h),
                                     ptr(step), *_ld(tv, tw), stream_handle()), "sparse_rows_update")


def scatter_rows(K, ukeys, UG, num, max_n, row_div, Gv, Gw):
    check(L().hfm_scatter_rows(K, ptr(ukeys), ptr(UG), ptr(num), max_n, row_div, ptr(Gv), ptr(Gw),
                               stream_handle()), "scatter_rows")


def dense_sweep(K, opt, R, tv, tw, Gv, Gw, slots, h: OptHyper, step):
    s0v, s1v, s0w, s1w = slots
    check(L().hfm_dense_sweep(K, opt, R, ptr(tv), ptr(tw), ptr(Gv), ptr(Gw), ptr(s0v), ptr(s1v),
                              ptr(s0w), ptr(s1w), C.byref(h), ptr(step), *_ld(tv, tw), stream_handle()),
          "dense_sweep")


def stamp_rows(keys, n, row_div, flags, val):
    """flags[key // row_div] = val for the first n (sorted) slot keys (tf1_dense split sweep)."""
    assert keys.dtype == torch.int32 and flags.dtype == torch.uint8 and keys.numel() >= n
    check(L().hfm_stamp_rows(ptr(keys), n, row_div, ptr(flags), val, stream_handle()), "stamp_rows")


def tf1_sweep(K, opt, rec, flags, h: OptHyper, sw_step, done_ctr, max_wg=2048):
    """TF1 dense-Adam (etc.) update with g = l2*w of every record row whose flag is 0; flagged
    rows (this step's batch, updated by the sparse kernel) are skipped and their flag cleared.
    The last workgroup advances ``sw_step`` (the sweep's own int64 step counter)."""
    R, ld = rec.shape
    assert rec.dtype == torch.float32 and rec.is_contiguous() and flags.numel() >= R
    assert sw_step.dtype == torch.int64 and done_ctr.dtype == torch.int32
    check(L().hfm_tf1_sweep(K, opt, R, ptr(rec), ld, ptr(flags), C.byref(h), ptr(sw_step),
                            ptr(done_ctr), max_wg, stream_handle()), "tf1_sweep")


def dense_opt(opt, p, g, s0, s1, n, h: OptHyper, step, segs_dev, nseg, done_ctr=None):
    """Fused dense optimizer + bf16 shadow refresh; with ``done_ctr`` (an int32 device word,
    zero-initialised) the last block also advances ``step`` (no separate step_inc launch)."""
    check(L().hfm_dense_opt(opt, ptr(p), ptr(g), ptr(s0), ptr(s1), n, C.byref(h), ptr(step),
                            ptr(segs_dev), nseg, ptr(done_ctr) if done_ctr is not None else None,
                            stream_handle()), "dense_opt")


def finalize(slab_jobs_dev, nsj, nslab_blocks, row_jobs_dev, nrj, total_rows):
    """Split-K / head-partial reductions and bias row sums in one launch (mlp.hip)."""
    check(L().hfm_finalize(ptr(slab_jobs_dev), nsj, nslab_blocks, ptr(row_jobs_dev), nrj, total_rows,
                           stream_handle()), "finalize")


def finalize_opt(opt, slab_jobs_dev, nsj, nslab_blocks, row_jobs_dev, nrj, total_rows, p, g, s0, s1,
                 n, h: OptHyper, step, segs_dev, nseg, done_ctr):
    """``finalize`` with the dense optimizer fused in (mlp.hip finalize_opt_kernel): every
    element's update is applied by the thread that produces its final gradient, the last block
    advances ``step``.  Only valid when the finalize outputs cover all n parameters."""
    check(L().hfm_finalize_opt(opt, ptr(slab_jobs_dev), nsj, nslab_blocks, ptr(row_jobs_dev), nrj,
                               total_rows, ptr(p), ptr(g), ptr(s0), ptr(s1), n, C.byref(h), ptr(step),
                               ptr(segs_dev), nseg, ptr(done_ctr), stream_handle()), "finalize_opt")


def shadow_transpose(segs_dev, nseg: int, ntiles: int):
    """wt16 = w16^T for the segments in ``segs_dev`` (64 x 64 LDS tiles; optim.hip)."""
    check(L().hfm_shadow_transpose(ptr(segs_dev), int(nseg), int(ntiles), stream_handle()), "shadow_transpose")


def shadow_refresh(p, n, segs_dev, nseg):
    check(L().hfm_shadow_refresh(ptr(p), n, ptr(segs_dev), nseg, stream_handle()), "shadow_refresh")


def step_inc(step):
    check(L().hfm_step_inc(ptr(step), stream_handle()), "step_inc")


def gemm_nt(epi, tile, A, lda, B, ldb, M, N, Kd, splitk, ep: EpiArgs):
    check(L().hfm_gemm_nt(epi, tile, ptr(A), lda, ptr(B), ldb, M, N, Kd, splitk, C.byref(ep),
                          stream_handle()), f"gemm_nt(epi={epi},tile={tile},M={M},N={N},K={Kd})")


def epi_pass(epi, Cf32, M, N, ep: EpiArgs):
    """The forward / dgrad epilogue (EPI_FWD, EPI_FWD_EVAL, EPI_DGRAD) over an fp32 product
    ``Cf32`` [M, N] from a library GEMM: mlp.hip epi_pass_kernel, the same values as the fused
    epilogues of gemm_nt."""
    check(L().hfm_epi_pass(epi, ptr(Cf32), M, N, C.byref(ep), stream_handle()),
          f"epi_pass(epi={epi},M={M},N={N})")


def head(a: HeadArgs):
    check(L().hfm_head(C.byref(a), stream_handle()), "head")


def wgfin(opt: int, a):
    """Weight gradients + split-K combine + bias / head reductions + dense optimizer (opt >= 0)
    or the gradient only (opt = -1) in one launch (tower.hip wgfin_kernel)."""
    check(L().hfm_wgfin(int(opt), C.byref(a), stream_handle()), "wgfin")


def tower_stamp_rows_per_wg() -> int:
    """Sorted keys per row-flag stamping workgroup of the tower launch (tower.hip)."""
    return int(L().hfm_tower_stamp_rows_per_wg())


def tower(a: TowerArgs, KE: int = 0):
    """Fused deep tower: [FM gather (KE = embedding size) +] forward + head (+ dgrad chain when
    a.train) (csrc/kernels/tower.hip)."""
    check(L().hfm_tower(C.byref(a), int(KE), stream_handle()), "tower")


def w8_quant(jobs_dev, njobs: int, total_rows: int):
    """fp8 e4m3 weight shadows with per-output-channel power-of-two scales (tower.hip)."""
    check(L().hfm_w8_quant(ptr(jobs_dev), njobs, total_rows, stream_handle()), "w8_quant")


def wgrad_group(jobs_dev, njobs: int, ntasks: int):
    """All layers' split-K weight-gradient GEMMs in one launch (wave-granular tasks)."""
    check(L().hfm_wgrad_group(ptr(jobs_dev), njobs, ntasks, stream_handle()), "wgrad_group")


BN_FWD_PARTIAL, BN_FWD_FINALIZE, BN_EVAL_FINALIZE, BN_FWD_APPLY = 0, 1, 2, 3
BN_BWD_PARTIAL, BN_BWD_FINALIZE, BN_BWD_APPLY = 4, 5, 6


def bn(phase: int, a: BnArgs):
    """Batch-norm phase (csrc/kernels/bn.hip); M % 64 == 0 and N % 32 == 0 are required."""
    if a.M % 64 or a.N % 32:
        raise ValueError(f"bn: M={a.M} must be a multiple of 64 and N={a.N} of 32")
    check(L().hfm_bn(phase, C.byref(a), stream_handle()), f"bn[{phase}]")


def slab_reduce(jobs_dev, njobs, max_n):
    check(L().hfm_slab_reduce(ptr(jobs_dev), njobs, max_n, stream_handle()), "slab_reduce")


def rowsum(jobs_dev, njobs, total_rows):
    check(L().hfm_rowsum(ptr(jobs_dev), njobs, total_rows, stream_handle()), "rowsum")


def auc_hist(pred, label, n, hist):
    check(L().hfm_auc_hist(ptr(pred), ptr(label), n, ptr(hist), stream_handle()), "auc_hist")


def sumsq(x: torch.Tensor, nblocks: int = 512) -> torch.Tensor:
    if x.dtype == torch.bfloat16 or not x.is_contiguous():   # record views / bf16 rows: row blocks
        tot = torch.zeros((), dtype=torch.float64, device=x.device)
        step = 1 << 22
        for i in range(0, x.shape[0], step):
            tot += sumsq(x[i: i + step].float().contiguous(), nblocks)
        return tot
    out = torch.empty(nblocks, dtype=torch.float64, device=x.device)
    check(L().hfm_sumsq_partials(ptr(x), x.numel(), ptr(out), nblocks, stream_handle()), "sumsq")
    return out.sum()


def struct_array_to_device(structs: Sequence[C.Structure], device) -> torch.Tensor:
    """Pack ctypes structs into a device byte tensor (job tables, shadow segment lists)."""
    if not structs:
        return torch.zeros(16, dtype=torch.uint8, device=device)
    sz = C.sizeof(structs[0])
    buf = (C.c_uint8 * (sz * len(structs)))()
    for i, s in enumerate(structs):
        C.memmove(C.addressof(buf) + i * sz, C.addressof(s), sz)
    host = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
    return host.to(device)


# ------------------------------------------------------------------ Example decode (decode.hip)
def decode_examples(raw, offs, rows: int, F: int, limit: int, ids, vals, labels, err, crc: bool = False):
    """Serialized tf.train.Example records (``raw`` bytes, ``offs`` rows + 1 uint32 offsets) ->
    ids int32 [rows, F], vals f32 [rows, F], labels f32 [rows] on the current stream; ``err``
    int32 [2] = (error bits, smallest bad record index; initialise it to (0, INT32_MAX)).
    ``crc``: every record ends with its 4-byte masked CRC32C (a raw loader with
    ``device_crc``), verified on the GPU (err bit value 4 on a mismatch, the row zeroed)."""
    check(L().hfm_decode_examples(ptr(raw), ptr(offs), int(rows), int(F), int(limit), ptr(ids), ptr(vals),
                                  ptr(labels), ptr(err), 1 if crc else 0, stream_handle()), "decode_examples")


# ------------------------------------------------------------------ RCCL engine (comm.hip)
def comm_unique_id() -> bytes:
    n = int(L().hfm_comm_id_bytes())
    buf = (C.c_char * n)()
    check(L().hfm_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


def comm_init(nranks: int, rank: int, uid: bytes) -> int:
    h = C.c_void_p()
    buf = (C.c_char * len(uid)).from_buffer_copy(uid)
    check(L().hfm_comm_init(C.byref(h), nranks, rank, buf), "comm_init")
    return int(h.value)


def comm_destroy(h: int):
    check(L().hfm_comm_destroy(h), "comm_destroy")


def comm_allreduce_(h: int, t: torch.Tensor):
    assert t.dtype == torch.float32 and t.is_contiguous()
    check(L().hfm_comm_allreduce_f32(h, ptr(t), t.numel(), stream_handle()), "comm_allreduce")


def comm_alltoall(h: int, send: torch.Tensor, recv: torch.Tensor, bytes_per_peer: int):
    assert send.is_contiguous() and recv.is_contiguous()
    check(L().hfm_comm_alltoall(h, ptr(send), ptr(recv), bytes_per_peer, stream_handle()), "comm_alltoall")


def comm_alltoall_allgather(h: int, send, recv, bytes_per_peer: int, gsend, grecv, gbytes_per_rank: int):
    """All-to-all + all-gather as one aggregated RCCL operation (comm.hip)."""
    for t in (send, recv, gsend, grecv):
        assert t.is_contiguous()
    check(L().hfm_comm_alltoall_allgather(h, ptr(send), ptr(recv), bytes_per_peer, ptr(gsend), ptr(grecv),
                                          gbytes_per_rank, stream_handle()), "comm_alltoall_allgather")


def comm_allgather(h: int, send: torch.Tensor, recv: torch.Tensor, bytes_per_rank: int):
    assert send.is_contiguous() and recv.is_contiguous()
    check(L().hfm_comm_allgather(h, ptr(send), ptr(recv), bytes_per_rank, stream_handle()), "comm_allgather")


COMM_A2A, COMM_ALLGATHER, COMM_ALLREDUCE = 0, 1, 2


def comm_group(h: int, ops):
    """Collectives as ONE aggregated RCCL operation on the current stream (comm.hip
    hfm_comm_group).  ``ops``: (kind, send, recv, bytes) with kind COMM_A2A (bytes per peer),
    COMM_ALLGATHER (bytes per rank) or COMM_ALLREDUCE (f32 sum, bytes in total)."""
    from ._lib import CommOp
    arr = (CommOp * max(1, len(ops)))()
    for i, (kind, send, recv, nbytes) in enumerate(ops):
        assert send.is_contiguous() and recv.is_contiguous()
        arr[i].kind, arr[i].send, arr[i].recv, arr[i].bytes = int(kind), ptr(send), ptr(recv), int(nbytes)
    check(L().hfm_comm_group(h, arr, len(ops), stream_handle()), "comm_group")


# ------------------------------------------------------------------ row-sharded exchange (shard.hip)
def sh_count_blocks(nmax: int) -> int:
    return int(L().hfm_sh_count_blocks(nmax))


def sh_bucket(ukeys, num_u, nmax, N, Cap, cnt_tmp, send_ids, upos, send_cnt, err):
    check(L().hfm_sh_bucket(ptr(ukeys), ptr(num_u), nmax, N, Cap, ptr(cnt_tmp), ptr(send_ids), ptr(upos),
                            ptr(send_cnt), ptr(err), stream_handle()), "sh_bucket")


def sh_route_tiles(n: int) -> int:
    return int(L().hfm_sh_route_tiles(n))


def sh_route(sorted_keys, n, N, Cap, tcnt, sid_incl, send_ids, upos, send_cnt, num_u, err):
    """Sorted slot ids -> 1-based unique index per slot + owner buckets in two launches
    (shard.hip sh_route_*; same outputs as segments + sh_bucket)."""
    check(L().hfm_sh_route(ptr(sorted_keys), n, N, Cap, ptr(tcnt), ptr(sid_incl), ptr(send_ids), ptr(upos),
                           ptr(send_cnt), ptr(num_u), ptr(err), stream_handle()), "sh_route")


def sh_route_run(descs_dev, G: int, n: int, N: int, Cap: int, err, ostride: int, F: int, ld: int = 0,
                 slot_rows: bool = True):
    """Routing of G batches (``descs_dev``: device array of ``_lib.ShRouteBatch``) in three
    launches: owner buckets (owner o's ids at send_ids + o * ostride), unique indices and the slot
    -> row maps of every batch (row-major, or field-major [F][ld] with ``ld``; not with
    ``slot_rows=False``)."""
    check(L().hfm_sh_route_run(ptr(descs_dev), G, n, N, Cap, ostride, F, ld, 1 if slot_rows else 0, ptr(err),
                               stream_handle()),
          "sh_route_run")


def sh_slot_rows(perm, sid_incl, upos, n, idx):
    check(L().hfm_sh_slot_rows(ptr(perm), ptr(sid_incl), ptr(upos), n, ptr(idx), stream_handle()),
          "sh_slot_rows")


_byref = C.byref


def sh_serve(K, recv_ids, total, N, tv, tw, rows, C: int = 0, step=None, table=None, rstride: int = 0,
             ahead: bool = False, rbf16: bool = False, rflag=None):
    """Owner side of the row fetch: rows[e] = {v, w} of every requested id (``rbf16``: compact rows,
    v as bf16 -- shard_table.h sh_row_words; ``rflag``: tf1_dense split form, a byte flag set per
    requested row).  With ``table`` (a
    ShTable; training steps) it also records each request (row, requester, slot) stamped with
    step + 1 in the owner's request table read by sh_owner_apply -- step + 2 with ``ahead`` (the
    NEXT step's rows, served during this step; this step's owner update patches the rows it
    changes).  ``recv_ids``: a tensor or a device address; ``rstride``: its request-row stride
    (0: contiguous [N][C])."""
    rp = recv_ids if isinstance(recv_ids, int) else ptr(recv_ids)
    check(L().hfm_sh_serve(K, rp, total, N, C, rstride, ptr(tv), ptr(tw), *_ld(tv, tw), ptr(rows),
                           ptr(step), _byref(table) if table is not None else None, 2 if ahead else 1,
                           _bf(tv), 1 if rbf16 else 0, ptr(rflag), stream_handle()), "sh_serve")


def sh_apply_dense(K, opt, args: ShApplyArgs, dense):
    """Lazy owner update + dense optimizer in one launch (shard.hip sh_apply_dense_kernel); the
    launch advances the step counter."""
    check(L().hfm_sh_apply_dense(K, opt, C.byref(args), C.byref(dense), stream_handle()), "sh_apply_dense")


def sh_owner_apply(K, opt, args: ShApplyArgs):
    check(L().hfm_sh_owner_apply(K, opt, C.byref(args), stream_handle()), "sh_owner_apply")
