"""ctypes binding of ``_lib/libhipfm_kernels.so`` (the gfx950 HIP kernels, csrc/kernels).

The library is loaded AFTER ``import torch`` so its ``libamdhip64.so.7`` dependency resolves to
the HIP runtime torch already loaded (same SONAME) — device pointers and ``hipStream_t``
handles from torch are then valid in our kernels, and launches on torch's current stream are
captured by ``torch.cuda.CUDAGraph`` like any torch op.

There is no silent fallback: on a GPU run, a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

from .build import KERNELS_SO
from ..utils.knobs import knob

_lock = threading.Lock()
_lib = None

c_int, c_long, c_float, c_void_p, c_uint32 = C.c_int, C.c_long, C.c_float, C.c_void_p, C.c_uint32
c_size_t = C.c_size_t


class OptHyper(C.Structure):
    _fields_ = [("lr", c_float), ("l2", c_float), ("b1", c_float), ("b2", c_float),
                ("eps", c_float), ("momentum", c_float)]


class EpiArgs(C.Structure):
    _fields_ = [("bias", c_void_p), ("hprev", c_void_p), ("scale", c_float), ("seed", c_uint32),
                ("layer", c_uint32), ("keep_thr", c_uint32), ("drop", c_int), ("step", c_void_p),
                ("out", c_void_p), ("out_t", c_void_p)]


class HeadArgs(C.Structure):
    _fields_ = [("h", c_void_p), ("w_out", c_void_p), ("b_out", c_void_p), ("y_fm", c_void_p),
                ("labels", c_void_p), ("M", c_int), ("L", c_int), ("nvalid", c_int),
                ("square_loss", c_int), ("train", c_int), ("gscale", c_float), ("scale_l", c_float),
                ("prob", c_void_p), ("logit", c_void_p), ("dlogit", c_void_p), ("dz", c_void_p),
                ("dz_t", c_void_p), ("partial", c_void_p), ("dh", c_void_p)]


class BnArgs(C.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("nvalid", c_int), ("r", c_void_p), ("dh", c_void_p),
                ("gamma", c_void_p), ("beta", c_void_p), ("mm", c_void_p), ("mv", c_void_p),
                ("save", c_void_p), ("part", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p),
                ("eps", c_float), ("decay", c_float), ("seed", c_uint32), ("layer", c_uint32),
                ("keep_thr", c_uint32), ("drop", c_int), ("inv_keep", c_float), ("step", c_void_p),
                ("out", c_void_p), ("out_t", c_void_p)]


class SlabJob(C.Structure):
    _fields_ = [("dst", c_void_p), ("src", c_void_p), ("n", c_long), ("nslab", c_int),
                ("stride", c_long), ("src_ld", c_long), ("cols", c_int), ("scale", c_float),
                ("lanes", c_int), ("chunk0", c_int)]


class RowSumJob(C.Structure):
    _fields_ = [("dst", c_void_p), ("src", c_void_p), ("rows", c_int), ("n", c_int), ("ld", c_long)]


class ShadowSeg(C.Structure):
    _fields_ = [("off", c_long), ("rows", c_int), ("cols", c_int), ("w16", c_void_p),
                ("wt16", c_void_p)]


class FinOpt(C.Structure):
    _fields_ = [("p", c_void_p), ("g", c_void_p), ("s0", c_void_p), ("s1", c_void_p), ("n", c_long),
                ("h", OptHyper), ("step", c_void_p), ("segs", c_void_p), ("nseg", c_int),
                ("done_ctr", c_void_p)]


class WgFinJob(C.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("slab", c_void_p), ("bslab", c_void_p),
                ("gw", c_void_p), ("gb", c_void_p), ("w16", c_void_p), ("wt16", c_void_p),
                ("w8", c_void_p), ("sdq", c_void_p), ("amax3", c_void_p),
                ("M", c_int), ("N", c_int), ("tiles_m", c_int),
                ("tiles_n", c_int), ("tile0", c_int), ("wg0", c_int)]


class WgFinArgs(C.Structure):
    _fields_ = [("jobs", c_void_p), ("njobs", c_int), ("ldk", c_int), ("kchunk", c_int), ("ns", c_int),
                ("tile_wgs", c_int), ("tile_ctr", c_void_p), ("done_ctr", c_void_p),
                ("partial", c_void_p), ("nhead", c_int), ("L", c_int), ("g_wout", c_void_p),
                ("g_bout", c_void_p), ("g_fmbias", c_void_p), ("loss_sum", c_void_p), ("o", FinOpt),
                ("opt_on", c_int)]


class SegApplyArgs(C.Structure):
    _fields_ = [("sorted_keys", c_void_p), ("ukeys", c_void_p), ("seg_start", c_void_p),
                ("num", c_void_p), ("n", c_int), ("ntiles", c_int), ("compact", c_int),
                ("row_div", c_int), ("vsrc_compact", c_int), ("vsrc", c_void_p),
                ("partial", c_void_p), ("cont", c_void_p), ("UG", c_void_p), ("tv", c_void_p),
                ("tw", c_void_p), ("s0v", c_void_p), ("s1v", c_void_p), ("s0w", c_void_p),
                ("s1w", c_void_p), ("Gv", c_void_p), ("Gw", c_void_p), ("h", OptHyper),
                ("step", c_void_p), ("ldv", c_long), ("ldw", c_long)]


class SweepArgs(C.Structure):
    """tf1_sweep.h SweepArgs: the sweep workgroups of the merged sparse launch (nblk 0: none)."""
    _fields_ = [("rec", c_void_p), ("flags", c_void_p), ("sw_step", c_void_p), ("R", c_long),
                ("ld", c_int), ("nblk", c_int)]


class SfArgs(C.Structure):
    _fields_ = [("sorted_keys", c_void_p), ("perm", c_void_p), ("vals", c_void_p), ("dlogit", c_void_p),
                ("dX0", c_void_p), ("S", c_void_p), ("n", c_int), ("F", c_int), ("KP", c_int),
                ("row_div", c_int), ("ctail", c_void_p), ("lead", c_void_p), ("tinfo", c_void_p),
                ("tv", c_void_p), ("tw", c_void_p), ("s0v", c_void_p), ("s1v", c_void_p),
                ("s0w", c_void_p), ("s1w", c_void_p), ("Gv", c_void_p), ("Gw", c_void_p),
                ("h", OptHyper), ("step", c_void_p), ("ldv", c_long), ("ldw", c_long),
                ("sid", c_void_p), ("upos", c_void_p), ("gout", c_void_p), ("step_off", c_int),
                ("flags", c_void_p), ("sync", c_void_p), ("v_by_key", c_int), ("vbf16", c_int),
                ("grow", c_void_p), ("grow_perm", c_int)]


class ShTable(C.Structure):
    """Owner-side request table (csrc/kernels/shard.hip): key [slots] u64, pos [slots][N] u64."""
    _fields_ = [("key", c_void_p), ("pos", c_void_p), ("mask", C.c_uint32), ("pad", c_int)]


class ShServeArgs(C.Structure):
    """shard_table.h ShServeArgs: a row serve (here: the next batch's, inside the tower launch)."""
    _fields_ = [("recv_ids", c_void_p), ("total", c_int), ("N", c_int), ("C", c_int), ("rstride", c_int),
                ("tv", c_void_p), ("tw", c_void_p), ("ldv", c_long), ("ldw", c_long), ("rows", c_void_p),
                ("step", c_void_p), ("T", ShTable), ("stamp_off", c_int), ("vbf16", c_int),
                ("rbf16", c_int), ("rdiv", c_int), ("rflag", c_void_p)]


class ShApplyArgs(C.Structure):
    _fields_ = [("recv_ids", c_void_p), ("total", c_int), ("N", c_int), ("C", c_int), ("mode", c_int),
                ("rstride", c_int), ("recv_g", c_void_p), ("table", ShTable), ("tv", c_void_p), ("tw", c_void_p),
                ("s0v", c_void_p), ("s1v", c_void_p), ("s0w", c_void_p), ("s1w", c_void_p),
                ("ldv", c_long), ("ldw", c_long), ("Gv", c_void_p), ("Gw", c_void_p), ("h", OptHyper),
                ("step", c_void_p), ("next", ShTable), ("next_rows", c_void_p), ("rdiv", c_int),
                ("vbf16", c_int), ("rbf16", c_int), ("rec", c_void_p), ("rflag", c_void_p), ("R", c_long),
                ("rec_ld", c_int), ("sweep_blocks", c_int)]


class ShDenseArgs(C.Structure):
    _fields_ = [("p", c_void_p), ("g", c_void_p), ("s0", c_void_p), ("s1", c_void_p), ("n", c_long),
                ("h", OptHyper), ("segs", c_void_p), ("nseg", c_int), ("blocks", c_int), ("done", c_void_p),
                ("nsum", c_int)]


class ShRouteBatch(C.Structure):
    """shard.hip ShRouteBatch: one batch's routing set for the run-level routing launches."""
    _fields_ = [("sk", c_void_p), ("perm", c_void_p), ("tcnt", c_void_p), ("sid_incl", c_void_p),
                ("send_ids", c_void_p), ("upos", c_void_p), ("send_cnt", c_void_p), ("num_u", c_void_p),
                ("slot_row", c_void_p)]


class FsJob(C.Structure):
    """fsort_run.h FsJob: one batch of the run-level field sort (chunk sorts + merge)."""
    _fields_ = [("ids", c_void_p), ("ld", c_int), ("B", c_int), ("F", c_int), ("fr", c_void_p),
                ("work", c_void_p), ("nwork", c_int), ("rk", c_void_p), ("rp", c_void_p),
                ("keys", c_void_p), ("perm", c_void_p), ("err", c_void_p), ("mfields", c_void_p),
                ("nmf", c_int), ("mwpf", c_int), ("inv", c_void_p)]


TW_MAXL = 8


class TowerArgs(C.Structure):
    _fields_ = [("M", c_int), ("nvalid", c_int), ("nl", c_int), ("K0p", c_int),
                ("Np", c_int * TW_MAXL), ("E", c_void_p), ("W", c_void_p * TW_MAXL),
                ("WT", c_void_p * TW_MAXL), ("bias", c_void_p * TW_MAXL),
                ("keep_thr", c_uint32 * TW_MAXL), ("inv_keep", c_float * TW_MAXL),
                ("drop", c_int * TW_MAXL), ("seed", c_uint32), ("train", c_int),
                ("square_loss", c_int), ("gscale", c_float), ("step", c_void_p),
                ("w_out", c_void_p), ("b_out", c_void_p), ("y_fm", c_void_p), ("labels", c_void_p),
                ("Ht", c_void_p * TW_MAXL), ("dZt", c_void_p * TW_MAXL), ("dX0", c_void_p),
                ("prob", c_void_p), ("dlogit", c_void_p), ("partial", c_void_p),
                ("h_off", c_int * TW_MAXL), ("dz_off", c_int * 2), ("lds_bytes", c_int),
                ("fp8", c_int), ("E8", c_void_p), ("sE", c_void_p), ("W8", c_void_p * TW_MAXL),
                ("sW", c_void_p * TW_MAXL),
                ("idx", c_void_p), ("vals", c_void_p), ("tv", c_void_p), ("tw", c_void_p),
                ("ldv", c_long), ("ldw", c_long), ("fm_bias", c_void_p), ("F", c_int),
                ("x_off", c_int), ("x8_off", c_int), ("S", c_void_p), ("Et", c_void_p), ("idx_ld", c_int),
                ("id_lim", c_uint32), ("vbf16", c_int), ("serve_wgs", c_int), ("sv", ShServeArgs),
                ("stamp_wgs", c_int), ("stamp_n", c_int), ("stamp_div", c_int), ("stamp_keys", c_void_p),
                ("stamp_flags", c_void_p), ("grow", c_void_p), ("inv", c_void_p), ("g_off", c_int), ("inv_ld", c_int),
                ("dx0_split", c_int), ("l0s", c_int), ("l0_ks", c_int), ("l0z", c_void_p), ("l0fm", c_void_p)]


class CommOp(C.Structure):
    _fields_ = [("kind", c_int), ("pad", c_int), ("send", c_void_p), ("recv", c_void_p),
                ("bytes", C.c_size_t)]


class W8Job(C.Structure):
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("sdq", c_void_p), ("rows", c_int),
                ("cols", c_int), ("row0", c_int), ("pad", c_int), ("amax3", c_void_p)]


class WgJob(C.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("out", c_void_p), ("lda", c_int), ("ldb", c_int),
                ("M", c_int), ("N", c_int), ("tiles_m", c_int), ("tiles_n", c_int),
                ("splitk", c_int), ("kchunk", c_int), ("task0", c_int), ("pad", c_int)]


_SIGS = {
    "hfm_fm_fwd": [c_void_p] * 5 + [c_int] * 4 + [c_void_p] * 6 + [c_long, c_long, c_void_p, c_int,
                                                                      c_void_p],
    "hfm_fm_bwd_sorted": [c_void_p] * 7 + [c_int] * 4 + [c_void_p, c_void_p],
    "hfm_grad_row_bytes": [c_int],
    "hfm_sort_pairs_temp_bytes": [c_int, c_int, C.POINTER(c_size_t)],
    "hfm_sort_ids": [c_void_p] * 4 + [c_int, c_int, c_void_p, c_size_t, c_void_p],
    "hfm_reduce_by_key_temp_bytes": [c_int, c_int, C.POINTER(c_size_t)],
    "hfm_reduce_by_key": [c_int] + [c_void_p] * 5 + [c_int, c_void_p, c_size_t, c_void_p],
    "hfm_scan_temp_bytes": [c_int, C.POINTER(c_size_t)],
    "hfm_unique_inverse": [c_void_p, c_void_p, c_int] + [c_void_p] * 6 + [c_size_t, c_void_p],
    "hfm_owner_keys": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "hfm_gather_i32": [c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "hfm_expand_vals": [c_void_p, c_int, C.c_uint64, c_int, c_long, c_void_p, c_void_p],
    "hfm_sparse_rows_update": [c_int, c_int] + [c_void_p] * 3 + [c_int, c_int] + [c_void_p] * 6
                              + [C.POINTER(OptHyper), c_void_p, c_long, c_long, c_void_p],
    "hfm_scatter_rows": [c_int] + [c_void_p] * 3 + [c_int, c_int, c_void_p, c_void_p, c_void_p],
    "hfm_dense_sweep": [c_int, c_int, c_long] + [c_void_p] * 8 + [C.POINTER(OptHyper), c_void_p, c_long,
                                                                  c_long, c_void_p],
    "hfm_stamp_rows": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p],
    "hfm_tf1_sweep": [c_int, c_int, c_long, c_void_p, c_int, c_void_p, C.POINTER(OptHyper), c_void_p,
                      c_void_p, c_int, c_void_p],
    "hfm_dense_opt": [c_int] + [c_void_p] * 4+ [c_long, C.POINTER(OptHyper), c_void_p, c_void_p, c_int,
                                                 c_void_p, c_void_p],
    "hfm_finalize": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p],
    "hfm_finalize_opt": [c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int] + [c_void_p] * 4
                        + [c_long, C.POINTER(OptHyper), c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "hfm_shadow_refresh": [c_void_p, c_long, c_void_p, c_int, c_void_p],
    "hfm_step_inc": [c_void_p, c_void_p],
    "hfm_shadow_seg_bytes": [],
    "hfm_opt_hyper_bytes": [],
    "hfm_gemm_nt": [c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                    C.POINTER(EpiArgs), c_void_p],
    "hfm_epi_pass": [c_int, c_void_p, c_int, c_int, C.POINTER(EpiArgs), c_void_p],
    "hfm_epi_args_bytes": [],
    "hfm_head": [C.POINTER(HeadArgs), c_void_p],
    "hfm_shadow_transpose": [c_void_p, c_int, c_int, c_void_p],
    "hfm_head_args_bytes": [],
    "hfm_slab_reduce": [c_void_p, c_int, c_int, c_void_p],
    "hfm_slab_job_bytes": [],
    "hfm_rowsum": [c_void_p, c_int, c_int, c_void_p],
    "hfm_rowsum_job_bytes": [],
    "hfm_auc_hist": [c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "hfm_sumsq_partials": [c_void_p, c_long, c_void_p, c_int, c_void_p],
    "hfm_seg_tiles": [c_int, c_int],
    "hfm_radix_sort_temp_bytes": [c_int, C.POINTER(c_size_t)],
    "hfm_onesweep_temp_bytes": [c_int, C.POINTER(c_size_t)],
    "hfm_onesweep_sort_ids": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_uint32,
                              c_void_p, c_void_p],
    "hfm_onesweep_error_offset": [],
    "hfm_field_sort_max_rows": [],
    "hfm_field_sort_chunk_rows": [],
    "hfm_comm_id_bytes": [],
    "hfm_comm_unique_id": [c_void_p],
    "hfm_comm_init": [C.POINTER(c_void_p), c_int, c_int, c_void_p],
    "hfm_comm_destroy": [c_void_p],
    "hfm_comm_allreduce_f32": [c_void_p, c_void_p, c_size_t, c_void_p],
    "hfm_comm_alltoall": [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
    "hfm_comm_allgather": [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
    "hfm_comm_alltoall_allgather": [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, c_void_p],
    "hfm_comm_group": [c_void_p, c_void_p, c_int, c_void_p],
    "hfm_decode_examples": [c_void_p, c_void_p, c_int, c_int, C.c_longlong, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_int, c_void_p],
    "hfm_lb_shared_bytes": [],
    "hfm_lb_barrier_selftest": [C.c_char_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int],
    "hfm_lb_create": [C.POINTER(c_void_p), c_int, c_int, C.c_char_p, c_int, c_int],
    "hfm_lb_ipc_handle_bytes": [],
    "hfm_lb_alloc_stage": [c_void_p, c_size_t, c_void_p],
    "hfm_lb_open_peers": [c_void_p, c_void_p],
    "hfm_lb_group": [c_void_p, c_void_p, c_int, c_void_p],
    "hfm_lb_stage_half_kb": [c_void_p],
    "hfm_lb_error": [c_void_p],
    "hfm_lb_destroy": [c_void_p],
    "hfm_sh_count_blocks": [c_int],
    "hfm_sh_route_tiles": [c_int],
    "hfm_sh_route": [c_void_p, c_int, c_int, c_int] + [c_void_p] * 7 + [c_void_p],
    "hfm_sh_route_run": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "hfm_sh_route_batch_bytes": [],
    "hfm_sh_bucket": [c_void_p, c_void_p, c_int, c_int, c_int] + [c_void_p] * 5 + [c_void_p],
    "hfm_sh_slot_rows": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "hfm_sh_serve": [c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_long, c_long, c_void_p,
                     c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "hfm_sh_owner_apply": [c_int, c_int, c_void_p, c_void_p],
    "hfm_sh_apply_args_bytes": [],
    "hfm_sh_apply_dense": [c_int, c_int, c_void_p, c_void_p, c_void_p],
    "hfm_sh_dense_args_bytes": [],
    "hfm_sparse_fused_tiles": [c_int, c_int],
    "hfm_sparse_fused": [c_int, c_int, c_int, c_void_p, c_void_p],
    "hfm_sparse_fused_args_bytes": [],
    "hfm_field_sort_max_pb": [],
    "hfm_field_sort": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int] + [c_void_p] * 6 + [c_void_p],
    "hfm_field_sort_pre": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int] + [c_void_p] * 5 + [c_void_p],
    "hfm_radix_sort_ids": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p],
    "hfm_segments": [c_void_p, c_int] + [c_void_p] * 5 + [c_void_p, c_size_t, c_void_p],
    "hfm_fm_bwd_seg": [c_int] + [c_void_p] * 7 + [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "hfm_seg_apply": [c_int, c_int, c_int, C.POINTER(SegApplyArgs), c_int, c_void_p],
    "hfm_seg_apply_args_bytes": [],
    "hfm_bn": [c_int, C.POINTER(BnArgs), c_void_p],
    "hfm_tower": [C.POINTER(TowerArgs), c_int, c_void_p],
    "hfm_wgfin": [c_int, C.POINTER(WgFinArgs), c_void_p],
    "hfm_sparse_wgfin": [c_int, c_int, c_void_p, C.POINTER(WgFinArgs), c_void_p, c_void_p, c_void_p],
    "hfm_fs_job_bytes": [],
    "hfm_fs2_chunk_rows": [],
    "hfm_fs2_merge_wgs_per_run": [],
    "hfm_field_sort_run": [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p],
    "hfm_sparse_wgfin_x": [c_int, c_void_p, C.POINTER(WgFinArgs), c_void_p, c_void_p],
    "hfm_wgfin_job_bytes": [],
    "hfm_wgfin_args_bytes": [],
    "hfm_tower_args_bytes": [],
    "hfm_tower_stamp_rows_per_wg": [],
    "hfm_wgrad_group": [c_void_p, c_int, c_int, c_void_p],
    "hfm_wg_job_bytes": [],
    "hfm_w8_quant": [c_void_p, c_int, c_int, c_void_p],
    "hfm_w8_job_bytes": [],
    "hfm_bn_args_bytes": [],
}


def lib_path() -> str:
    return knob("HIPFM_KERNELS_SO") or KERNELS_SO


def available() -> bool:
    return os.path.exists(lib_path())


def get_lib():
    """Load (once) and return the kernel library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = lib_path()
        if not os.path.exists(p):
            raise RuntimeError(f"hipfm kernel library not found at {p}; build it with "
                               "`python -m hipfm.ops.build` (or __graft_entry__.build())")
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        # ABI checks: ctypes struct layouts must match the C structs
        for cname, pys in (("hfm_epi_args_bytes", EpiArgs), ("hfm_head_args_bytes", HeadArgs),
                           ("hfm_slab_job_bytes", SlabJob), ("hfm_rowsum_job_bytes", RowSumJob),
                           ("hfm_shadow_seg_bytes", ShadowSeg), ("hfm_opt_hyper_bytes", OptHyper),
                           ("hfm_seg_apply_args_bytes", SegApplyArgs), ("hfm_bn_args_bytes", BnArgs),
                           ("hfm_tower_args_bytes", TowerArgs), ("hfm_wg_job_bytes", WgJob),
                           ("hfm_wgfin_job_bytes", WgFinJob), ("hfm_wgfin_args_bytes", WgFinArgs),
                           ("hfm_w8_job_bytes", W8Job),
                           ("hfm_sparse_fused_args_bytes", SfArgs),
                           ("hfm_sh_apply_args_bytes", ShApplyArgs),
                           ("hfm_sh_dense_args_bytes", ShDenseArgs), ("hfm_fs_job_bytes", FsJob),
                           ("hfm_sh_route_batch_bytes", ShRouteBatch)):
            n = getattr(lib, cname)()
            if n != C.sizeof(pys):
                raise RuntimeError(f"ABI mismatch {pys.__name__}: C {n} vs ctypes {C.sizeof(pys)}")
        _lib = lib
        return _lib


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"hipfm kernel call {what} failed with hipError {rc}")


def stream_handle(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


STAMP_BUFS = ("hfm_st_tower", "hfm_st_sf")


def dump_stamps(path: str) -> bool:
    """Diagnostic stamp build (HIPFM_BUILD_STAMPS=1): save every stamp buffer the loaded library
    has ([slots, 16] uint64 100-MHz wall-clock stamps per workgroup) to ``path`` (.npz).  Returns
    False for a production library (it has no stamp buffers)."""
    import numpy as np
    lib = get_lib()
    out = {}
    for name in STAMP_BUFS:
        fn = getattr(lib, name + "_read", None)
        if fn is None:
            continue
        slots = getattr(lib, name + "_slots")()
        buf = np.zeros((slots, 16), dtype=np.uint64)
        fn.argtypes = [c_void_p, C.c_size_t]
        fn.restype = c_int
        check(fn(buf.ctypes.data, buf.nbytes), name + "_read")
        out[name] = buf
    if not out:
        return False
    np.savez_compressed(path, **out)
    return True
