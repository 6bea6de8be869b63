"""The per-layer (unfused) MLP path of NativeDeepFM: towers the fused kernel cannot hold -- batch
norm (batch-wide statistics between the GEMMs, 2-hvd-gpu/DeepFM-hvd-tfrecord-vectorized-map.py
:204-210,283-287) and wide layers (the reference's GPU recipe, deep_layers 4096,4096,4096, DOC
p.37) -- as one NT GEMM launch per layer and direction (csrc/kernels/mlp.hip), the head
(hfm_head), the split-K / bias finalize and batch norm (bn.hip); plus the tile and split-K
choices of those GEMMs.  Mixed into NativeDeepFM (models/deepfm.py), whose buffers it uses."""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import kernels as KN
from ..ops._lib import BnArgs, EpiArgs, HeadArgs, RowSumJob, SlabJob
from ..utils.knobs import flag
from ..utils.rng import keep_threshold

_LDS_GEMM = flag("HIPFM_LDS_GEMM")           # wide per-layer GEMMs on the LDS-staged MFMA tiles
_WG_DIRECT = flag("HIPFM_WG_DIRECT")         # unsplit wide wgrad stores straight into g
_WG_BLAS = flag("HIPFM_WG_BLAS")             # ... as a plain library GEMM (no epilogue to fuse)
_EPI_BLAS = flag("HIPFM_EPI_BLAS")           # wide fwd / dgrad: library GEMM + epilogue pass
_DX0_BLAS = flag("HIPFM_DX0_BLAS")           # the wide tower's dX0 as a library GEMM (bf16 out)


def _lds_tile_ok(M: int, N: int, Kd: Optional[int], splitk: int = 1) -> bool:
    """The 128 x 128 LDS-staged tile (mlp.hip gemm_lds_kernel) for a GEMM with at least 256
    output tiles (a 4096-wide layer at any batch >= 1024; the reference's GPU tower, DOC p.37):
    there the register-fed 32-row tiles re-read both operands from L2 per wave."""
    return (Kd is not None and M % 128 == 0 and N % 128 == 0 and Kd % (64 * splitk) == 0
            and (M // 128) * (N // 128) * splitk >= 256)


def _pick_tile(M: int, N: int, row_major_stream: bool = True, Kd: Optional[int] = None,
               allow_lds: bool = True) -> int:
    """Tile for an NT GEMM.  Wide layers (``_lds_tile_ok``, the reduction depth ``Kd`` given) take
    the LDS-staged 128 x 128 workgroup tile; otherwise activation GEMMs (M = batch) take the
    widest column tile that covers N in one workgroup row, so the big A operand (E, H, dZ) is
    streamed exactly once."""
    if allow_lds and _LDS_GEMM and _lds_tile_ok(M, N, Kd):
        # 256 x 256 ping-pong tile where it tiles the output 128+ times (0.45-0.66x hipBLASLt at the
        # 4096-wide tower, 1.15-1.3x the 128 x 128 tile: profiles/r6_gemm_bench_pingpong.log)
        if M % 256 == 0 and N % 256 == 0 and (M // 256) * (N // 256) >= 128:
            return KN.TILE_PP
        return KN.TILE_LDS
    if row_major_stream and M % 32 == 0:
        for t, w in ((3, 32), (4, 64), (2, 128), (5, 160), (7, 256), (6, 320)):
            if N == w:
                return t
        if N % 320 == 0:
            return 6
        if N % 256 == 0:
            return 7
        if N % 160 == 0:
            return 5
        if N % 128 == 0:
            return 2
    if M % 64 == 0 and N % 64 == 0:
        return 0
    if N == 32 and M % 128 == 0:
        return 1
    if M == 32 and N % 128 == 0:
        return 2
    if M == 32 and N % 64 == 0:
        return 4
    return 3


def _epi_blas_ok(M: int, N: int, Kd: int) -> bool:
    """Wide forward / dgrad GEMMs (the 256 x 256 ping-pong tile's shapes, reduction >= 1024) as a
    library GEMM into an fp32 scratch + the stand-alone epilogue pass (mlp.hip epi_pass_kernel)."""
    return bool(_EPI_BLAS and Kd >= 1024 and _pick_tile(M, N, Kd=Kd) == KN.TILE_PP)


def _pick_splitk(M: int, N: int, Kd: int, tile: int, target_blocks: int = 512,
                 max_split: int = 32) -> int:
    """Split the batch reduction of a weight-gradient GEMM: enough workgroups to fill the
    256 CUs, but few enough slabs that the finalize pass stays a short, coalesced read."""
    bm, bn = KN.TILES[tile]
    tiles = (M // bm) * (N // bn)
    ksteps = Kd // (64 if tile in (KN.TILE_LDS, KN.TILE_PP) else 32)
    want = max(1, min(ksteps, max_split, target_blocks // max(1, tiles)))
    for s in range(want, 0, -1):
        if ksteps % s == 0:
            return s
    return 1


class LayerPathMixin:
    """Per-layer forward / backward of the deep tower (NativeDeepFM, unfused)."""

    def _forward(self, B: int, train: bool):
        M = self.M
        idx, tv = self._fm_forward(B, train)
        X = self.E
        for i in range(len(self.layers)):
            s = self.dense_segs[f"Deep-part/mlp{i}/biases"]
            keep = self.keep[i]
            drop = train and keep < 1.0
            ep = EpiArgs()
            ep.bias = self.p.data_ptr() + 4 * s.off
            ep.scale = (1.0 / keep) if drop else 1.0
            ep.seed = self.seed & 0xFFFFFFFF
            ep.layer = i
            ep.keep_thr = min(keep_threshold(keep), 0xFFFFFFFF)
            ep.drop = 1 if drop else 0
            ep.step = self.step.data_ptr()
            ep.out = self.H[i].data_ptr()
            ep.out_t = self.Ht[i].data_ptr() if train else 0
            N = self.Np[i]
            if self.batch_norm:
                ep.out, ep.out_t = self.Rb[i].data_ptr(), 0
                KN.gemm_nt(KN.EPI_RELU_F32, _pick_tile(M, N, Kd=self.Kp[i]), X, self.Kp[i], self.W16[i],
                           self.Kp[i], M, N, self.Kp[i], 1, ep)
                self._bn_forward(i, B, train)
            elif _epi_blas_ok(M, N, self.Kp[i]):
                cf = self.cbuf[:M * N].view(M, N)
                torch.mm(X.view(M, self.Kp[i]), self.W16[i].view(N, self.Kp[i]).t(), out_dtype=torch.float32,
                         out=cf)
                KN.epi_pass(KN.EPI_FWD if train else KN.EPI_FWD_EVAL, cf, M, N, ep)
            else:
                KN.gemm_nt(KN.EPI_FWD if train else KN.EPI_FWD_EVAL, _pick_tile(M, N, Kd=self.Kp[i]), X,
                           self.Kp[i], self.W16[i], self.Kp[i], M, N, self.Kp[i], 1, ep)
            X = self.H[i]
        return idx, tv

    def _bn_args(self, i: int, B: int, drop: bool) -> BnArgs:
        a = BnArgs()
        a.M, a.N, a.nvalid = self.M, self.Np[i], B
        a.r = self.Rb[i].data_ptr()
        a.dh = self.dH[i].data_ptr()
        pb = self.p.data_ptr()
        gb = self.g.data_ptr()
        sb = self.dense_segs[f"Deep-part/bn_{i}/beta"].off
        sg = self.dense_segs[f"Deep-part/bn_{i}/gamma"].off
        a.beta, a.gamma = pb + 4 * sb, pb + 4 * sg
        a.dbeta, a.dgamma = gb + 4 * sb, gb + 4 * sg
        a.mm, a.mv = self.bn_mm[i].data_ptr(), self.bn_mv[i].data_ptr()
        a.save = self.bn_save[i].data_ptr()
        a.part = self.bn_part.data_ptr()
        a.eps, a.decay = self.bn_eps, self.bn_decay
        keep = self.keep[i]
        a.seed = self.seed & 0xFFFFFFFF
        a.layer = i
        a.keep_thr = min(keep_threshold(keep), 0xFFFFFFFF)
        a.drop = 1 if (drop and keep < 1.0) else 0
        a.inv_keep = (1.0 / keep) if a.drop else 1.0
        a.step = self.step.data_ptr()
        return a

    def _bn_forward(self, i: int, B: int, train: bool):
        """relu output R -> batch norm (batch stats + moving update, or moving stats) ->
        dropout -> H (and H^T when training)."""
        a = self._bn_args(i, B, drop=train)
        if train:
            KN.bn(KN.BN_FWD_PARTIAL, a)
            KN.bn(KN.BN_FWD_FINALIZE, a)
        else:
            KN.bn(KN.BN_EVAL_FINALIZE, a)
        a.out = self.H[i].data_ptr()
        a.out_t = self.Ht[i].data_ptr() if train else 0
        KN.bn(KN.BN_FWD_APPLY, a)

    def _bn_backward(self, i: int, B: int):
        """dH_i (f32) -> dZ_i, dZ_i^T (bf16) through dropout, batch norm and relu; writes the
        beta/gamma gradients into the flat gradient buffer."""
        a = self._bn_args(i, B, drop=True)
        KN.bn(KN.BN_BWD_PARTIAL, a)
        KN.bn(KN.BN_BWD_FINALIZE, a)
        a.out, a.out_t = self.dZ[i].data_ptr(), self.dZt[i].data_ptr()
        KN.bn(KN.BN_BWD_APPLY, a)

    def _head(self, B: int, train: bool, with_labels: bool = True):
        a = HeadArgs()
        a.h = self.H[-1].data_ptr()
        a.w_out = self.p.data_ptr() + 4 * self.dense_segs["Deep-part/deep_out/weights"].off
        a.b_out = self.p.data_ptr() + 4 * self.dense_segs["Deep-part/deep_out/biases"].off
        a.y_fm = self.y_fm.data_ptr()
        a.labels = self.labels.data_ptr() if with_labels else 0
        a.M, a.L, a.nvalid = self.M, self.Np[-1], B
        a.square_loss = 1 if self.loss_type == "square_loss" else 0
        a.train = 1 if train else 0
        a.gscale = 1.0 / (B * self.world)
        keep = self.keep[-1]
        a.scale_l = (1.0 / keep) if keep < 1.0 else 1.0
        a.prob = self.prob.data_ptr()
        a.logit = 0
        a.dlogit = self.dlogit.data_ptr()
        a.dz = self.dZ[-1].data_ptr()
        a.dz_t = self.dZt[-1].data_ptr()
        a.partial = self.partial.data_ptr()
        a.dh = self.dH[-1].data_ptr() if (self.batch_norm and train) else 0
        KN.head(a)

    # ------------------------------------------------------------------ backward pieces
    def _mlp_backward(self, B: int):
        M = self.M
        for i in reversed(range(len(self.layers))):
            if self.batch_norm:
                self._bn_backward(i, B)
            Xt = self.Et if i == 0 else self.Ht[i - 1]
            t, s = self.wg_cfg[i]
            ep = EpiArgs()
            if self.wg_direct[i] and _WG_BLAS:
                # a plain GEMM with nothing to fuse: bf16 operands, fp32 result written in place
                go = self.dense_segs[f"Deep-part/mlp{i}/weights"].off
                gw = self.g[go:go + self.Np[i] * self.Kp[i]].view(self.Np[i], self.Kp[i])
                torch.mm(self.dZt[i], Xt.t(), out_dtype=torch.float32, out=gw)
            else:
                if self.wg_direct[i]:   # unsplit: the GEMM writes the final gradient itself
                    ep.out = self.g.data_ptr() + 4 * self.dense_segs[f"Deep-part/mlp{i}/weights"].off
                else:
                    ep.out = self.slabs[i].data_ptr()
                KN.gemm_nt(KN.EPI_F32, t, self.dZt[i], M, Xt, M, self.Np[i], self.Kp[i], M, s, ep)
            ep = EpiArgs()
            if i > 0 and self.batch_norm:
                ep.out = self.dH[i - 1].data_ptr()    # f32 dL/dH_{i-1}; BN backward masks it
                N = self.Np[i - 1]
                if _epi_blas_ok(M, N, self.Np[i]):    # a plain GEMM: nothing to fuse
                    torch.mm(self.dZ[i].view(M, self.Np[i]), self.WT16[i].view(N, self.Np[i]).t(),
                             out_dtype=torch.float32, out=self.dH[i - 1].view(M, N))
                else:
                    KN.gemm_nt(KN.EPI_F32, _pick_tile(M, N, Kd=self.Np[i]), self.dZ[i], self.Np[i],
                               self.WT16[i], self.Np[i], M, N, self.Np[i], 1, ep)
            elif i > 0:
                keep = self.keep[i - 1]
                ep.hprev = self.H[i - 1].data_ptr()
                ep.scale = (1.0 / keep) if keep < 1.0 else 1.0
                ep.out = self.dZ[i - 1].data_ptr()
                ep.out_t = self.dZt[i - 1].data_ptr()
                N = self.Np[i - 1]
                if _epi_blas_ok(M, N, self.Np[i]):
                    cf = self.cbuf[:M * N].view(M, N)
                    torch.mm(self.dZ[i].view(M, self.Np[i]), self.WT16[i].view(N, self.Np[i]).t(),
                             out_dtype=torch.float32, out=cf)
                    KN.epi_pass(KN.EPI_DGRAD, cf, M, N, ep)
                else:
                    KN.gemm_nt(KN.EPI_DGRAD, _pick_tile(M, N, Kd=self.Np[i]), self.dZ[i], self.Np[i],
                               self.WT16[i], self.Np[i], M, N, self.Np[i], 1, ep)
            elif _DX0_BLAS and self.Np[0] >= 1024 and not self.batch_norm:
                # unmasked, unscaled bf16 product: a plain library GEMM with a bf16 result
                torch.mm(self.dZ[0].view(M, self.Np[0]), self.WT16[0].view(self.K0p, self.Np[0]).t(),
                         out=self.dX0.view(M, self.K0p))
            else:
                ep.out = self.dX0.data_ptr()          # hprev = 0: unmasked bf16 store
                ep.scale = 1.0
                KN.gemm_nt(KN.EPI_DGRAD, _pick_tile(M, self.K0p, Kd=self.Np[0]), self.dZ[0], self.Np[0],
                           self.WT16[0], self.Np[0], M, self.K0p, self.Np[0], 1, ep)
        self._finalize_grads()

    def _finalize_grads(self):
        if self._sp.fuse_opt:
            KN.finalize_opt(self.opt_id, self._slab_jobs, self._nslab_jobs, self._slab_blocks,
                            self._row_jobs, self._nrow_jobs, self._row_total, self.p, self.g,
                            self.sd[0], self.sd[1], self.P, self.h_dense, self.step,
                            self._shadow_opt, self._nshadow, self._done_ctr)
            if self._shadow_t is not None:
                KN.shadow_transpose(*self._shadow_t)
            return
        KN.finalize(self._slab_jobs, self._nslab_jobs, self._slab_blocks, self._row_jobs,
                    self._nrow_jobs, self._row_total)

    def _build_finalize_jobs(self):
        jobs = []
        maxn = 1
        for i in range(len(self.layers)):
            if self.wg_direct[i]:
                continue
            s = self.dense_segs[f"Deep-part/mlp{i}/weights"]
            n = self.Np[i] * self.Kp[i]
            nsl = self.wg_cfg[i][1]
            jobs.append(SlabJob(self.g.data_ptr() + 4 * s.off, self.slabs[i].data_ptr(), n, nsl, n,
                                self.Kp[i], self.Kp[i], 1.0))
            maxn = max(maxn, n)
        Lp = self.Np[-1]
        pw = self.partial.data_ptr()
        so = self.dense_segs["Deep-part/deep_out/weights"].off
        sb = self.dense_segs["Deep-part/deep_out/biases"].off
        sf = self.dense_segs["fm_bias"].off
        g0 = self.g.data_ptr()
        jobs.append(SlabJob(g0 + 4 * so, pw, Lp, self.nhead, Lp + 2, Lp, Lp, 1.0))
        jobs.append(SlabJob(g0 + 4 * sb, pw + 4 * Lp, 1, self.nhead, Lp + 2, 1, 1, 1.0))
        jobs.append(SlabJob(g0 + 4 * sf, pw + 4 * Lp, 1, self.nhead, Lp + 2, 1, 1, 1.0))
        jobs.append(SlabJob(self.loss_sum.data_ptr(), pw + 4 * (Lp + 1), 1, self.nhead, Lp + 2, 1, 1, 1.0))
        nb = 0
        for j in jobs:                       # finalize_kernel block mapping
            # slab-lanes per output: each thread sums <= 8 slabs, all its loads in flight at once
            # (the 512 head-partial rows of the 1-block jobs were 64 dependent-load rounds)
            # (<= 4 slabs -- the per-layer wide wgrad's split-K -- one thread per element, its
            # slabs summed in order: the same sums as 4 lanes, at 256 elements per workgroup
            # instead of 64; 16.7M-element layers had 262K workgroups)
            j.lanes = 64 if j.nslab >= 256 else (8 if j.nslab >= 64 else (4 if j.nslab > 4 else 1))
            j.chunk0 = nb
            nb += (j.n + 256 // j.lanes - 1) // (256 // j.lanes)
        self._slab_blocks = nb
        self._slab_jobs = KN.struct_array_to_device(jobs, self.device)
        self._nslab_jobs = len(jobs)
        self._slab_maxn = maxn
        rj = []
        for i in range(len(self.layers)):
            sbias = self.dense_segs[f"Deep-part/mlp{i}/biases"].off
            rj.append(RowSumJob(g0 + 4 * sbias, self.dZt[i].data_ptr(), self.Np[i], self.M, self.M))
        self._row_jobs = KN.struct_array_to_device(rj, self.device)
        self._nrow_jobs = len(rj)
        self._row_total = sum(self.Np)
        # the dense optimizer can ride on the finalize launch only if finalize writes the final
        # gradient of EVERY flat parameter (not so with batch norm: bn.hip writes beta / gamma).
        # Only the segments count: the 64-element alignment gaps between them hold no parameter
        # (their p / g / slots stay 0, which every optimizer maps to 0 -- dense_opt's sweep over
        # them is a no-op).
        cov = torch.zeros(self.P, dtype=torch.bool)
        for d, n in [(j.dst, j.n) for j in jobs] + [(r.dst, r.rows) for r in rj]:
            o = (d - g0) // 4
            if 0 <= o < self.P:
                cov[o:o + n] = True
        need = torch.zeros(self.P, dtype=torch.bool)
        for s in self.dense_segs.values():
            need[s.off:s.off + int(torch.Size(s.shape).numel())] = True
        self._fin_covers_all = bool(cov[need].all()) and not self.batch_norm
