// Fused deep tower (SURVEY §2.5 rows 2-7, 9-12, 15-16 "small-N specialization fuses the whole
// tower, with activations kept in LDS"): for a block of 32 samples ONE workgroup runs
//
//   gather    (K1, optional) E = fm_v[ids] * x, y_w, y_v, S = sum_f E straight into an LDS tile:
//             E never goes through HBM; E^T (wgrad operand) and S (sparse backward) are written
//   forward   H_i = dropout(relu(H_{i-1} W_i^T + b_i))      i = 0..nl-1   (H_{-1} = E)
//   head      y = y_fm + H_last . w_out + b_out, p, loss, dlogit, dZ_last
//   dgrad     dZ_{i-1} = (dZ_i W_i) (.) [H_{i-1} > 0] / keep   (row-local: needs only this block)
//             dX0      =  dZ_0 W_0
//
// with every H_i and dZ_i tile resident in LDS (bf16, rows padded by 8 elements), weights read
// from L2 as MFMA B fragments, and only what later kernels need written to HBM: H_i^T and
// dZ_i^T (operands of the batch-reduction wgrad GEMMs), dX0 (FM backward), prob / dlogit and
// per-block head partials.  This replaces 3 forward GEMMs + head + 3 dgrad GEMMs (7 launches;
// each kernel boundary in a HIP graph costs a few us on MI355X, see tools/bench_launch.py) by
// one.  The weight gradients (reductions over the whole batch) run afterwards as ONE grouped
// launch (wgrad_group_kernel) whose unit of work is a single wave owning a 32x32 tile of one
// layer's split-K slab.
//
// MFMA: v_mfma_f32_16x16x32_bf16, one wave = 32x32 outputs (2x2 tiles); A fragment lane l:
// A[l&15][8(l>>4)+j], B fragment B[8(l>>4)+j][l&15]; C: col = l&15, row = (l>>4)*4 + j.
// Dropout masks: counter hash, flat index (global row) * Npad + col, identical to mlp.hip.
#include "common.h"
#include "mma32.h"
#include "shard_table.h"

constexpr int TW_MAXL = 8;
constexpr int TW_ROWS = 32;
// k-steps of A/B fragments in flight per wave: PF0 = 4 for layer 0, PF1 = 2 for the other GEMMs
// (deeper rings need > 128 VGPRs, i.e. fewer resident waves, and measured slower).

struct TowerArgs {
  int M, nvalid, nl, K0p;
  int Np[TW_MAXL];
  const bf16* E;                  // [M, K0p]
  const bf16* W[TW_MAXL];         // [Np_i, Kp_i]
  const bf16* WT[TW_MAXL];        // [Kp_i, Np_i]
  const float* bias[TW_MAXL];
  uint32_t keep_thr[TW_MAXL];
  float inv_keep[TW_MAXL];
  int drop[TW_MAXL];
  uint32_t seed;
  int train;                      // 1: forward + head + dgrad chain; 0: forward + head (eval)
  int square_loss;
  float gscale;                   // 1 / global batch
  const int64_t* step;
  const float* w_out;             // [Np_last]
  const float* b_out;             // [1]
  float* y_fm;                    // [M] (gather variant: written, the FM logit part)
  const float* labels;            // [M] or null
  bf16* Ht[TW_MAXL];              // [Np_i, M]   (train)
  bf16* dZt[TW_MAXL];             // [Np_i, M]   (train)
  bf16* dX0;                      // [M, K0p]    (train)
  float* prob;                    // [M]
  float* dlogit;                  // [M]         (train)
  float* partial;                 // [M/32, Np_last + 2]
  int h_off[TW_MAXL];             // LDS element offsets of the H tiles
  int dz_off[2];                  // LDS element offsets of the two dZ tiles
  int lds_bytes;
  // fp8 forward (mlp_dtype = fp8): every forward GEMM on v_mfma_f32_16x16x32_fp8_fp8 with OCP
  // e4m3 operands — E8 rows (fm_fwd) / H rows (quantized from the LDS tile) with per-row
  // power-of-two scales, W8 with per-output-channel scales — dequantized in the fp32 epilogue.
  // The backward (dgrad chain, wgrad) stays bf16.
  int fp8;
  const uint8_t* E8;              // [M, K0p]
  const float* sE;                // [M]     row dequant factors of E8
  const uint8_t* W8[TW_MAXL];     // [Np_i, Kp_i]
  const float* sW[TW_MAXL];       // [Np_i]  channel dequant factors of W8
  // fused FM gather (K1 in the prologue; template KE = embedding size, 0 = E read from global):
  // per slot (b, f) row id = idx[b*F + f] of the table (tv, tw: row strides ldv, ldw)
  const int* idx;
  const float* vals;              // [M, F]
  const float* tv;
  const float* tw;
  long ldv, ldw;
  const float* fm_bias;           // [1]
  int F;
  int x_off;                      // LDS element offset of the bf16 E tile [32][K0p + 8]
  int x8_off;                     // LDS byte offset of the fp8 E tile [32][K0p + 16] (fp8)
  float* S;                       // [M, K]  sum_f E (sparse backward)
  bf16* Et;                       // [K0p, M] (train: wgrad operand)
  int idx_ld;                     // 0: idx row-major [M, F]; else field-major [F, idx_ld] (the
                                  // layout the per-field sort reads, so it needs no transpose)
  unsigned id_lim;                // > 0: gathered row ids clamped to [0, id_lim) (a bad id never
                                  // reads out of bounds; the slot sort flags it for the host)
  int vbf16;                      // table v rows are bf16 (mixed-precision embeddings)
  // run-routed row-sharded step: serve_wgs workgroups AFTER the tower's serve the NEXT batch's
  // rows ahead (shard_table.h; the owner update of this step patches the rows it changes)
  int serve_wgs;
  ShServeArgs sv;
  // tf1_dense run-sorted step: stamp_wgs workgroups after those flag this batch's rows for the
  // sparse launch's merged sweep (stamp_flags[key / stamp_div] = 1 per run of the sorted keys)
  int stamp_wgs, stamp_n, stamp_div;
  const int* stamp_keys;
  unsigned char* stamp_flags;
  // sorted gradient rows (bf16 gather tower, train, run-sorted step): every slot's embedding
  // gradient row {a[K], g_w, c} is written to grow[inv[slot]] -- its SORTED position -- so
  // the sparse backward streams them (no per-slot gather); dX0 / S are then not written.  g_off:
  // LDS byte offset of the scratch [x 32 x F][S 32 x K][inv 32 x F][4 wave tiles 32 x 40 bf16].
  float* grow;
  const int* inv;   // [F][inv_ld] field-major sorted index of slot (b, f) (fsort_run.h FsJob.inv)
  int g_off;
  int inv_ld;
  // dX0 in a launch of its own (hfm_tower enqueues tower_dx0_kernel after the tower; bf16 tower,
  // train, no gradient rows): at B = 1024 the tower has 32 blocks on 256 CUs and its dX0 phase
  // (K0p / 32 tiles of W_0 per block) was 15 of its 51 us at K = 32
  int dx0_split;
  // FM gather + layer 0 split over field slices (small batches: at B = 1024 the tower has 32
  // blocks on 256 CUs and its gather + layer-0 reduction over 39 fields was 18 of its 36 us):
  // tower_l0s_kernel, l0s workgroups per 32-row block, each gathers the fields of l0_ks k-steps
  // (32 columns of E each), stores its E^T columns and writes fp32 partials -- layer 0's pre-
  // activations l0z [l0s][M][Np0] and the FM sums l0fm [l0s][M][KE + 2] = {S[KE], sum_k Q_k, y_w};
  // the tower then sums the partials in slice order instead of gathering
  int l0s, l0_ks;
  float* l0z;
  float* l0fm;
};
constexpr int TW_GINV = 8;  // inv entries prefetched per thread (32 F / 256 <= 8: F <= 64)

constexpr int TW_STAMP_EPT = 16;  // sorted keys per thread of a stamp workgroup
HFM_STAMP_BUF(hfm_st_tower)
#define TW_ST(k) HFM_STAMP(hfm_st_tower, blockIdx.x, (k) < 15 ? (k) : 15)

// fp8 variant of mma32 (16x16x32 fp8 MFMA; same fragment map as bf16 with 8 one-byte elements
// per lane): A and B are e4m3 rows in global memory (row strides in bytes).
template <int PF>
__device__ __forceinline__ void mma32_f8(const uint8_t* __restrict__ A, int lda, const uint8_t* __restrict__ B,
                                         int ldb, int nk, int lane, f32x4& c00, f32x4& c01, f32x4& c10,
                                         f32x4& c11) {
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const uint8_t* a0 = A + r * lda + kq;
  const uint8_t* a1 = a0 + 16 * lda;
  const uint8_t* b0 = B + r * ldb + kq;
  const uint8_t* b1 = b0 + 16 * ldb;
  long ra0[PF], ra1[PF], rb0[PF], rb1[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    if (j < nk) {
      ra0[j] = *reinterpret_cast<const long*>(a0 + j * 32);
      ra1[j] = *reinterpret_cast<const long*>(a1 + j * 32);
      rb0[j] = *reinterpret_cast<const long*>(b0 + j * 32);
      rb1[j] = *reinterpret_cast<const long*>(b1 + j * 32);
    }
  }
  for (int kb = 0; kb < nk; kb += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int ks = kb + j;
      if (ks < nk) {
        c00 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra0[j], rb0[j], c00, 0, 0, 0);
        c01 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra0[j], rb1[j], c01, 0, 0, 0);
        c10 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra1[j], rb0[j], c10, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra1[j], rb1[j], c11, 0, 0, 0);
        const int kn = (ks + PF) * 32;
        if (ks + PF < nk) {
          ra0[j] = *reinterpret_cast<const long*>(a0 + kn);
          ra1[j] = *reinterpret_cast<const long*>(a1 + kn);
          rb0[j] = *reinterpret_cast<const long*>(b0 + kn);
          rb1[j] = *reinterpret_cast<const long*>(b1 + kn);
        }
      }
    }
  }
}

// 8 bf16 LDS elements * q -> one fp8 A fragment (8 e4m3 bytes)
__device__ __forceinline__ long lds_to_fp8x8(const bf16* p, float q) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
  const uint32_t lo = pack4_fp8(bf2f(v[0]) * q, bf2f(v[1]) * q, bf2f(v[2]) * q, bf2f(v[3]) * q);
  const uint32_t hi = pack4_fp8(bf2f(v[4]) * q, bf2f(v[5]) * q, bf2f(v[6]) * q, bf2f(v[7]) * q);
  return (long)(((unsigned long)hi << 32) | lo);
}

// fp8 GEMM with the A operand quantized on the fly from a bf16 LDS tile (row r scaled by q[r])
__device__ __forceinline__ void mma32_f8_lds(const bf16* A, int lda, const float* q,
                                             const uint8_t* __restrict__ B, int ldb, int nk, int lane,
                                             f32x4& c00, f32x4& c01, f32x4& c10, f32x4& c11) {
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const bf16* a0 = A + r * lda + kq;
  const bf16* a1 = a0 + 16 * lda;
  const float q0 = q[r], q1 = q[r + 16];
  const uint8_t* b0 = B + r * ldb + kq;
  const uint8_t* b1 = b0 + 16 * ldb;
  for (int ks = 0; ks < nk; ++ks) {
    const long ra0 = lds_to_fp8x8(a0 + ks * 32, q0);
    const long ra1 = lds_to_fp8x8(a1 + ks * 32, q1);
    const long rb0 = *reinterpret_cast<const long*>(b0 + ks * 32);
    const long rb1 = *reinterpret_cast<const long*>(b1 + ks * 32);
    c00 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra0, rb0, c00, 0, 0, 0);
    c01 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra0, rb1, c01, 0, 0, 0);
    c10 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra1, rb0, c10, 0, 0, 0);
    c11 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(ra1, rb1, c11, 0, 0, 0);
  }
}

// Copy a [32 x N] bf16 LDS tile (row stride ld) to its transpose in global memory:
// out[c * M + row0 + r].  Each thread moves 8 consecutive rows of 4 adjacent columns: 8 LDS reads
// of 8 B and four 16-B stores (N % 4 == 0, ld % 4 == 0: every tile here has N % 32 == 0 and
// ld = N + 8) -- a quarter of the LDS read instructions of one column per thread (TW_TSTORE1:
// that form, for A/B).
__device__ __forceinline__ void store_tile_t(const bf16* t, int ld, int N, bf16* out, int M, int row0) {
  for (int e = threadIdx.x; e < N; e += blockDim.x) {   // N / 4 column quads x 4 row octets
    const int c = (e >> 2) * 4, r8 = (e & 3) * 8;
    bf16x8 v0, v1, v2, v3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x4 q = *reinterpret_cast<const bf16x4*>(t + (r8 + j) * ld + c);
      v0[j] = q[0];
      v1[j] = q[1];
      v2[j] = q[2];
      v3[j] = q[3];
    }
    bf16* o = out + (size_t)c * M + row0 + r8;
    *reinterpret_cast<bf16x8*>(o) = v0;
    *reinterpret_cast<bf16x8*>(o + M) = v1;
    *reinterpret_cast<bf16x8*>(o + 2 * (size_t)M) = v2;
    *reinterpret_cast<bf16x8*>(o + 3 * (size_t)M) = v3;
  }
}

// FM gather of one 32-sample block (K1): 8 threads per sample, each owning fields q, q+8, ...;
// E rows go to the bf16 LDS tile (and the fp8 tile), per-sample S / sum E^2 / y_w are summed in
// registers over the thread's fields, then over its 8 lanes (fixed xor order: deterministic).
struct TwNoHook {
  __device__ void operator()() const {}
};

// ``hook()`` runs once, right after the first pass's table-row loads are issued (their HBM round
// trip is the gather's longest wait: the tower issues its first GEMM's weight loads there)
template <bool FP8, int KE, int FMX = 0, class Hook = TwNoHook>
__device__ __forceinline__ void tower_gather(const TowerArgs& a, int row0, bf16* Xl, int ldx,
                                             uint8_t* X8, int ld8, float* s_yfm, float* s_dq0,
                                             float* gx = nullptr, float* gS = nullptr, Hook hook = Hook()) {
  constexpr int V4 = KE / 4;
  // fields per thread per pass, all loads in flight (Criteo: 39 <= 40); K = 32 rows are 8 f32x4
  // each, so fewer fields per pass keep the loads in registers
  // (3 per pass for K = 32 -- 2 dependent load rounds instead of 3 -- measured no faster on the
  // B = 1024 reference workload: 0.0981-0.0997 vs 0.0974-0.0979 ms/step, profiles/r4o_ref_ab.log)
  constexpr int FMAX = FMX ? FMX : (KE >= 32 ? 2 : 5);
  const int tid = threadIdx.x, sl = tid >> 3, q = tid & 7;
  const int b = row0 + sl, F = a.F;
  f32x4 S[V4], Q[V4];
#pragma unroll
  for (int j = 0; j < V4; ++j) S[j] = Q[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float yw = 0.f, am = 0.f;
  bf16* xr = Xl + sl * ldx;
  // the ids / values of a pass are loaded during the pass before (issued after its table-row
  // loads): a pass then waits one dependent round trip (the rows), not two (ids, then rows) --
  // K = 32 takes ceil(F / 16) passes
  int id[FMAX];
  float x[FMAX];
  auto load_ids = [&](int f0, int (&idv)[FMAX], float (&xv)[FMAX]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < FMAX; ++t) {
      const int f = f0 + 8 * t;
      idv[t] = f < F ? a.idx[a.idx_ld ? (size_t)f * a.idx_ld + b : (size_t)b * F + f] : 0;
      if (a.id_lim && (unsigned)idv[t] >= a.id_lim) idv[t] = (int)a.id_lim - 1;
      xv[t] = f < F ? a.vals[(size_t)b * F + f] : 0.f;
    }
  };
  load_ids(q, id, x);
  for (int f0 = q; f0 < F; f0 += 8 * FMAX) {
    f32x4 v[FMAX][V4];
    float w[FMAX];
#pragma unroll
    for (int t = 0; t < FMAX; ++t) {
      const bool ok = f0 + 8 * t < F;
      const float* row = a.tv + (size_t)id[t] * a.ldv;
#pragma unroll
      for (int j = 0; j < V4; ++j) v[t][j] = ok ? ld_row4(row, 4 * j, a.vbf16) : f32x4{0.f, 0.f, 0.f, 0.f};
      w[t] = ok ? a.tw[(size_t)id[t] * a.ldw] : 0.f;
    }
    int idn[FMAX];
    float xn[FMAX];
    const bool more = f0 + 8 * FMAX < F;   // (K <= 16 at Criteo's F: one pass)
    if (more) load_ids(f0 + 8 * FMAX, idn, xn);
    if (f0 == q) hook();
#pragma unroll
    for (int t = 0; t < FMAX; ++t) {
      const int f = f0 + 8 * t;
      if (f >= F) break;
      if (gx) gx[sl * F + f] = x[t];
      yw += w[t] * x[t];
#pragma unroll
      for (int j = 0; j < V4; ++j) {
        const f32x4 e = v[t][j] * x[t];
        S[j] += e;
        Q[j] += e * e;
        am = fmaxf(am, fmaxf(fmaxf(fabsf(e[0]), fabsf(e[1])), fmaxf(fabsf(e[2]), fabsf(e[3]))));
        bf16x4 eh = {f2bf(e[0]), f2bf(e[1]), f2bf(e[2]), f2bf(e[3])};
        *reinterpret_cast<bf16x4*>(xr + f * KE + 4 * j) = eh;
      }
    }
    if (more) {
#pragma unroll
      for (int t = 0; t < FMAX; ++t) {
        id[t] = idn[t];
        x[t] = xn[t];
      }
    }
  }
  // zero the padding columns [F*K, K0p) of the row
  for (int c = F * KE + q; c < a.K0p; c += 8) xr[c] = f2bf(0.f);
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
#pragma unroll
    for (int j = 0; j < V4; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        S[j][c] += __shfl_xor(S[j][c], o, 64);
        Q[j][c] += __shfl_xor(Q[j][c], o, 64);
      }
    yw += __shfl_xor(yw, o, 64);
    am = fmaxf(am, __shfl_xor(am, o, 64));
  }
  float yv = 0.f;
#pragma unroll
  for (int j = 0; j < V4; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) yv += S[j][c] * S[j][c] - Q[j][c];
  if (q == 0) {
    s_yfm[sl] = a.fm_bias[0] + yw + 0.5f * yv;
    if (a.S) {
#pragma unroll
      for (int j = 0; j < V4; ++j) *reinterpret_cast<f32x4*>(a.S + (size_t)b * KE + 4 * j) = S[j];
    }
    if (gS) {
#pragma unroll
      for (int j = 0; j < V4; ++j) *reinterpret_cast<f32x4*>(gS + sl * KE + 4 * j) = S[j];
    }
  }
  if (FP8) {  // per-row power-of-two scale of the fp8 layer-0 operand (current scaling)
    const float qs = fp8_pow2_scale(am);
    if (q == 0) s_dq0[sl] = 1.f / qs;
    __syncthreads();  // the bf16 row is complete
    uint8_t* r8 = X8 + sl * ld8;
    for (int c4 = q; c4 < a.K0p / 4; c4 += 8) {
      const bf16* e = xr + 4 * c4;
      *reinterpret_cast<uint32_t*>(r8 + 4 * c4) =
          pack4_fp8(bf2f(e[0]) * qs, bf2f(e[1]) * qs, bf2f(e[2]) * qs, bf2f(e[3]) * qs);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Split gather + layer 0 (a.l0s slices): block (rb, s) gathers rows [32 rb, 32 rb + 32) x the
// fields of k-steps [s l0_ks, (s + 1) l0_ks) into an LDS tile, stores those E^T columns (train),
// and writes its partial FM sums and its partial layer-0 pre-activation tile (one 32 x 32 MFMA
// tile per wave and column tile, the slice's k-steps in order).  KE divides 32, so a k-step holds
// whole fields.
template <int KE>
__global__ void __launch_bounds__(256) tower_l0s_kernel(TowerArgs a) {
  extern __shared__ __align__(16) unsigned char tw_lds_raw[];
  bf16* Xs = reinterpret_cast<bf16*>(tw_lds_raw);
  constexpr int V4 = KE / 4;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int sl = tid >> 3, q = tid & 7;
  const int row0 = blockIdx.x * TW_ROWS, s = blockIdx.y, F = a.F;
  const int T = a.K0p / 32;
  const int ks0 = s * a.l0_ks, nk = min(a.l0_ks, T - ks0);
  if (nk <= 0) return;
  const int c0 = ks0 * 32, ncol = nk * 32, ldx = ncol + 8;
  const int f_lo = c0 / KE, f_hi = min(F, (c0 + ncol) / KE);
  const int b = row0 + sl;
  bf16* xr = Xs + sl * ldx;
  f32x4 S[V4];
#pragma unroll
  for (int j = 0; j < V4; ++j) S[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float Q = 0.f, yw = 0.f;
  // up to FPS fields per thread per pass, every id, then every row in flight at once
  constexpr int FPS = KE >= 32 ? 2 : 4;
  for (int f0 = f_lo + q; f0 < f_hi; f0 += 8 * FPS) {
    int id[FPS];
    float x[FPS];
#pragma unroll
    for (int t = 0; t < FPS; ++t) {
      const int f = f0 + 8 * t;
      id[t] = f < f_hi ? a.idx[a.idx_ld ? (size_t)f * a.idx_ld + b : (size_t)b * F + f] : 0;
      if (a.id_lim && (unsigned)id[t] >= a.id_lim) id[t] = (int)a.id_lim - 1;
      x[t] = f < f_hi ? a.vals[(size_t)b * F + f] : 0.f;
    }
    f32x4 v[FPS][V4];
    float w[FPS];
#pragma unroll
    for (int t = 0; t < FPS; ++t) {
      const bool ok = f0 + 8 * t < f_hi;
      const float* row = a.tv + (size_t)id[t] * a.ldv;
#pragma unroll
      for (int j = 0; j < V4; ++j) v[t][j] = ok ? ld_row4(row, 4 * j, a.vbf16) : f32x4{0.f, 0.f, 0.f, 0.f};
      w[t] = ok ? a.tw[(size_t)id[t] * a.ldw] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < FPS; ++t) {
      const int f = f0 + 8 * t;
      if (f >= f_hi) break;
      yw += w[t] * x[t];
#pragma unroll
      for (int j = 0; j < V4; ++j) {
        const f32x4 e = v[t][j] * x[t];
        S[j] += e;
        Q += (e[0] * e[0] + e[1] * e[1]) + (e[2] * e[2] + e[3] * e[3]);
        bf16x4 eh = {f2bf(e[0]), f2bf(e[1]), f2bf(e[2]), f2bf(e[3])};
        *reinterpret_cast<bf16x4*>(xr + f * KE - c0 + 4 * j) = eh;
      }
    }
  }
  for (int c = max(F * KE - c0, 0) + q; c < ncol; c += 8) xr[c] = f2bf(0.f);   // padding columns
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
#pragma unroll
    for (int j = 0; j < V4; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) S[j][c] += __shfl_xor(S[j][c], o, 64);
    Q += __shfl_xor(Q, o, 64);
    yw += __shfl_xor(yw, o, 64);
  }
  if (q == 0) {
    float* fm = a.l0fm + ((size_t)s * a.M + b) * (KE + 2);
#pragma unroll
    for (int j = 0; j < V4; ++j) *reinterpret_cast<f32x4*>(fm + 4 * j) = S[j];
    fm[KE] = Q;
    fm[KE + 1] = yw;
  }
  __syncthreads();
  if (a.train) store_tile_t(Xs, ldx, ncol, a.Et + (size_t)c0 * a.M, a.M, row0);
  const int N0 = a.Np[0], cr = (lane >> 4) * 4, cc = lane & 15;
  for (int ct = wave; ct < N0 / 32; ct += 4) {
    f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
    mma32<2>(Xs, ldx, a.W[0] + (size_t)ct * 32 * a.K0p + c0, a.K0p, nk, lane, c00, c01, c10, c11);
    const f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
    float* z = a.l0z + ((size_t)s * a.M + row0) * N0 + ct * 32;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int j = 0; j < 4; ++j) z[(size_t)(ti * 16 + cr + j) * N0 + tj * 16 + cc] = acc[ti][tj][j];
  }
}

// The tower's side of the split: y_fm, S (and the grow scratch's S) from the slices' FM partials,
// summed in slice order (8 threads per row, as the gather's lanes).  Every partial is loaded before
// the first add (one round trip, not one per slice).
constexpr int TW_L0S_MAX = 8;
template <int KE>
__device__ __forceinline__ void tower_l0s_fm(const TowerArgs& a, int row0, float* s_yfm, float* gS) {
  constexpr int KQ = (KE + 7) / 8;   // components per thread
  const int tid = threadIdx.x, sl = tid >> 3, q = tid & 7, b = row0 + sl;
  float part[TW_L0S_MAX][KQ], pq[TW_L0S_MAX], pw[TW_L0S_MAX];
#pragma unroll
  for (int s = 0; s < TW_L0S_MAX; ++s) {
    const float* fm = a.l0fm + ((size_t)s * a.M + b) * (KE + 2);
#pragma unroll
    for (int t = 0; t < KQ; ++t) part[s][t] = (s < a.l0s && q + 8 * t < KE) ? fm[q + 8 * t] : 0.f;
    pq[s] = (s < a.l0s && q == 0) ? fm[KE] : 0.f;
    pw[s] = (s < a.l0s && q == 0) ? fm[KE + 1] : 0.f;
  }
  float yv = 0.f, Q = 0.f, yw = 0.f;
#pragma unroll
  for (int t = 0; t < KQ; ++t) {
    float sk = 0.f;
#pragma unroll
    for (int s = 0; s < TW_L0S_MAX; ++s)
      if (s < a.l0s) sk += part[s][t];
    const int k = q + 8 * t;
    if (k < KE) {
      yv += sk * sk;
      if (a.S) a.S[(size_t)b * KE + k] = sk;
      if (gS) gS[sl * KE + k] = sk;
    }
  }
#pragma unroll
  for (int s = 0; s < TW_L0S_MAX; ++s)
    if (s < a.l0s) {
      Q += pq[s];
      yw += pw[s];
    }
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) yv += __shfl_xor(yv, o, 64);
  if (q == 0) s_yfm[sl] = a.fm_bias[0] + yw + 0.5f * (yv - Q);
}

// one wave's 32 x 32 layer-0 pre-activation tile from the slices' partials, in slice order: the
// loads of 4 slices (64 registers: the layer-0 B-fragment ring is idle in this mode) per round
__device__ __forceinline__ void tower_l0s_tile(const TowerArgs& a, int row0, int N, int ct, int lane,
                                               f32x4& c00, f32x4& c01, f32x4& c10, f32x4& c11) {
  const int cr = (lane >> 4) * 4, cc = lane & 15;
  f32x4* cs[2][2] = {{&c00, &c01}, {&c10, &c11}};
  for (int s0 = 0; s0 < a.l0s; s0 += 4) {
    float v[4][2][2][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* z = a.l0z + ((size_t)(s0 + u) * a.M + row0) * N + ct * 32;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[u][ti][tj][j] = s0 + u < a.l0s ? z[(size_t)(ti * 16 + cr + j) * N + tj * 16 + cc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (s0 + u < a.l0s)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int j = 0; j < 4; ++j) (*cs[ti][tj])[j] += v[u][ti][tj][j];
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 tower body (everything after the serve / stamp workgroup split).  Same math, same outputs,
// bit for bit, as the generic body below; the difference is WHEN operands arrive: every GEMM
// tile's weight fragments (and the forward bias, the head's w_out / labels) are loaded one phase
// ahead -- the first tile's during the FM gather -- so no phase starts with an L2 round trip.
// Phases: fwd 0..nl-1, dgrad nl-1..1, dX0 (tile ct of phase ph: tw_phase_b).
// primed k-steps: K0p / 32 = 10 for Criteo at K = 8 (layer 0 entirely on registers); K = 32 rings
// through 6 (two waves / SIMD need <= 256 registers)
__host__ __device__ constexpr int tw_np(int KE) { return KE >= 16 ? 6 : (KE == 0 ? 4 : 10); }
constexpr int TW_HQ = 8;   // head w_out values prefetched per thread (L / 8 <= 8)

__device__ __forceinline__ int tw_nphase(const TowerArgs& a) { return a.train ? 2 * a.nl - (a.dx0_split ? 1 : 0) : a.nl; }

// B operand / row stride / k-steps / tiles of phase ph (tile ct)
struct TwPhase {
  const bf16* B;
  int ld, nk, ntile;
};
__device__ __forceinline__ TwPhase tw_phase_b(const TowerArgs& a, int ph, int ct) {
  const int nl = a.nl;
  TwPhase r;
  if (ph < nl) {  // forward layer ph: H_ph = X W_ph^T
    r.ld = ph == 0 ? a.K0p : a.Np[ph - 1];
    r.ntile = a.Np[ph] / 32;
    r.nk = r.ld / 32;
    r.B = a.W[ph] + (size_t)ct * 32 * r.ld;
    return r;
  }
  const int i = 2 * nl - 1 - ph;  // dgrad i (nl-1 .. 1), then dX0 (i = 0)
  r.ld = a.Np[i];
  r.nk = r.ld / 32;
  r.ntile = i > 0 ? a.Np[i - 1] / 32 : a.K0p / 32;
  r.B = a.WT[i] + (size_t)ct * 32 * r.ld;
  return r;
}

// One dX0 tile (32 rows x 32 columns = 32 / K fields) -> the sorted gradient rows of its slots:
// bf16-rounded dX0 (the values the unsorted path stores) staged in the wave's own LDS tile, then
// a = x (dx + dy S), g_w, c per slot (sf_slot_*), written to grow[inv[slot]].  Wave-local: only
// this wave reads its tile.
template <int KE>
__device__ __forceinline__ void tw_grow_tile(const TowerArgs& a, const f32x4 (&acc)[2][2], int ct, int row0, int lane,
                                             bf16* wt, const float* gx, const float* gS, const int* ginv,
                                             const float* s_dl) {
  constexpr int FPT = 32 / KE, LPS = KE / 4, RS = grow_stride(KE);
  const int cr = (lane >> 4) * 4, cc = lane & 15, F = a.F;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int j = 0; j < 4; ++j) wt[(ti * 16 + cr + j) * 40 + tj * 16 + cc] = f2bf(acc[ti][tj][j]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int t = lane + 64 * k;
    const int sub = t % LPS, sl = t / LPS;
    const int row = sl / FPT, fl = sl - row * FPT;
    const int f = ct * FPT + fl;
    if (f < F) {
      const bf16x4 dxh = *reinterpret_cast<const bf16x4*>(wt + row * 40 + fl * KE + sub * 4);
      const f32x4 dx = {bf2f(dxh[0]), bf2f(dxh[1]), bf2f(dxh[2]), bf2f(dxh[3])};
      const f32x4 s = *reinterpret_cast<const f32x4*>(gS + row * KE + sub * 4);
      const float x = gx[row * F + f], dy = s_dl[row];
      const int pos = !a.inv ? (row0 + row) * F + f
                             : ginv ? ginv[f * 32 + row] : a.inv[(size_t)f * a.inv_ld + row0 + row];
      float* gr = a.grow + (size_t)pos * RS;
      *reinterpret_cast<f32x4a8*>(gr + sub * 4) = sf_slot_a(dx, dy, s, x);
      if (sub == 0) *reinterpret_cast<f32x2a8*>(gr + KE) = f32x2a8{sf_slot_gw(dy, x), sf_slot_c(dy, x)};
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One dX0 tile (32 rows x 32 columns) -> dX0 in HBM through the wave's LDS tile: each lane stores
// 2 x 16 B of contiguous row data instead of 16 scattered 2-B values (the dX0 phase of a K = 32
// tower, whose rows go to HBM, measured 15 us of its 51: r4j reference-workload stamps)
__device__ __forceinline__ void tw_dx0_tile(const TowerArgs& a, const f32x4 (&acc)[2][2], int ct, int row0, int lane,
                                            bf16* wt) {
  const int cr = (lane >> 4) * 4, cc = lane & 15;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int j = 0; j < 4; ++j) wt[(ti * 16 + cr + j) * 40 + tj * 16 + cc] = f2bf(acc[ti][tj][j]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = lane + 64 * k, row = q >> 2, part = q & 3;   // 32 rows x 4 chunks of 8 bf16
    const uint4 v = *reinterpret_cast<const uint4*>(wt + row * 40 + part * 8);
    *reinterpret_cast<uint4*>(a.dX0 + (size_t)(row0 + row) * a.K0p + ct * 32 + part * 8) = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LIGHT: a 2-deep ring instead of the primed layer-0 / dX0 weights -- a launch that carries serve
// workgroups (run-routed row-sharded step) keeps the register count low enough for them to
// co-reside with two tower workgroups per CU (240 registers left them queued behind the tower:
// 68.7 vs 47.3 us)
template <int KE, bool LIGHT, bool L0S = false>
__device__ __forceinline__ void tower_bf16_body(const TowerArgs& a, bf16* lds, float* s_dl, float* s_loss,
                                                float* s_yfm) {
  constexpr int TW_NP = LIGHT ? 2 : tw_np(KE);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * TW_ROWS;
  const int cr = (lane >> 4) * 4, cc = lane & 15;
  const int nl = a.nl, nph = tw_nphase(a);
  bf16x8 pb0[TW_NP], pb1[TW_NP];
  float pbias0 = 0.f, pbias1 = 0.f;
  // prime the B fragments of (phase ph, tile ct) if that tile exists
  auto prime = [&](int ph, int ct) __attribute__((always_inline)) {
    if (ph >= nph) return;
    const TwPhase q = tw_phase_b(a, ph, ct);
    if (ct >= q.ntile) return;
    bfrag_prime<TW_NP>(pb0, pb1, q.B, q.ld, q.nk, lane);
    if (ph < nl) {
      pbias0 = a.bias[ph][ct * 32 + cc];
      pbias1 = a.bias[ph][ct * 32 + 16 + cc];
    }
  };
  const uint32_t step = (uint32_t)(*a.step);
  const int L = a.Np[nl - 1];
  const int hrow = tid >> 3, hq = tid & 7, Q = L / 8;
  const int ldx = a.K0p + 8;
  bf16* Xl = lds + (KE > 0 ? a.x_off : 0);
  // sorted gradient rows: LDS scratch and this block's inverse permutation (prefetched now)
  // (with dx0_split the dX0 launch writes the gradient rows: the tower runs its plain layout)
  const bool grow = KE > 0 && a.train && a.grow != nullptr && !a.dx0_split;
  // sorted positions (else rows in slot order); LIGHT reads them from global in the dX0 phase
  // instead of staging this block's share in LDS (registers held across the dgrad chain)
  const bool ginv_on = grow && a.inv != nullptr && !LIGHT;
  float* gx = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(lds) + (grow ? a.g_off : 0));
  float* gS = gx + TW_ROWS * a.F;
  int* ginv = reinterpret_cast<int*>(gS + TW_ROWS * (KE > 0 ? KE : 1));
  // the 4 wave tiles of the dX0 phase live in the H tiles' region (dead by then) when it is large
  // enough: the launch's LDS stays small enough for serve / stamp workgroups to co-reside
  int hbytes = 0;
  for (int i = 0; i < nl; ++i) hbytes += 2 * TW_ROWS * (a.Np[i] + 8);
  bf16* gwt = (hbytes >= 4 * TW_ROWS * 40 * 2 ? lds + a.h_off[0] : reinterpret_cast<bf16*>(ginv + TW_ROWS * a.F)) +
              wave * TW_ROWS * 40;
  int ivr[TW_GINV];
  if constexpr (KE > 0) {
    // (weights primed DURING the gather slowed it more than they saved: its table-row loads
    // compete with them for the same address path)
    if constexpr (L0S)   // gather + layer 0 done by tower_l0s_kernel: sum its FM partials
      tower_l0s_fm<KE>(a, row0, s_yfm, grow ? gS : nullptr);
    else
      tower_gather<false, KE, (LIGHT && KE >= 32) ? 2 : 0>(a, row0, Xl, ldx, nullptr, 0, s_yfm, nullptr,
                                                           grow ? gx : nullptr, grow ? gS : nullptr);
    __syncthreads();
    TW_ST(1);
  }
  // the head's operands, then (behind the E^T stores in the memory queue) the first GEMM tile's
  // weights
  float wo[TW_HQ];
  if (!LIGHT) {
#pragma unroll
    for (int j = 0; j < TW_HQ; ++j) wo[j] = j < Q ? a.w_out[hq * Q + j] : 0.f;
  }
  const float bout = a.b_out[0];
  const bool hvalid = a.labels && row0 + hrow < a.nvalid;
  const float hlab = hvalid ? a.labels[row0 + hrow] : 0.f;
  const float yfm_g = KE > 0 ? 0.f : a.y_fm[row0 + hrow];
  if constexpr (KE > 0) {
    if constexpr (!L0S) {
      if (a.train) store_tile_t(Xl, ldx, a.K0p, a.Et, a.M, row0);
      prime(0, wave);
    }
    TW_ST(2);
  }
  // ---------------------------------------------------------------- forward
  for (int i = 0; i < nl; ++i) {
    const int N = a.Np[i];
    const int Kp = i == 0 ? a.K0p : a.Np[i - 1];
    const int ldh = N + 8;
    bf16* Hl = lds + a.h_off[i];
    const bool drop = a.train && a.drop[i];
    const uint32_t salt = drop ? dropout_salt(a.seed, step, (uint32_t)i) : 0u;
    const float sc = a.inv_keep[i];
    const bf16* Asrc = i == 0 ? (KE > 0 ? Xl : nullptr) : lds + a.h_off[i - 1];
    const int lda = i == 0 ? ldx : Kp + 8;
    for (int ct = wave; ct < N / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      float bc[2];
      if (L0S && i == 0) {   // the slices' partial pre-activations, in slice order
        tower_l0s_tile(a, row0, N, ct, lane, c00, c01, c10, c11);
      } else if (KE == 0 && i == 0) {
        mma32<TW_NP>(a.E + (size_t)row0 * a.K0p, a.K0p, a.W[0] + (size_t)ct * 32 * Kp, Kp, Kp / 32, lane, c00,
                     c01, c10, c11);
      } else if (i == 0) {  // layer 0 (the longest reduction): weights primed one tile ahead
        mma32_primed<TW_NP>(Asrc, lda, a.W[0] + (size_t)ct * 32 * Kp, Kp, Kp / 32, lane, pb0, pb1, c00, c01,
                            c10, c11);
        bc[0] = pbias0;
        bc[1] = pbias1;
        if (ct + 4 < N / 32) prime(0, ct + 4);
      } else {
        // (priming the short layers' weights measured no faster: 2-4 k-steps, one L2 trip)
        mma32<2>(Asrc, lda, a.W[i] + (size_t)ct * 32 * Kp, Kp, Kp / 32, lane, c00, c01, c10, c11);
      }
      if (KE == 0 || i > 0 || L0S) {
        bc[0] = a.bias[i][ct * 32 + cc];
        bc[1] = a.bias[i][ct * 32 + 16 + cc];
      }
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = ti * 16 + cr + j;
            float v = fmaxf(acc[ti][tj][j] + bc[tj], 0.f);
            if (drop)
              v = dropout_keep((uint32_t)((row0 + row) * N + col), salt, a.keep_thr[i]) ? v * sc : 0.f;
            Hl[row * ldh + col] = f2bf(v);
          }
        }
      }
    }
    __syncthreads();
    TW_ST(3 + i);
    if (a.train && a.Ht[i]) store_tile_t(Hl, ldh, N, a.Ht[i], a.M, row0);
  }
  // ---------------------------------------------------------------- head
  {
    const bf16* H = lds + a.h_off[nl - 1];
    const int ldh = L + 8;
    const int grow = row0 + hrow;
    float yd = 0.f;
#pragma unroll
    for (int j = 0; j < TW_HQ; ++j)
      if (j < Q) yd += bf2f(H[hrow * ldh + hq * Q + j]) * (LIGHT ? a.w_out[hq * Q + j] : wo[j]);
    for (int j = TW_HQ; j < Q; ++j) yd += bf2f(H[hrow * ldh + hq * Q + j]) * a.w_out[hq * Q + j];
    yd += __shfl_xor(yd, 1, 64);
    yd += __shfl_xor(yd, 2, 64);
    yd += __shfl_xor(yd, 4, 64);
    const float y = (KE > 0 ? s_yfm[hrow] : yfm_g) + yd + bout;
    const float p = 1.f / (1.f + __expf(-y));
    float dl = 0.f, lossb = 0.f;
    if (hvalid) {
      if (a.square_loss) {
        lossb = (p - hlab) * (p - hlab);
        dl = 2.f * (p - hlab) * p * (1.f - p) * a.gscale;
      } else {
        lossb = fmaxf(y, 0.f) - y * hlab + log1pf(__expf(-fabsf(y)));
        dl = (p - hlab) * a.gscale;
      }
    }
    if (hq == 0) {
      if (KE > 0) a.y_fm[grow] = s_yfm[hrow];
      a.prob[grow] = p;
      s_dl[hrow] = dl;
      s_loss[hrow] = lossb;
      if (a.train) a.dlogit[grow] = dl;
    }
    if (a.train) {
      bf16* Z = lds + a.dz_off[0];
      const int ldz = L + 8;
      const float sl = a.inv_keep[nl - 1];
#pragma unroll
      for (int j = 0; j < TW_HQ; ++j) {
        if (j < Q) {
          const int col = hq * Q + j;
          const float g = bf2f(H[hrow * ldh + col]) > 0.f ? dl * (LIGHT ? a.w_out[col] : wo[j]) * sl : 0.f;
          Z[hrow * ldz + col] = f2bf(g);
        }
      }
      for (int j = TW_HQ; j < Q; ++j) {
        const int col = hq * Q + j;
        const float g = bf2f(H[hrow * ldh + col]) > 0.f ? dl * a.w_out[col] * sl : 0.f;
        Z[hrow * ldz + col] = f2bf(g);
      }
    }
    __syncthreads();
    float* part = a.partial + (size_t)blockIdx.x * (L + 2);
    for (int c = tid; c < L + 2; c += blockDim.x) {
      float s = 0.f;
      if (c < L) {
        if (a.train)
          for (int r = 0; r < TW_ROWS; ++r) s += s_dl[r] * bf2f(H[r * ldh + c]);
      } else if (c == L) {
        for (int r = 0; r < TW_ROWS; ++r) s += s_dl[r];
      } else {
        for (int r = 0; r < TW_ROWS; ++r) s += s_loss[r];
      }
      part[c] = s;
    }
  }
  TW_ST(7);
  if (!a.train) return;
  store_tile_t(lds + a.dz_off[0], L + 8, L, a.dZt[nl - 1], a.M, row0);
  TW_ST(8);
  // ---------------------------------------------------------------- dgrad chain
  if (ginv_on) {  // this block's inverse permutation, for the dX0 phase's sorted rows
#pragma unroll
    for (int k = 0; k < TW_GINV; ++k) {  // block entry e = f * 32 + r (32 contiguous ints per field)
      const int e = tid + 256 * k;
      ivr[k] = e < TW_ROWS * a.F ? a.inv[(size_t)(e / TW_ROWS) * a.inv_ld + row0 + (e % TW_ROWS)] : 0;
    }
  }
  if (nl == 1) prime(1, wave);
  int cur = 0;
  for (int i = nl - 1; i >= 1; --i) {
    const int ph = 2 * nl - 1 - i;
    const int Nout = a.Np[i - 1], Kin = a.Np[i];
    const bf16* Az = lds + a.dz_off[cur];
    bf16* Zo = lds + a.dz_off[cur ^ 1];
    const bf16* Hp = lds + a.h_off[i - 1];
    const int ldh = Nout + 8, ldz_in = Kin + 8, ldz_out = Nout + 8;
    const float sc = a.inv_keep[i - 1];
    for (int ct = wave; ct < Nout / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      mma32<2>(Az, ldz_in, a.WT[i] + (size_t)ct * 32 * Kin, Kin, Kin / 32, lane, c00, c01, c10, c11);
      if (i == 1) prime(ph + 1, wave);  // dX0's first tile: its weights while this epilogue runs
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = ti * 16 + cr + j;
            const float v = bf2f(Hp[row * ldh + col]) > 0.f ? acc[ti][tj][j] * sc : 0.f;
            Zo[row * ldz_out + col] = f2bf(v);
          }
        }
      }
    }
    if (i == 1 && wave >= Nout / 32) prime(ph + 1, wave);
    __syncthreads();
    TW_ST(8 + 2 * (nl - i) - 1);
    store_tile_t(Zo, ldz_out, Nout, a.dZt[i - 1], a.M, row0);
    TW_ST(8 + 2 * (nl - i));
    cur ^= 1;
  }
  if (a.dx0_split) {  // dX0 from dZ_0^T by tower_dx0_kernel
    TW_ST(15);
    return;
  }
  {
    const int N0 = a.Np[0];
    const bf16* Az = lds + a.dz_off[cur];
    const int ph = 2 * nl - 1;
    if (ginv_on) {
#pragma unroll
      for (int k = 0; k < TW_GINV; ++k) {
        const int e = tid + 256 * k;
        if (e < TW_ROWS * a.F) ginv[e] = ivr[k];
      }
      __syncthreads();
    } else if (nl == 1) {
      // one hidden layer: no dgrad chain (and its barriers) since the head's partial sums read
      // H_0, and the dX0 wave tiles (gwt) may live in that region -- wait for every reader
      __syncthreads();
    }
    for (int ct = wave; ct < a.K0p / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      mma32_primed<TW_NP>(Az, N0 + 8, a.WT[0] + (size_t)ct * 32 * N0, N0, N0 / 32, lane, pb0, pb1, c00, c01,
                          c10, c11);
      if (ct + 4 < a.K0p / 32) prime(ph, ct + 4);
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
      if (grow) {
        if constexpr (KE > 0) tw_grow_tile<KE>(a, acc, ct, row0, lane, gwt, gx, gS, ginv_on ? ginv : nullptr, s_dl);
        continue;
      }
      if (hbytes >= 4 * TW_ROWS * 40 * 2) {   // (the dead H region holds the 4 wave tiles)
        tw_dx0_tile(a, acc, ct, row0, lane, gwt);
        continue;
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int rl = ti * 16 + cr + j;
            a.dX0[(size_t)(row0 + rl) * a.K0p + col] = f2bf(acc[ti][tj][j]);
          }
        }
      }
    }
  }
  TW_ST(15);
}

template <int KE>
__device__ __forceinline__ bool tower_aux_wg(const TowerArgs& a) {
  // the workgroups after the tower's blocks: serve (run-routed sharded step) or stamp (tf1_dense)
  const int tid = threadIdx.x;
  const int sb = (int)blockIdx.x - a.M / TW_ROWS;
  if (sb < 0) return false;
  if (sb < a.serve_wgs) {
    if (a.sv.rows) sh_serve_elem<KE>(a.sv, sb * 256 + tid);
    else sh_tag_elem(a.sv, sb * 256 + tid);
    return true;
  }
  const int i0 = (sb - a.serve_wgs) * 256 * TW_STAMP_EPT + tid;
#pragma unroll
  for (int k = 0; k < TW_STAMP_EPT; ++k) {
    const int i = i0 + k * 256;
    if (i < a.stamp_n) {
      const int key = a.stamp_keys[i];
      if (i == 0 || a.stamp_keys[i - 1] != key) a.stamp_flags[key / a.stamp_div] = 1;
    }
  }
  return true;
}

// the run-routed sharded step's launch (tower blocks + serve workgroups): LIGHT body, and the
// register budget of three workgroups per CU, so the serve workgroups share the CUs with the
// tower's blocks instead of waiting for them
template <int KE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3)))
tower_light_kernel(TowerArgs a) {
  extern __shared__ __align__(16) unsigned char tw_lds_raw[];
  __shared__ float s_dl[TW_ROWS];
  __shared__ float s_loss[TW_ROWS];
  __shared__ float s_yfm[TW_ROWS];
  if (tower_aux_wg<KE>(a)) return;
  TW_ST(0);
  tower_bf16_body<KE, true>(a, reinterpret_cast<bf16*>(tw_lds_raw), s_dl, s_loss, s_yfm);
}

// the tower after tower_l0s_kernel (split gather + layer 0): its own instantiation, so the
// partial sums' registers never count against the default towers' occupancy
template <int KE>
__global__ void __launch_bounds__(256) tower_l0s_tower_kernel(TowerArgs a) {
  extern __shared__ __align__(16) unsigned char tw_lds_raw[];
  __shared__ float s_dl[TW_ROWS];
  __shared__ float s_loss[TW_ROWS];
  __shared__ float s_yfm[TW_ROWS];
  if (tower_aux_wg<KE>(a)) return;
  TW_ST(0);
  tower_bf16_body<KE, false, true>(a, reinterpret_cast<bf16*>(tw_lds_raw), s_dl, s_loss, s_yfm);
}

template <bool FP8, int KE, int TW_PF0, int TW_PF1>
__global__ void __launch_bounds__(256) tower_kernel(TowerArgs a) {
  extern __shared__ __align__(16) unsigned char tw_lds_raw[];
  bf16* lds = reinterpret_cast<bf16*>(tw_lds_raw);
  __shared__ float s_dl[TW_ROWS];
  __shared__ float s_loss[TW_ROWS];
  __shared__ float s_q[TW_ROWS];   // fp8: quantization scales of the current H rows
  __shared__ float s_dq[TW_ROWS];  //      and their inverses
  __shared__ float s_yfm[TW_ROWS];  // gather: y_b + y_w + y_v per sample
  __shared__ float s_dq0[TW_ROWS];  // gather + fp8: dequant factors of the E rows
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if constexpr (KE > 0) {
    const int sb = (int)blockIdx.x - a.M / TW_ROWS;
    if (sb >= 0) {
      if (sb < a.serve_wgs) {  // a serve workgroup (run-routed sharded step) or a tag one (replicated)
        if (a.sv.rows) sh_serve_elem<KE>(a.sv, sb * 256 + tid);
        else sh_tag_elem(a.sv, sb * 256 + tid);
        return;
      }
      const int i0 = (sb - a.serve_wgs) * 256 * TW_STAMP_EPT + tid;  // a stamp workgroup
#pragma unroll
      for (int k = 0; k < TW_STAMP_EPT; ++k) {
        const int i = i0 + k * 256;
        if (i < a.stamp_n) {
          const int key = a.stamp_keys[i];
          if (i == 0 || a.stamp_keys[i - 1] != key) a.stamp_flags[key / a.stamp_div] = 1;
        }
      }
      return;
    }
  }
  const int row0 = blockIdx.x * TW_ROWS;
  TW_ST(0);
  if constexpr (!FP8) {
    tower_bf16_body<KE, false>(a, lds, s_dl, s_loss, s_yfm);
    return;
  }
  const int cr = (lane >> 4) * 4, cc = lane & 15;
  const uint32_t step = (uint32_t)(*a.step);
  const int nl = a.nl;
  const int ldx = a.K0p + 8, ld8 = a.K0p + 16;
  bf16* Xl = lds + (KE > 0 ? a.x_off : 0);
  uint8_t* X8 = tw_lds_raw + (KE > 0 && FP8 ? a.x8_off : 0);

  // ------------------------------------------------------------------ gather (K1)
  if constexpr (KE > 0) {
    tower_gather<FP8, KE>(a, row0, Xl, ldx, X8, ld8, s_yfm, s_dq0);
    __syncthreads();
    TW_ST(1);
    if (a.train) store_tile_t(Xl, ldx, a.K0p, a.Et, a.M, row0);
    TW_ST(2);
  }

  // ------------------------------------------------------------------ forward
  for (int i = 0; i < nl; ++i) {
    const int N = a.Np[i];
    const int Kp = i == 0 ? a.K0p : a.Np[i - 1];
    const int ldh = N + 8;
    bf16* Hl = lds + a.h_off[i];
    const bool drop = a.train && a.drop[i];
    const uint32_t salt = drop ? dropout_salt(a.seed, step, (uint32_t)i) : 0u;
    const float sc = a.inv_keep[i];
    for (int ct = wave; ct < N / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      if (FP8) {
        const uint8_t* Bw8 = a.W8[i] + (size_t)ct * 32 * Kp;
        if (i == 0 && KE > 0)
          mma32_f8<4>(X8, ld8, Bw8, Kp, Kp / 32, lane, c00, c01, c10, c11);
        else if (i == 0)
          mma32_f8<4>(a.E8 + (size_t)row0 * a.K0p, a.K0p, Bw8, Kp, Kp / 32, lane, c00, c01, c10, c11);
        else if (KE > 0)  // H_{i-1} quantized once into the (dead) fp8 E tile below
          mma32_f8<4>(X8, Kp + 16, Bw8, Kp, Kp / 32, lane, c00, c01, c10, c11);
        else
          mma32_f8_lds(lds + a.h_off[i - 1], Kp + 8, s_q, Bw8, Kp, Kp / 32, lane, c00, c01, c10, c11);
      } else {
        const bf16* Bw = a.W[i] + (size_t)ct * 32 * Kp;
        if (i == 0 && KE > 0)
          mma32<TW_PF0>(Xl, ldx, Bw, Kp, Kp / 32, lane, c00, c01, c10, c11);
        else if (i == 0)
          mma32<TW_PF0>(a.E + (size_t)row0 * a.K0p, a.K0p, Bw, Kp, Kp / 32, lane, c00, c01, c10, c11);
        else
          mma32<TW_PF1>(lds + a.h_off[i - 1], Kp + 8, Bw, Kp, Kp / 32, lane, c00, c01, c10, c11);
      }
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
          const float bc = a.bias[i][col];
          const float dqc = FP8 ? a.sW[i][col] : 1.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = ti * 16 + cr + j;
            const float dq = FP8 ? dqc * (i == 0 ? (KE > 0 ? s_dq0[row] : a.sE[row0 + row]) : s_dq[row]) : 1.f;
            float v = fmaxf(acc[ti][tj][j] * dq + bc, 0.f);
            if (drop)
              v = dropout_keep((uint32_t)((row0 + row) * N + col), salt, a.keep_thr[i]) ? v * sc : 0.f;
            Hl[row * ldh + col] = f2bf(v);
          }
        }
      }
    }
    __syncthreads();
    TW_ST(3 + i);
    if (a.train && a.Ht[i]) store_tile_t(Hl, ldh, N, a.Ht[i], a.M, row0);
    if (FP8 && i + 1 < nl) {  // per-row scales of H_i, the next layer's fp8 A operand
      const int r = tid >> 3, q8 = tid & 7;
      float m = 0.f;
      for (int c = q8; c < N; c += 8) m = fmaxf(m, fabsf(bf2f(Hl[r * ldh + c])));
      m = fmaxf(m, __shfl_xor(m, 1, 64));
      m = fmaxf(m, __shfl_xor(m, 2, 64));
      m = fmaxf(m, __shfl_xor(m, 4, 64));
      if (q8 == 0) {
        const float q = fp8_pow2_scale(m);
        s_q[r] = q;
        s_dq[r] = 1.f / q;
      }
      __syncthreads();
      if constexpr (KE > 0) {
        // quantize H_i once into the fp8 E tile's LDS (dead after layer 0; row stride N + 16
        // bytes), so the next GEMM streams fp8 A fragments with the prefetch ring of layer 0
        // instead of converting bf16 inside its k loop
        for (int e = tid; e < TW_ROWS * (N / 8); e += 256) {
          const int rr = e / (N / 8), c8 = (e - rr * (N / 8)) * 8;
          const bf16* h = Hl + rr * ldh + c8;
          const float q = s_q[rr];
          const uint32_t lo = pack4_fp8(bf2f(h[0]) * q, bf2f(h[1]) * q, bf2f(h[2]) * q, bf2f(h[3]) * q);
          const uint32_t hi = pack4_fp8(bf2f(h[4]) * q, bf2f(h[5]) * q, bf2f(h[6]) * q, bf2f(h[7]) * q);
          *reinterpret_cast<uint2*>(X8 + rr * (N + 16) + c8) = uint2{lo, hi};
        }
        __syncthreads();
      }
    }
  }

  // ------------------------------------------------------------------ head
  const int L = a.Np[nl - 1];
  {
    const bf16* H = lds + a.h_off[nl - 1];
    const int ldh = L + 8;
    const int row = tid >> 3, q = tid & 7, Q = L / 8;
    const int grow = row0 + row;
    float yd = 0.f;
    for (int j = 0; j < Q; ++j) yd += bf2f(H[row * ldh + q * Q + j]) * a.w_out[q * Q + j];
    yd += __shfl_xor(yd, 1, 64);
    yd += __shfl_xor(yd, 2, 64);
    yd += __shfl_xor(yd, 4, 64);
    const float y = (KE > 0 ? s_yfm[row] : a.y_fm[grow]) + yd + a.b_out[0];
    const float p = 1.f / (1.f + __expf(-y));
    float dl = 0.f, lossb = 0.f;
    if (a.labels && grow < a.nvalid) {
      const float lab = a.labels[grow];
      if (a.square_loss) {
        lossb = (p - lab) * (p - lab);
        dl = 2.f * (p - lab) * p * (1.f - p) * a.gscale;
      } else {
        lossb = fmaxf(y, 0.f) - y * lab + log1pf(__expf(-fabsf(y)));
        dl = (p - lab) * a.gscale;
      }
    }
    if (q == 0) {
      if (KE > 0) a.y_fm[grow] = s_yfm[row];   // (the FM logit part, for tests / diagnostics)
      a.prob[grow] = p;
      s_dl[row] = dl;
      s_loss[row] = lossb;
      if (a.train) a.dlogit[grow] = dl;
    }
    if (a.train) {
      bf16* Z = lds + a.dz_off[0];
      const int ldz = L + 8;
      const float sl = a.inv_keep[nl - 1];
      for (int j = 0; j < Q; ++j) {
        const int col = q * Q + j;
        const float g = bf2f(H[row * ldh + col]) > 0.f ? dl * a.w_out[col] * sl : 0.f;
        Z[row * ldz + col] = f2bf(g);
      }
    }
    __syncthreads();
    // block partials [sum_rows dl*h (L) | sum dl | sum loss], fixed summation order
    float* part = a.partial + (size_t)blockIdx.x * (L + 2);
    for (int c = tid; c < L + 2; c += blockDim.x) {
      float s = 0.f;
      if (c < L) {
        if (a.train)
          for (int r = 0; r < TW_ROWS; ++r) s += s_dl[r] * bf2f(H[r * ldh + c]);
      } else if (c == L) {
        for (int r = 0; r < TW_ROWS; ++r) s += s_dl[r];
      } else {
        for (int r = 0; r < TW_ROWS; ++r) s += s_loss[r];
      }
      part[c] = s;
    }
  }
  TW_ST(7);
  if (!a.train) return;
  store_tile_t(lds + a.dz_off[0], L + 8, L, a.dZt[nl - 1], a.M, row0);
  TW_ST(8);

  // ------------------------------------------------------------------ dgrad chain
  int cur = 0;
  for (int i = nl - 1; i >= 1; --i) {
    const int Nout = a.Np[i - 1], Kin = a.Np[i];
    const bf16* Az = lds + a.dz_off[cur];
    bf16* Zo = lds + a.dz_off[cur ^ 1];
    const bf16* Hp = lds + a.h_off[i - 1];
    const int ldh = Nout + 8, ldz_in = Kin + 8, ldz_out = Nout + 8;
    const float sc = a.inv_keep[i - 1];
    for (int ct = wave; ct < Nout / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      mma32<TW_PF1>(Az, ldz_in, a.WT[i] + (size_t)ct * 32 * Kin, Kin, Kin / 32, lane, c00, c01, c10, c11);
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = ti * 16 + cr + j;
            const float v = bf2f(Hp[row * ldh + col]) > 0.f ? acc[ti][tj][j] * sc : 0.f;
            Zo[row * ldz_out + col] = f2bf(v);
          }
        }
      }
    }
    __syncthreads();
    TW_ST(8 + 2 * (nl - i) - 1);
    store_tile_t(Zo, ldz_out, Nout, a.dZt[i - 1], a.M, row0);
    TW_ST(8 + 2 * (nl - i));
    cur ^= 1;
  }
  {
    const int N0 = a.Np[0];
    const bf16* Az = lds + a.dz_off[cur];
    for (int ct = wave; ct < a.K0p / 32; ct += 4) {
      f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
      mma32<TW_PF1>(Az, N0 + 8, a.WT[0] + (size_t)ct * 32 * N0, N0, N0 / 32, lane, c00, c01, c10, c11);
      f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const int col = ct * 32 + tj * 16 + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int rl = ti * 16 + cr + j;
            a.dX0[(size_t)(row0 + rl) * a.K0p + col] = f2bf(acc[ti][tj][j]);
          }
        }
      }
    }
  }
  TW_ST(15);
}

template <bool FP8>
static int tower_launch(const TowerArgs& a, int KE, hipStream_t st) {
  const dim3 g(a.M / TW_ROWS + (KE > 0 ? a.serve_wgs + a.stamp_wgs : 0)), blk(256);
  if (!FP8 && a.l0s) {
    switch (KE) {
      case 4: hipLaunchKernelGGL((tower_l0s_tower_kernel<4>), g, blk, a.lds_bytes, st, a); return 0;
      case 8: hipLaunchKernelGGL((tower_l0s_tower_kernel<8>), g, blk, a.lds_bytes, st, a); return 0;
      case 16: hipLaunchKernelGGL((tower_l0s_tower_kernel<16>), g, blk, a.lds_bytes, st, a); return 0;
      case 32: hipLaunchKernelGGL((tower_l0s_tower_kernel<32>), g, blk, a.lds_bytes, st, a); return 0;
      default: return (int)hipErrorInvalidValue;
    }
  }
  if (!FP8 && a.serve_wgs > 0 && a.sv.rows) {   // (tag-only workgroups: the default tower)
    switch (KE) {
      case 4: hipLaunchKernelGGL((tower_light_kernel<4>), g, blk, a.lds_bytes, st, a); return 0;
      case 8: hipLaunchKernelGGL((tower_light_kernel<8>), g, blk, a.lds_bytes, st, a); return 0;
      case 16: hipLaunchKernelGGL((tower_light_kernel<16>), g, blk, a.lds_bytes, st, a); return 0;
      case 32: hipLaunchKernelGGL((tower_light_kernel<32>), g, blk, a.lds_bytes, st, a); return 0;
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (KE) {
    case 0: hipLaunchKernelGGL((tower_kernel<FP8, 0, 4, 2>), g, blk, a.lds_bytes, st, a); break;
    case 4: hipLaunchKernelGGL((tower_kernel<FP8, 4, 4, 2>), g, blk, a.lds_bytes, st, a); break;
    case 8: hipLaunchKernelGGL((tower_kernel<FP8, 8, 4, 2>), g, blk, a.lds_bytes, st, a); break;
    case 16: hipLaunchKernelGGL((tower_kernel<FP8, 16, 4, 2>), g, blk, a.lds_bytes, st, a); break;
    case 32: hipLaunchKernelGGL((tower_kernel<FP8, 32, 4, 2>), g, blk, a.lds_bytes, st, a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return 0;
}

// dX0 = dZ_0 W_0 for the tower's row block blockIdx.x, column tiles 4 blockIdx.y .. + 3 (one per
// wave): dZ_0 (the tower's bf16 tile, from dZ_0^T) transposed into LDS, then the same MFMA chain
// in the same k order as the tower's dX0 phase, so dX0 is bit-identical to the fused launch's.
// With gradient rows (a.grow, run-sorted step) each tile becomes its slots' sorted gradient rows
// (tw_grow_tile, from the block's x / S / dlogit staged in LDS) instead of dX0 -- the path that
// brings sorted rows to K = 32, whose tower has no LDS left for the rows' scratch.
// LDS: [32][N0 + 8] bf16 dZ_0 + 4 wave tiles [32][40] bf16 (+ grow: x [32][F], S [32][KE], dl [32],
// sorted positions [F][32]).
template <int KE>
__global__ void __launch_bounds__(256) tower_dx0_kernel(TowerArgs a) {
  extern __shared__ __align__(16) unsigned char dx_lds_raw[];
  bf16* Az = reinterpret_cast<bf16*>(dx_lds_raw);
  const int N0 = a.Np[0], ldz = N0 + 8;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * TW_ROWS;
  const int ct = blockIdx.y * 4 + wave;
  const bool has_tile = ct < a.K0p / 32;
  bf16* wt = Az + TW_ROWS * ldz + wave * TW_ROWS * 40;
  float* gx = reinterpret_cast<float*>(Az + TW_ROWS * ldz + 4 * TW_ROWS * 40);
  float* gS = gx + TW_ROWS * a.F;
  float* s_dl = gS + TW_ROWS * (KE > 0 ? KE : 1);
  int* ginv = reinterpret_cast<int*>(s_dl + TW_ROWS);   // [F][32] the block's sorted positions
  const bool grow = KE > 0 && a.grow != nullptr;
  // the tile's W_0 fragments first (up to 4 k-steps: N0 <= 128 entirely on registers), so their L2
  // round trip overlaps the dZ_0 load + transpose below
  constexpr int NP = 4;
  bf16x8 pb0[NP], pb1[NP];
  const bf16* Bw = a.WT[0] + (size_t)(has_tile ? ct : 0) * 32 * N0;
  bfrag_prime<NP>(pb0, pb1, Bw, N0, N0 / 32, lane);
  const bf16* zt = a.dZt[0];
  for (int e = tid; e < N0 * 2; e += 256) {  // (n pair, 8-row chunk c): 16 B of rows n, n + 1
    const int n = (e >> 2) * 2, c = e & 3;
    const bf16x8 v0 = *reinterpret_cast<const bf16x8*>(zt + (size_t)n * a.M + row0 + c * 8);
    const bf16x8 v1 = *reinterpret_cast<const bf16x8*>(zt + (size_t)(n + 1) * a.M + row0 + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // 4-B LDS writes (N0 and ldz even)
      bf16 pr[2] = {v0[j], v1[j]};
      *reinterpret_cast<uint32_t*>(Az + (c * 8 + j) * ldz + n) = *reinterpret_cast<const uint32_t*>(pr);
    }
  }
  if (grow) {  // the block's x, S and dlogit (the tower wrote S and dlogit; x = the slot values)
    for (int e = tid; e < TW_ROWS * a.F; e += 256) gx[e] = a.vals[(size_t)row0 * a.F + e];
    for (int e = tid; e < TW_ROWS * KE; e += 256) gS[e] = a.S[(size_t)row0 * KE + e];
    if (tid < TW_ROWS) s_dl[tid] = a.dlogit[row0 + tid];
    if (a.inv)  // (loaded with the rest: the row stores then wait on no dependent load)
      for (int e = tid; e < TW_ROWS * a.F; e += 256)
        ginv[e] = a.inv[(size_t)(e / TW_ROWS) * a.inv_ld + row0 + (e % TW_ROWS)];
  }
  __syncthreads();
  if (!has_tile) return;
  f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
  mma32_primed<NP>(Az, ldz, Bw, N0, N0 / 32, lane, pb0, pb1, c00, c01, c10, c11);
  const f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
  if constexpr (KE > 0) {
    if (grow) {
      tw_grow_tile<KE>(a, acc, ct, row0, lane, wt, gx, gS, a.inv ? ginv : nullptr, s_dl);
      return;
    }
  }
  tw_dx0_tile(a, acc, ct, row0, lane, wt);
}

static int tower_dx0_lds(const TowerArgs& a, int KE) {
  return 2 * TW_ROWS * (a.Np[0] + 8) + 4 * TW_ROWS * 40 * 2 +
         (a.grow ? 4 * TW_ROWS * (2 * a.F + (KE > 0 ? KE : 1) + 1) : 0);
}

// KE: embedding size of the fused gather (4, 8, 16 or 32), or 0 when E comes from fm_fwd (global)
HFM_API int hfm_tower_stamp_rows_per_wg() { return 256 * TW_STAMP_EPT; }

HFM_API int hfm_tower(const TowerArgs* ap, int KE, hipStream_t st) {
  const TowerArgs& a = *ap;
  if (a.M % TW_ROWS || a.nl < 1 || a.nl > TW_MAXL || a.K0p % 32) return (int)hipErrorInvalidValue;
  for (int i = 0; i < a.nl; ++i)
    if (a.Np[i] % 32 || a.Np[i] <= 0) return (int)hipErrorInvalidValue;
  if (a.Np[a.nl - 1] % 8) return (int)hipErrorInvalidValue;
  if (a.lds_bytes > 160 * 1024 - 1024) return (int)hipErrorInvalidValue;
  // serve workgroups: the next step's rows served ahead (stamp 2), or -- rows == null -- this step's
  // requests tagged (stamp 1: the replicated exchange's run steps)
  if (a.serve_wgs < 0 || (a.serve_wgs && (!KE || !a.train || !a.sv.recv_ids || !a.sv.step || !a.sv.T.key ||
                                          a.sv.C <= 0 || a.sv.stamp_off != (a.sv.rows ? 2 : 1) ||
                                          (long)a.serve_wgs * 256 < (long)a.sv.total * (a.sv.rows ? KE / 4 : 1))))
    return (int)hipErrorInvalidValue;
  int hbytes = 0;
  for (int i = 0; i < a.nl; ++i) hbytes += 2 * TW_ROWS * (a.Np[i] + 8);
  const int gwt_bytes = hbytes >= 4 * TW_ROWS * 40 * 2 ? 0 : 4 * TW_ROWS * 40 * 2;
  if (a.grow && a.dx0_split && (!KE || a.fp8 || !a.train || !a.S || !a.vals || !a.dlogit || (a.inv && a.inv_ld < a.M)))
    return (int)hipErrorInvalidValue;
  if (a.grow && !a.dx0_split && (!KE || a.fp8 || !a.train || (a.inv && a.inv_ld < a.M) || a.F > TW_GINV * 256 / TW_ROWS || a.g_off < 0 || (a.g_off & 15) ||
                 KE > 16 || a.g_off + TW_ROWS * (8 * a.F + 4 * KE) + gwt_bytes > a.lds_bytes))
    return (int)hipErrorInvalidValue;
  if (a.stamp_wgs < 0 || (a.stamp_wgs && (!KE || !a.train || !a.stamp_keys || !a.stamp_flags || a.stamp_div <= 0 ||
                                          (long)a.stamp_wgs * 256 * TW_STAMP_EPT < a.stamp_n)))
    return (int)hipErrorInvalidValue;
  if (KE) {
    if (a.fp8)  // H_i is re-quantized into the fp8 E tile (32 x (K0p + 16) bytes)
      for (int i = 0; i + 1 < a.nl; ++i)
        if (a.Np[i] > a.K0p) return (int)hipErrorInvalidValue;
    if (!a.idx || !a.vals || !a.tv || !a.tw || !a.fm_bias || a.F * KE > a.K0p || a.x_off < 0 ||
        (a.train && !a.Et) || (a.fp8 && a.x8_off < 0) || (a.ldv & (a.vbf16 ? 1 : 3)) || (a.idx_ld && a.idx_ld < a.M))
      return (int)hipErrorInvalidValue;
  }
  if (a.dx0_split && (a.fp8 || !a.train || !a.dX0 || !a.dZt[0] || tower_dx0_lds(a, KE) > 64 * 1024))
    return (int)hipErrorInvalidValue;
  if (a.l0s && (a.fp8 || !KE)) return (int)hipErrorInvalidValue;
  if (a.fp8) {
    if (!KE && (!a.E8 || !a.sE)) return (int)hipErrorInvalidValue;
    for (int i = 0; i < a.nl; ++i)
      if (!a.W8[i] || !a.sW[i]) return (int)hipErrorInvalidValue;
    const int rc = tower_launch<true>(a, KE, st);
    if (rc) return rc;
  } else {
    if (a.l0s) {
      if (!(KE == 4 || KE == 8 || KE == 16 || KE == 32) || a.l0s < 2 || a.l0s > TW_L0S_MAX || a.l0_ks < 1 ||
          !a.l0z || !a.l0fm ||
          (a.l0s - 1) * a.l0_ks >= a.K0p / 32 || a.l0s * a.l0_ks < a.K0p / 32 || (a.grow && !a.dx0_split) ||
          a.Np[0] % 32)
        return (int)hipErrorInvalidValue;
      const dim3 g(a.M / TW_ROWS, a.l0s), blk(256);
      const int lb = 2 * TW_ROWS * (a.l0_ks * 32 + 8);
      switch (KE) {
        case 4: hipLaunchKernelGGL(tower_l0s_kernel<4>, g, blk, lb, st, a); break;
        case 8: hipLaunchKernelGGL(tower_l0s_kernel<8>, g, blk, lb, st, a); break;
        case 16: hipLaunchKernelGGL(tower_l0s_kernel<16>, g, blk, lb, st, a); break;
        case 32: hipLaunchKernelGGL(tower_l0s_kernel<32>, g, blk, lb, st, a); break;
      }
    }
    const int rc = tower_launch<false>(a, KE, st);
    if (rc) return rc;
    if (a.dx0_split) {
      const dim3 g(a.M / TW_ROWS, (a.K0p / 32 + 3) / 4), blk(256);
      const int lb = tower_dx0_lds(a, KE);
      switch (KE) {
        case 0: hipLaunchKernelGGL(tower_dx0_kernel<0>, g, blk, lb, st, a); break;
        case 4: hipLaunchKernelGGL(tower_dx0_kernel<4>, g, blk, lb, st, a); break;
        case 8: hipLaunchKernelGGL(tower_dx0_kernel<8>, g, blk, lb, st, a); break;
        case 16: hipLaunchKernelGGL(tower_dx0_kernel<16>, g, blk, lb, st, a); break;
        case 32: hipLaunchKernelGGL(tower_dx0_kernel<32>, g, blk, lb, st, a); break;
        default: return (int)hipErrorInvalidValue;
      }
    }
  }
  HFM_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// fp8 weight shadows: W8[r, :] = e4m3(W[r, :] * q_r), sW[r] = 1 / q_r with a power-of-two q_r
// from the row's absolute max (per output channel), from the fp32 master weights.  One wave per
// row of every layer, one launch (run after each dense optimizer update and after loads).
struct W8Job {
  const float* src;  // [rows, cols] fp32 (the flat parameter buffer segment)
  uint8_t* dst;      // [rows, cols]
  float* sdq;        // [rows]
  int rows, cols;
  int row0;          // first global row of this job
  int pad;
  unsigned* amax3;   // [3][rows] row |W| maxima (float bits) for wgfin's delayed scaling, or null
};

__global__ void __launch_bounds__(256) w8_quant_kernel(const W8Job* __restrict__ jobs, int njobs, int total) {
  const int grow = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (grow >= total) return;
  int j = 0;
  while (j + 1 < njobs && grow >= jobs[j + 1].row0) ++j;
  const W8Job jb = jobs[j];
  const int r = grow - jb.row0;
  const float* src = jb.src + (size_t)r * jb.cols;
  float m = 0.f;
  for (int c = lane; c < jb.cols; c += 64) m = fmaxf(m, fabsf(src[c]));
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float q = fp8_pow2_scale(m);
  uint8_t* dst = jb.dst + (size_t)r * jb.cols;
  for (int c4 = lane; c4 < jb.cols / 4; c4 += 64) {
    const float* s4 = src + 4 * c4;
    *reinterpret_cast<uint32_t*>(dst + 4 * c4) = pack4_fp8(s4[0] * q, s4[1] * q, s4[2] * q, s4[3] * q);
  }
  if (lane == 0) {
    jb.sdq[r] = 1.f / q;
    if (jb.amax3)  // every slot: the next fused step reads a valid previous-step maximum
      for (int k = 0; k < 3; ++k) jb.amax3[k * jb.rows + r] = __float_as_uint(m);
  }
}

HFM_API int hfm_w8_quant(const void* jobs_dev, int njobs, int total_rows, hipStream_t st) {
  if (total_rows <= 0) return 0;
  hipLaunchKernelGGL(w8_quant_kernel, dim3((total_rows + 3) / 4), dim3(256), 0, st,
                     (const W8Job*)jobs_dev, njobs, total_rows);
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_w8_job_bytes() { return (int)sizeof(W8Job); }
HFM_API int hfm_tower_args_bytes() { return (int)sizeof(TowerArgs); }

// ---------------------------------------------------------------------------------------------
// Grouped weight-gradient GEMMs: dW_i = dZ_i^T X_i for every layer in ONE launch.  A wave task
// is (job, split z, tile_m, tile_n) with tile_n fastest, so the 4 waves of a workgroup usually
// share the same dZ^T rows.  Output: f32 slab z of job j at out + z * M * N.
struct WgJob {
  const bf16* A;   // [M, K] = dZ_i^T  (M = Np_i, K = batch)
  const bf16* B;   // [N, K] = X_i^T   (N = Kp_i)
  float* out;      // [splitk, M, N]
  int lda, ldb;
  int M, N;
  int tiles_m, tiles_n, splitk, kchunk;
  int task0;       // first global wave-task of this job
  int pad;
};

__global__ void __launch_bounds__(256) wgrad_group_kernel(const WgJob* __restrict__ jobs, int njobs,
                                                          int ntasks) {
  const int lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= ntasks) return;
  int j = 0;
  while (j + 1 < njobs && task >= jobs[j + 1].task0) ++j;
  const WgJob jb = jobs[j];
  int t = task - jb.task0;
  const int tn = t % jb.tiles_n;
  t /= jb.tiles_n;
  const int tm = t % jb.tiles_m;
  const int z = t / jb.tiles_m;
  const int row0 = tm * 32, col0 = tn * 32, k0 = z * jb.kchunk;
  f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
  mma32<4>(jb.A + (size_t)row0 * jb.lda + k0, jb.lda, jb.B + (size_t)col0 * jb.ldb + k0, jb.ldb,
           jb.kchunk / 32, lane, c00, c01, c10, c11);
  float* C = jb.out + (size_t)z * jb.M * jb.N;
  const int cr = (lane >> 4) * 4, cc = lane & 15;
  f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        C[(size_t)(row0 + ti * 16 + cr + q) * jb.N + col0 + tj * 16 + cc] = acc[ti][tj][q];
}

HFM_API int hfm_wgrad_group(const void* jobs_dev, int njobs, int ntasks, hipStream_t st) {
  if (ntasks <= 0) return 0;
  hipLaunchKernelGGL(wgrad_group_kernel, dim3((ntasks + 3) / 4), dim3(256), 0, st,
                     (const WgJob*)jobs_dev, njobs, ntasks);
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_wg_job_bytes() { return (int)sizeof(WgJob); }

// ---------------------------------------------------------------------------------------------
// wgfin: weight gradients + split-K combine + bias / head reductions + dense optimizer in ONE
// launch (wgfin.h); the launch's last workgroup advances the step counter.  (The single-GPU lazy
// step runs the same work inside the sparse backward's launch instead: sparse_fused.hip.)
#include "wgfin.h"

template <int OPT>
__global__ void __launch_bounds__(256) wgfin_kernel(WgFinArgs a) {
  __shared__ WgfSmem sm;
  wgfin_body<OPT, 4, WGF_MAXNS>(a, blockIdx.x, sm);
  // the launch's last workgroup (arrivals only grow: % grid) advances the step counter
  if (OPT >= 0) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(a.done_ctr, 1u, HFM_RLX_AGENT);
      if (prev % gridDim.x == gridDim.x - 1) *a.o.step += 1;
    }
  }
}

HFM_API int hfm_wgfin(int opt, const WgFinArgs* ap, hipStream_t st) {
  const WgFinArgs& a = *ap;
  if (a.ns < 1 || a.ns > WGF_MAXNS || a.kchunk % 32 || a.ldk != a.ns * 4 * a.kchunk || a.L + 2 > WGF_MAXC ||
      !a.tile_ctr || !a.done_ctr)
    return (int)hipErrorInvalidValue;
  const dim3 g(a.tile_wgs + 1), blk(256);
  switch (opt) {
    case -1: hipLaunchKernelGGL(wgfin_kernel<-1>, g, blk, 0, st, a); break;
    case OPT_ADAM: hipLaunchKernelGGL(wgfin_kernel<OPT_ADAM>, g, blk, 0, st, a); break;
    case OPT_ADAGRAD: hipLaunchKernelGGL(wgfin_kernel<OPT_ADAGRAD>, g, blk, 0, st, a); break;
    case OPT_MOMENTUM: hipLaunchKernelGGL(wgfin_kernel<OPT_MOMENTUM>, g, blk, 0, st, a); break;
    case OPT_FTRL: hipLaunchKernelGGL(wgfin_kernel<OPT_FTRL>, g, blk, 0, st, a); break;
    case OPT_GD: hipLaunchKernelGGL(wgfin_kernel<OPT_GD>, g, blk, 0, st, a); break;
    default: return (int)hipErrorInvalidValue;
  }
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_wgfin_job_bytes() { return (int)sizeof(WgFinJob); }
HFM_API int hfm_wgfin_args_bytes() { return (int)sizeof(WgFinArgs); }
