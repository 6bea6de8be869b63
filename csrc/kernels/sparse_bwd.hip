// Fused embedding backward: K2 (per-slot FM/MLP-input gradient) + K3 (sum per unique id) +
// optionally K4 (lazy row optimizer / tf1_dense scatter).  SURVEY §2.5 rows 17-20, §7.4 item 1.
//
// Per slot (b, f) with id r and value x:
//     d fm_v[r] += x*(dX0[b, f*K:(f+1)*K] + dy_b*(S_b - x*V[r]))  =  a_slot - V[r]*c_slot
// (dX0, the layer-1 input gradient, arrives in bf16 like every other MLP activation)
//     d fm_w[r] += dy_b*x
// with a_slot = x*(dX0 + dy_b*S_b) and c_slot = x^2*dy_b.  V[r] is the SAME row for every slot
// of an id, so it is factored out of the sum: the per-slot pass never touches the embedding
// table (no random table-row reads for the 640K slots of a 16K batch); the row is read once per
// unique id, by the update kernel that reads it anyway.
//
// Input: the slot ids sorted by radix_sort.hip (sorted_keys, perm).
// Kernel A (one workgroup per TP consecutive sorted slots): computes [a(K) | g_w | c] of every
//   slot into LDS, sums each run of equal ids inside the tile from LDS, and writes
//     partial[h]  for a run whose id starts in the tile (h = head position, or the compact
//                 unique index sid when the caller needs compact rows for an exchange),
//     cont[tile]  for the run that continues an id from the previous tile.
// Kernel B: one lane group per head slot (position-indexed mode) or per unique id (compact
//   mode); total = partial + cont of every later tile the id spans (tile order: bitwise
//   deterministic), g = a - V[row]*c, then: lazy optimizer on the row / scatter into the
//   tf1_dense gradient buffer / write the compact unique-row gradient UG[s].
#include <hipcub/hipcub.hpp>
#include "common.h"

template <int K>
struct TileCfg {
  static constexpr int TP = (K <= 16) ? 512 : (K == 32 ? 256 : 128);
  static constexpr int LPS = K / 4;
  static constexpr int PPP = 256 / LPS;  // positions per pass
  static constexpr int PASSES = TP / PPP;
  static constexpr int C = K + 2;        // columns: a[K], g_w, c
  static constexpr int RS = K + 4;       // row stride of partial / cont / UG (16-B aligned)
};

__global__ void seg_flags_kernel(const int* __restrict__ sk, int* __restrict__ flags, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1 : 0;
}

__global__ void seg_info_kernel(const int* __restrict__ sk, const int* __restrict__ sid_incl, int n,
                                int* __restrict__ ukeys, int* __restrict__ seg_start,
                                int* __restrict__ num) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = sid_incl[i] - 1;
  if (i == 0 || sk[i] != sk[i - 1]) {
    seg_start[s] = i;
    ukeys[s] = sk[i];
  }
  if (i == n - 1) {
    *num = s + 1;
    seg_start[s + 1] = n;
  }
}

// sid_incl == nullptr -> position-indexed partials (partial[head position])
template <int K>
__global__ void __launch_bounds__(256) fm_bwd_seg_kernel(
    const int* __restrict__ sorted_keys, const int* __restrict__ perm, const int* __restrict__ sid_incl,
    const float* __restrict__ vals, const float* __restrict__ dlogit, const bf16* __restrict__ dX0,
    const float* __restrict__ S, int n, int F, int KP, float* __restrict__ partial,
    float* __restrict__ cont) {
  using T = TileCfg<K>;
  __shared__ float g[T::TP][T::C];
  __shared__ int skl[T::TP];
  const int b0 = blockIdx.x * T::TP;
  const int sub = threadIdx.x % T::LPS;
#pragma unroll
  for (int ps = 0; ps < T::PASSES; ++ps) {
    const int p = ps * T::PPP + threadIdx.x / T::LPS;
    const int i = b0 + p;
    if (i < n) {
      const int q = perm[i];
      const int b = q / F, f = q - b * F;
      const float x = vals[q];
      const float dy = dlogit[b];
      const f32x4 s = *reinterpret_cast<const f32x4*>(S + (size_t)b * K + sub * 4);
      const bf16x4 dxh = *reinterpret_cast<const bf16x4*>(dX0 + (size_t)b * KP + f * K + sub * 4);
      const f32x4 dx = {bf2f(dxh[0]), bf2f(dxh[1]), bf2f(dxh[2]), bf2f(dxh[3])};
      const f32x4 a = (dx + dy * s) * x;
#pragma unroll
      for (int j = 0; j < 4; ++j) g[p][sub * 4 + j] = a[j];
      if (sub == 0) {
        g[p][K] = dy * x;
        g[p][K + 1] = dy * x * x;
        skl[p] = sorted_keys[i];
      }
    } else if (sub == 0) {
      skl[p] = 0x7fffffff;
    }
  }
  __syncthreads();
  const int nloc = min(T::TP, n - b0);
  const bool first_is_head = (b0 == 0) || (sorted_keys[b0 - 1] != skl[0]);
  if (nloc == T::TP && skl[0] == skl[T::TP - 1]) {
    // the whole tile is one id (dense-field / Zipf-hot ids): all 256 threads reduce it —
    // 8 lanes per column sum strided slices, then the 8 partials are added in a fixed order
    __shared__ float red[8][T::C];
    const int zl = threadIdx.x / 32;
    for (int c = threadIdx.x % 32; c < T::C; c += 32) {   // K >= 32: C > 32 columns
      float a0 = 0.f, a1 = 0.f;
      for (int q = zl; q < T::TP; q += 16) {
        a0 += g[q][c];
        if (q + 8 < T::TP) a1 += g[q + 8][c];
      }
      red[zl][c] = a0 + a1;
    }
    __syncthreads();
    if (threadIdx.x < T::C) {
      const int cc = threadIdx.x;
      const float tot = ((red[0][cc] + red[1][cc]) + (red[2][cc] + red[3][cc])) +
                        ((red[4][cc] + red[5][cc]) + (red[6][cc] + red[7][cc]));
      if (first_is_head) {
        const int h = sid_incl ? sid_incl[b0] - 1 : b0;
        partial[(size_t)h * T::RS + cc] = tot;
      } else {
        cont[(size_t)blockIdx.x * T::RS + cc] = tot;
      }
    }
    return;
  }
  for (int e = threadIdx.x; e < nloc * T::C; e += blockDim.x) {
    const int p = e / T::C, c = e - p * T::C;
    if (p != 0 && skl[p] == skl[p - 1]) continue;  // not a run start
    const int key = skl[p];
    float s0 = g[p][c], s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int q = p + 1;
    for (; q + 3 < nloc && skl[q + 3] == key; q += 4) {
      s0 += g[q][c];
      s1 += g[q + 1][c];
      s2 += g[q + 2][c];
      s3 += g[q + 3][c];
    }
    for (; q < nloc && skl[q] == key; ++q) s0 += g[q][c];
    const float tot = (s0 + s1) + (s2 + s3);
    if (p > 0 || first_is_head) {
      const int h = sid_incl ? sid_incl[b0 + p] - 1 : b0 + p;
      partial[(size_t)h * T::RS + c] = tot;
    } else {
      cont[(size_t)blockIdx.x * T::RS + c] = tot;
    }
  }
}

// MODE: 0 = lazy optimizer (OPT), 1 = tf1_dense scatter into (Gv, Gw), 2 = write UG[s]
struct SegApplyArgs {
  const int* sorted_keys;  // position mode: heads found from the sorted keys
  const int* ukeys;        // compact mode: unique ids
  const int* seg_start;    // compact mode: [U+1]
  const int* num;          // compact mode: U (device)
  int n, ntiles, compact;  // compact = 1 -> one group per unique id
  int row_div;             // table row of id = id / row_div
  int vsrc_compact;        // 1 -> V row of unique s is vsrc[s] (gathered rows, sharded mode)
  const float* vsrc;       // rows used for g = a - V*c (nullable: then tv)
  const float* partial;
  const float* cont;
  float* UG;
  float *tv, *tw, *s0v, *s1v, *s0w, *s1w;
  float *Gv, *Gw;
  OptHyper h;
  const int64_t* step;
  long ldv, ldw;           // table row strides (record layout: both = record floats)
};

template <int K, int MODE, int OPT>
__global__ void __launch_bounds__(256) seg_apply_kernel(SegApplyArgs A) {
  using T = TileCfg<K>;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int u = gt / T::LPS, sub = gt % T::LPS;
  int key, first, ti;
  if (A.compact) {
    if (u >= *A.num) return;
    key = A.ukeys[u];
    first = A.seg_start[u];
    ti = u;
  } else {
    if (u >= A.n) return;
    key = A.sorted_keys[u];
    if (u > 0 && A.sorted_keys[u - 1] == key) return;  // not a head
    first = u;
    ti = u;
  }
  const float* pr = A.partial + (size_t)ti * T::RS;
  f32x4 a = *reinterpret_cast<const f32x4*>(pr + sub * 4);
  float w = pr[K], c = pr[K + 1];
  if (A.compact) {
    const int last = A.seg_start[u + 1] - 1;
    for (int b = first / T::TP + 1; b <= last / T::TP; ++b) {
      const float* cr = A.cont + (size_t)b * T::RS;
      a += *reinterpret_cast<const f32x4*>(cr + sub * 4);
      w += cr[K];
      c += cr[K + 1];
    }
  } else {
    for (int b = first / T::TP + 1; b < A.ntiles && A.sorted_keys[b * T::TP] == key; ++b) {
      const float* cr = A.cont + (size_t)b * T::RS;
      a += *reinterpret_cast<const f32x4*>(cr + sub * 4);
      w += cr[K];
      c += cr[K + 1];
    }
  }
  const size_t row = (size_t)(key / A.row_div);
  const float* vrow = A.vsrc ? (A.vsrc + (size_t)(A.vsrc_compact ? u : row) * K) : (A.tv + row * A.ldv);
  const f32x4 v = *reinterpret_cast<const f32x4*>(vrow + sub * 4);
  const f32x4 gv = row_grad4(a, v, c);
  if (MODE == 2) {
    *reinterpret_cast<f32x4*>(A.UG + (size_t)u * T::RS + sub * 4) = gv;
    if (sub == 0) *reinterpret_cast<f32x4*>(A.UG + (size_t)u * T::RS + K) = f32x4{w, 0.f, 0.f, 0.f};
  } else if (MODE == 1) {
    *reinterpret_cast<f32x4*>(A.Gv + row * K + sub * 4) = gv;
    if (sub == 0) A.Gw[row] = w;
  } else {
    constexpr int O = OPT;
    const float lr_t = (O == OPT_ADAM) ? adam_lr_t(A.h, *A.step + 1) : A.h.lr;
    const size_t o = row * A.ldv + sub * 4;
    const size_t ow = row * A.ldw;
    f32x4 p = A.vsrc ? *reinterpret_cast<f32x4*>(A.tv + o) : v;   // same row already loaded
    f32x4 s0 = {0, 0, 0, 0}, s1 = {0, 0, 0, 0};
    if (O != OPT_GD) s0 = *reinterpret_cast<f32x4*>(A.s0v + o);
    if (O == OPT_ADAM || O == OPT_FTRL) s1 = *reinterpret_cast<f32x4*>(A.s1v + o);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = l2_grad(gv[j], A.h.l2, p[j]);
      float pj = p[j], aj = s0[j], cj = s1[j];
      opt_update<O>(pj, gj, aj, cj, A.h, lr_t);
      p[j] = pj; s0[j] = aj; s1[j] = cj;
    }
    *reinterpret_cast<f32x4*>(A.tv + o) = p;
    if (O != OPT_GD) *reinterpret_cast<f32x4*>(A.s0v + o) = s0;
    if (O == OPT_ADAM || O == OPT_FTRL) *reinterpret_cast<f32x4*>(A.s1v + o) = s1;
    if (sub == 0) {
      float pw = A.tw[ow];
      float gw = l2_grad(w, A.h.l2, pw);
      float aw = (O != OPT_GD) ? A.s0w[ow] : 0.f;
      float cw = (O == OPT_ADAM || O == OPT_FTRL) ? A.s1w[ow] : 0.f;
      opt_update<O>(pw, gw, aw, cw, A.h, lr_t);
      A.tw[ow] = pw;
      if (O != OPT_GD) A.s0w[ow] = aw;
      if (O == OPT_ADAM || O == OPT_FTRL) A.s1w[ow] = cw;
    }
  }
}

HFM_API int hfm_seg_tiles(int K, int n) {
  int tp = (K <= 16) ? 512 : (K == 32 ? 256 : 128);
  return (n + tp - 1) / tp;
}

// Segment structure of a sorted key list: ukeys[U], seg_start[U+1], num = U.
HFM_API int hfm_segments(const int* sorted_keys, int n, int* flags_tmp, int* sid_incl, int* ukeys,
                         int* seg_start, int* num, void* temp, size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return (int)hipMemsetAsync(num, 0, sizeof(int), st);
  const int g = (n + 255) / 256;
  hipLaunchKernelGGL(seg_flags_kernel, dim3(g), dim3(256), 0, st, sorted_keys, flags_tmp, n);
  size_t tb = temp_bytes;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(temp, tb, flags_tmp, sid_incl, n, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(seg_info_kernel, dim3(g), dim3(256), 0, st, sorted_keys, sid_incl, n, ukeys,
                     seg_start, num);
  HFM_LAUNCH_CHECK();
}

template <int K>
static int bwd_seg_k(const int* sk, const int* perm, const int* sid_incl, const float* vals,
                     const float* dlogit, const bf16* dX0, const float* S, int n, int F, int KP,
                     float* partial, float* cont, hipStream_t st) {
  using T = TileCfg<K>;
  const int tiles = (n + T::TP - 1) / T::TP;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(fm_bwd_seg_kernel<K>, dim3(tiles), dim3(256), 0, st, sk, perm, sid_incl, vals,
                     dlogit, dX0, S, n, F, KP, partial, cont);
  HFM_LAUNCH_CHECK();
}

template <int K>
static int apply_k(int mode, int opt, const SegApplyArgs& A, int max_groups, hipStream_t st) {
  using T = TileCfg<K>;
  const long th = (long)max_groups * T::LPS;
  const int grid = (int)((th + 255) / 256);
  if (grid == 0) return 0;
#define L_(M, O) hipLaunchKernelGGL((seg_apply_kernel<K, M, O>), dim3(grid), dim3(256), 0, st, A)
  if (mode == 2) {
    L_(2, 0);
  } else if (mode == 1) {
    L_(1, 0);
  } else {
    switch (opt) {
      case OPT_ADAM: L_(0, OPT_ADAM); break;
      case OPT_ADAGRAD: L_(0, OPT_ADAGRAD); break;
      case OPT_MOMENTUM: L_(0, OPT_MOMENTUM); break;
      case OPT_FTRL: L_(0, OPT_FTRL); break;
      case OPT_GD: L_(0, OPT_GD); break;
      default: return (int)hipErrorInvalidValue;
    }
  }
#undef L_
  HFM_LAUNCH_CHECK();
}

#define HFM_K_DISPATCH(K, CALL) \
  switch (K) {                  \
    case 4: return CALL(4);     \
    case 8: return CALL(8);     \
    case 16: return CALL(16);   \
    case 32: return CALL(32);   \
    case 64: return CALL(64);   \
    default: return (int)hipErrorInvalidValue; \
  }

// sid_incl == nullptr -> position-indexed partials
HFM_API int hfm_fm_bwd_seg(int K, const int* sk, const int* perm, const int* sid_incl,
                           const float* vals, const float* dlogit, const void* dX0v, const float* S,
                           int n, int F, int KP, float* partial, float* cont, hipStream_t st) {
  const bf16* dX0 = (const bf16*)dX0v;   // dX0 is bf16 [B, KP] (layer-1 dgrad output)
#define CALL(KK) bwd_seg_k<KK>(sk, perm, sid_incl, vals, dlogit, dX0, S, n, F, KP, partial, cont, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

// mode 0: lazy optimizer `opt`; 1: tf1_dense scatter; 2: write compact UG.  max_groups = n
// (position mode) or an upper bound of U (compact mode).
HFM_API int hfm_seg_apply(int K, int mode, int opt, const SegApplyArgs* A, int max_groups,
                          hipStream_t st) {
#define CALL(KK) apply_k<KK>(mode, opt, *A, max_groups, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}
HFM_API int hfm_seg_apply_args_bytes() { return (int)sizeof(SegApplyArgs); }
