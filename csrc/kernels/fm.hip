// K1 fm_fused_fwd and K2 fm_fused_bwd.
//
// Reference ops replaced (2-hvd-gpu/DeepFM-hvd-tfrecord-vectorized-map.py):
//   embedding_lookup(FM_W) * x, reduce_sum          HVD:169-171   -> y_w
//   embedding_lookup(FM_V) * x                      HVD:173-176   -> E
//   0.5*sum((sum E)^2 - sum E^2)                    HVD:177-179   -> y_v
//   reshape(E, [-1, F*K])                           HVD:195       -> MLP input (bf16, + transpose)
// and their gradients, in two kernels instead of ~15 TF ops.
//
// Layout: K/4 lanes per sample, each lane owns a float4 slice of the K-wide embedding row,
// so a wave gathers 64/(K/4) samples' rows with 16-B loads; the row index for each field is
// wave-coherent per sample.  E is written row-major [B, KP] (KP = F*K padded to 32, the GEMM
// K dimension) and transposed [KP, B] (the B operand of the layer-1 weight-gradient GEMM,
// see mlp.hip), so no GEMM ever needs an LDS transpose.
#include "common.h"

template <int K>
__global__ void __launch_bounds__(256) fm_fwd_kernel(
    const int* __restrict__ idx, const float* __restrict__ vals, const float* __restrict__ tv,
    const float* __restrict__ tw, const float* __restrict__ bias, int B, int F, int KP,
    float* __restrict__ y_fm, float* __restrict__ S, bf16* __restrict__ E, bf16* __restrict__ Et,
    long ldv, long ldw) {
  constexpr int LPS = K / 4;       // lanes per sample
  constexpr int SB = 256 / LPS;    // samples per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* lidx = reinterpret_cast<int*>(smem);
  float* lval = reinterpret_cast<float*>(smem) + SB * F;
  // stage the workgroup's [SB, F] ids / values with coalesced loads, so every row gather of
  // the field loop below is independent of a preceding global load
  const int s0 = blockIdx.x * SB;
  const int cnt = min(SB, B - s0) * F;
  const size_t base = (size_t)s0 * F;
  for (int t = threadIdx.x; t < cnt; t += 256) {
    lidx[t] = idx[base + t];
    lval[t] = vals[base + t];
  }
  __syncthreads();
  const int ls = threadIdx.x / LPS;
  const int sub = threadIdx.x % LPS;
  const int b = s0 + ls;
  if (b >= B) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, q = {0.f, 0.f, 0.f, 0.f};
  float yw = 0.f;
  const int* ib = lidx + ls * F;
  const float* xb = lval + ls * F;
  bf16* eb = E + (size_t)b * KP + sub * 4;
#pragma unroll 8
  for (int f = 0; f < F; ++f) {
    const int id = ib[f];
    const float x = xb[f];
    const f32x4 v = *reinterpret_cast<const f32x4*>(tv + (size_t)id * ldv + sub * 4);
    const f32x4 e = v * x;
    s += e;
    q += e * e;
    if ((f % LPS) == sub) yw += tw[(size_t)id * ldw] * x;
    bf16x4 eh = {f2bf(e[0]), f2bf(e[1]), f2bf(e[2]), f2bf(e[3])};
    *reinterpret_cast<bf16x4*>(eb + f * K) = eh;
    if (Et) {
      const size_t c = (size_t)(f * K + sub * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) Et[(c + j) * B + b] = eh[j];
    }
  }
  float yv = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) yv += s[j] * s[j] - q[j];
#pragma unroll
  for (int o = 1; o < LPS; o <<= 1) {
    yv += __shfl_xor(yv, o, 64);
    yw += __shfl_xor(yw, o, 64);
  }
  if (S) *reinterpret_cast<f32x4*>(S + (size_t)b * K + sub * 4) = s;
  if (sub == 0) y_fm[b] = bias[0] + yw + 0.5f * yv;
}

// fm_fwd2: one thread per (sample, field) pair for the gathers — a workgroup owns SB = 256/K
// samples (32 at K = 8, i.e. 512 workgroups for a 16K batch instead of 128 with one lane group
// per sample looping over the fields), so the random row reads of the whole batch are in flight
// at once.  The scaled rows e = V[id]*x go to an LDS tile [SB][F*K+1] (fp32); the per-sample
// sums S, sum e^2 and y_w are then reduced in fixed field order (deterministic), and E^T is
// written from the tile with 32-sample contiguous runs.
template <int K>
__global__ void __launch_bounds__(256) fm_fwd2_kernel(
    const int* __restrict__ idx, const float* __restrict__ vals, const float* __restrict__ tv,
    const float* __restrict__ tw, const float* __restrict__ bias, int B, int F, int KP,
    float* __restrict__ y_fm, float* __restrict__ S, bf16* __restrict__ E, bf16* __restrict__ Et,
    uint8_t* __restrict__ E8, float* __restrict__ sE, long ldv, long ldw, int* __restrict__ idsT,
    int Bt) {
  constexpr int SB = 256 / K;
  constexpr int V4 = K / 4;
  extern __shared__ __attribute__((aligned(16))) float fsm[];
  const int RS = F * K + 1;            // padded tile row (bank spread for the E^T pass)
  float* et = fsm;                     // [SB][RS]
  float* wx = fsm + SB * RS;           // [SB][F]
  float* qs = wx + SB * F;             // [SB] fp8 row scales (E8 mode)
  int* il = reinterpret_cast<int*>(qs + SB);  // [SB][F] the tile's ids (idsT mode)
  const int s0 = blockIdx.x * SB;
  const int nsb = min(SB, B - s0);
  const int npair = nsb * F;
  const size_t base = (size_t)s0 * F;
#pragma unroll 4
  for (int p = threadIdx.x; p < npair; p += 256) {
    const int id = idx[base + p];
    const float x = vals[base + p];
    const f32x4* row = reinterpret_cast<const f32x4*>(tv + (size_t)id * ldv);
    f32x4 v[V4];
#pragma unroll
    for (int j = 0; j < V4; ++j) v[j] = row[j];
    const float w = tw[(size_t)id * ldw];
    const int sl = p / F, f = p - sl * F;
    wx[sl * F + f] = w * x;
    if (idsT) il[p] = id;
    float* dst = et + sl * RS + f * K;
#pragma unroll
    for (int j = 0; j < V4; ++j) {
      const f32x4 e = v[j] * x;
      dst[4 * j + 0] = e[0];
      dst[4 * j + 1] = e[1];
      dst[4 * j + 2] = e[2];
      dst[4 * j + 3] = e[3];
      if (E) {
        bf16x4 eh = {f2bf(e[0]), f2bf(e[1]), f2bf(e[2]), f2bf(e[3])};
        *reinterpret_cast<bf16x4*>(E + (size_t)(s0 + sl) * KP + f * K + 4 * j) = eh;
      }
    }
  }
  __syncthreads();
  if (idsT) {
    // field-major copy of the ids for the per-field sort (field_sort.hip), which then needs no
    // transpose launch of its own: one field's SB consecutive samples per coalesced segment
    // (LDS reads at stride F, odd for Criteo's 39: conflict-free)
    for (int e = threadIdx.x; e < F * SB; e += 256) {
      const int f = e / SB, sl = e - f * SB;
      if (sl < nsb && s0 + sl < Bt) idsT[(size_t)f * Bt + s0 + sl] = il[sl * F + f];
    }
  }
  {  // per (sample, k): S, sum e^2, y_w, y_v — fixed order over fields
    const int sl = threadIdx.x / K, k = threadIdx.x % K;
    float sum = 0.f, sq = 0.f, yw = 0.f, am = 0.f;
    if (sl < nsb) {
      const float* er = et + sl * RS + k;
      for (int f = 0; f < F; ++f) {
        const float e = er[f * K];
        sum += e;
        sq += e * e;
        am = fmaxf(am, fabsf(e));
      }
      for (int f = k; f < F; f += K) yw += wx[sl * F + f];
      if (S) S[(size_t)(s0 + sl) * K + k] = sum;
    }
    float yv = sum * sum - sq;
#pragma unroll
    for (int o = 1; o < K; o <<= 1) {
      yv += __shfl_xor(yv, o, 64);
      yw += __shfl_xor(yw, o, 64);
      am = fmaxf(am, __shfl_xor(am, o, 64));
    }
    if (sl < nsb && k == 0) {
      y_fm[s0 + sl] = bias[0] + yw + 0.5f * yv;
      if (E8) {
        const float q = fp8_pow2_scale(am);
        qs[sl] = q;
        sE[s0 + sl] = 1.f / q;
      }
    }
  }
  if (E8) {  // fp8 MLP input: per-sample power-of-two scale (current scaling, no amax history)
    __syncthreads();
    const int FK4 = F * K / 4;
    for (int e = threadIdx.x; e < nsb * FK4; e += 256) {
      const int sl = e / FK4, c4 = e - sl * FK4;
      const float* src = et + sl * RS + 4 * c4;
      const float q = qs[sl];
      *reinterpret_cast<uint32_t*>(E8 + (size_t)(s0 + sl) * KP + 4 * c4) =
          pack4_fp8(src[0] * q, src[1] * q, src[2] * q, src[3] * q);
    }
  }
  if (Et) {
    const int sl = threadIdx.x % SB;
    if (sl < nsb) {
      const int FK = F * K;
      for (int c = threadIdx.x / SB; c < FK; c += 256 / SB)
        Et[(size_t)c * B + s0 + sl] = f2bf(et[sl * RS + c]);
    }
  }
}

// Gradient rows in SORTED order (i = position in the id-sorted slot list):
//   dE[b,f,:] = dX0[b, f*K:(f+1)*K] + dy_b * (S_b - E_bf)        (E_bf = V[row]*x)
//   G[i].v    = x * dE[b,f,:]     (d fm_v row)     G[i].w = dy_b * x   (d fm_w)
// The caller reduces G by key (hipcub ReduceByKey) -> one deterministic row-gradient per
// unique id, with no atomics.
template <int K>
struct alignas(16) GradRow {
  float v[K];
  float w;
  float pad[3];
};

template <int K>
__global__ void __launch_bounds__(256) fm_bwd_sorted_kernel(
    const int* __restrict__ perm, const int* __restrict__ idx, const float* __restrict__ vals,
    const float* __restrict__ tv, const float* __restrict__ dlogit, const float* __restrict__ dX0,
    const float* __restrict__ S, int n, int F, int KP, GradRow<K>* __restrict__ G) {
  constexpr int LPS = K / 4;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = gt / LPS;
  const int sub = gt % LPS;
  if (i >= n) return;
  const int p = perm[i];
  const int b = p / F, f = p - b * F;
  const int row = idx[p];
  const float x = vals[p];
  const float dy = dlogit[b];
  const f32x4 v = *reinterpret_cast<const f32x4*>(tv + (size_t)row * K + sub * 4);
  const f32x4 s = *reinterpret_cast<const f32x4*>(S + (size_t)b * K + sub * 4);
  const f32x4 dx = *reinterpret_cast<const f32x4*>(dX0 + (size_t)b * KP + f * K + sub * 4);
  const f32x4 de = dx + dy * (s - v * x);
  *reinterpret_cast<f32x4*>(&G[i].v[sub * 4]) = de * x;
  if (sub == 0) *reinterpret_cast<f32x4*>(&G[i].w) = f32x4{dy * x, 0.f, 0.f, 0.f};
}

template <int K>
static int launch_fm_fwd(const int* idx, const float* vals, const float* tv, const float* tw,
                         const float* bias, int B, int F, int KP, float* y_fm, float* S, bf16* E,
                         bf16* Et, uint8_t* E8, float* sE, long ldv, long ldw, int* idsT, int Bt,
                         hipStream_t st) {
  constexpr int SB = 256 / K;
  const size_t lds2 = ((size_t)SB * (F * K + 1) + (size_t)SB * F * (idsT ? 2 : 1) + SB) * 4;
  if (lds2 <= 120 * 1024) {
    const int grid = (B + SB - 1) / SB;
    hipLaunchKernelGGL(fm_fwd2_kernel<K>, dim3(grid), dim3(256), lds2, st, idx, vals, tv, tw, bias,
                       B, F, KP, y_fm, S, E, Et, E8, sE, ldv, ldw, idsT, Bt);
    HFM_LAUNCH_CHECK();
  }
  // fp8 output and the field-major id copy: only the row-tile variant
  if (E8 || !E || idsT) return (int)hipErrorInvalidValue;  // fp8 output: only the row-tile variant
  // very wide inputs (F*K > ~30K): lane-group-per-sample variant, small LDS footprint
  constexpr int LPS = K / 4;
  constexpr int SB1 = 256 / LPS;
  const int grid = (B + SB1 - 1) / SB1;
  const size_t lds = (size_t)SB1 * F * 8;
  hipLaunchKernelGGL(fm_fwd_kernel<K>, dim3(grid), dim3(256), lds, st, idx, vals, tv, tw, bias, B,
                     F, KP, y_fm, S, E, Et, ldv, ldw);
  HFM_LAUNCH_CHECK();
}

template <int K>
static int launch_fm_bwd(const int* perm, const int* idx, const float* vals, const float* tv,
                         const float* dlogit, const float* dX0, const float* S, int n, int F,
                         int KP, void* G, hipStream_t st) {
  constexpr int LPS = K / 4;
  const long threads = (long)n * LPS;
  const int grid = (int)((threads + 255) / 256);
  hipLaunchKernelGGL(fm_bwd_sorted_kernel<K>, dim3(grid), dim3(256), 0, st, perm, idx, vals, tv,
                     dlogit, dX0, S, n, F, KP, (GradRow<K>*)G);
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

HFM_API int hfm_fm_fwd(const int* idx, const float* vals, const float* tv, const float* tw,
                       const float* bias, int B, int F, int K, int KP, float* y_fm, float* S,
                       void* E, void* Et, void* E8, float* sE, long ldv, long ldw, int* idsT,
                       int Bt, hipStream_t st) {
  // ldv / ldw: floats between consecutive rows of the v table and entries of the w table
  // (K and 1 for plain tables; the record stride for the interleaved row-record layout).
  // E8 / sE (optional): the MLP input as OCP fp8 e4m3 rows with per-row dequant factors
  // (mlp_dtype = fp8); E may then be null.
  // idsT (optional): also write the first Bt samples' ids field-major ([F, Bt]) for
  // hfm_field_sort_pre.
#define CALL(KK) launch_fm_fwd<KK>(idx, vals, tv, tw, bias, B, F, KP, y_fm, S, (bf16*)E, (bf16*)Et, (uint8_t*)E8, sE, ldv, ldw, idsT, Bt, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

HFM_API int hfm_fm_bwd_sorted(const int* perm, const int* idx, const float* vals, const float* tv,
                              const float* dlogit, const float* dX0, const float* S, int n, int F,
                              int K, int KP, void* G, hipStream_t st) {
#define CALL(KK) launch_fm_bwd<KK>(perm, idx, vals, tv, dlogit, dX0, S, n, F, KP, G, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

HFM_API int hfm_grad_row_bytes(int K) { return K * 4 + 16; }
