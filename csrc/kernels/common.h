// Shared definitions for the hipfm gfx950 (MI355X / CDNA4) kernels.
//
// Every kernel library entry point is a C ABI function (HFM_API) taking raw device
// pointers + a hipStream_t and returning a hipError_t as int.  Python binds them with
// ctypes after `import torch` (so the HIP runtime torch already loaded is reused: both
// carry SONAME libamdhip64.so.7) and launches on torch's current stream, which makes the
// whole train step capturable into a HIP graph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// sorted gradient rows (tower -> sparse backward) are {a[K], g_w, c}: K + 2 floats, so a row
// start is only 8-B aligned -- these types say so (the compiler must not assume 16 B)
typedef float f32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
typedef float f32x2a8 __attribute__((ext_vector_type(2), aligned(8)));
__host__ __device__ constexpr int grow_stride(int K) { return K + 2; }

#define HFM_API extern "C" __attribute__((visibility("default")))

#define HFM_LAUNCH_CHECK() return (int)hipGetLastError()

// ---- phase stamps (diagnostic build only: HIPFM_BUILD_STAMPS=1 compiles with -DHFM_STAMPS into
// its own library; the production kernels contain none of this).  HFM_STAMP_BUF(name) defines a
// per-translation-unit buffer of 100-MHz wall-clock stamps [slot][16] and C entry points
// name_read / name_clear; HFM_STAMP(name, slot, k) has thread 0 of the workgroup record stamp k
// of `slot` (a vector store from a VGPR; nothing in any kernel reads the buffer).
#ifdef HFM_STAMPS
#define HFM_STAMP_SLOTS (1 << 16)
#define HFM_STAMP_BUF(name)                                                                 \
  __device__ unsigned long long name[HFM_STAMP_SLOTS * 16];                                \
  HFM_API int name##_read(void* dst, size_t bytes) {                                        \
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(name), bytes, 0, hipMemcpyDeviceToHost); \
  }                                                                                         \
  HFM_API int name##_slots() { return HFM_STAMP_SLOTS; }
#define HFM_STAMP(name, slot, k)                                                            \
  do {                                                                                      \
    if (threadIdx.x == 0) {                                                                 \
      volatile unsigned long long t = __builtin_amdgcn_s_memrealtime();                     \
      name[((unsigned)(slot) % HFM_STAMP_SLOTS) * 16 + (k)] = t + threadIdx.x;              \
    }                                                                                       \
  } while (0)
#else
#define HFM_STAMP_BUF(name)
#define HFM_STAMP(name, slot, k) \
  do {                           \
  } while (0)
#endif

// ---- counter-based RNG (mirrors hipfm/utils/rng.py bit-for-bit) ----
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t dropout_salt(uint32_t seed, uint32_t step, uint32_t layer) {
  return fmix32(seed ^ fmix32(step + layer * 0x632BE5ABu));
}
__device__ __forceinline__ bool dropout_keep(uint32_t flat, uint32_t salt, uint32_t thr) {
  return fmix32((flat * 0x9E3779B1u) ^ salt) < thr;
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// Per-slot embedding gradient terms of the FM + MLP backward (sparse_fused.hip derivation): for
// slot (b, f) with value x, dX0 slice dx (bf16-rounded), dlogit dy and S_b = sum_f E:
//   a = x * (dx + dy * S_b),  g_w = dy * x,  c = dy * x * x.
// One definition for the sparse kernel's own gather and the tower's sorted-row emission, so the
// two produce the same bits.
__device__ __forceinline__ f32x4 sf_slot_a(f32x4 dx, float dy, f32x4 s, float x) { return (dx + dy * s) * x; }
__device__ __forceinline__ float sf_slot_gw(float dy, float x) { return dy * x; }
__device__ __forceinline__ float sf_slot_c(float dy, float x) { return dy * x * x; }
// A row's gradient from its summed slot terms, g_v = a - v * c, and the whole-table l2 term,
// g + l2 * p: written as explicit fmas so every kernel that forms them (sparse tile lazy / scatter /
// exchange rows, owner update, sweeps) rounds identically -- left to contraction, the compiler
// fused them differently in different kernels (1-ulp slot differences, tf1 split vs scatter).
__device__ __forceinline__ f32x4 row_grad4(f32x4 a, f32x4 v, float c) {
  return f32x4{fmaf(-v[0], c, a[0]), fmaf(-v[1], c, a[1]), fmaf(-v[2], c, a[2]), fmaf(-v[3], c, a[3])};
}
__device__ __forceinline__ float l2_grad(float g, float l2, float p) { return fmaf(l2, p, g); }

// ---- embedding-table rows: fp32, or bf16 (mixed-precision embeddings, BASELINE config #5) ----
// A row (or optimizer-slot row) starts at a float* inside the table record; a bf16 row holds its
// K values in the first K/2 floats.  4 consecutive elements from element e (e % 4 == 0):
__device__ __forceinline__ f32x4 ld_row4(const float* row, int e, bool bf) {
  if (!bf) return *reinterpret_cast<const f32x4*>(row + e);
  const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(row) + e);
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xFFFF0000u)};
}
// Stochastic rounding fp32 -> bf16 (unbiased: lazy-Adam moments move by ~0.1 % per step, below
// bf16's 0.4 % resolution, and would freeze under round-to-nearest).  Counter-based and
// deterministic: the random low half comes from fmix32 of (seed, element), so a replayed step
// rounds identically.  Non-finite values are truncated unchanged.
__device__ __forceinline__ uint32_t f2bf_sr(float x, uint32_t rnd) {
  uint32_t b = __float_as_uint(x);
  if ((b & 0x7F800000u) != 0x7F800000u) b += rnd & 0xFFFFu;
  return b >> 16;
}
__device__ __forceinline__ void st_row4(float* row, int e, f32x4 v, bool bf, uint32_t seed) {
  if (!bf) {
    *reinterpret_cast<f32x4*>(row + e) = v;
    return;
  }
  uint2 u;
  u.x = f2bf_sr(v[0], fmix32(seed + 4u * e)) | (f2bf_sr(v[1], fmix32(seed + 4u * e + 1u)) << 16);
  u.y = f2bf_sr(v[2], fmix32(seed + 4u * e + 2u)) | (f2bf_sr(v[3], fmix32(seed + 4u * e + 3u)) << 16);
  *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(row) + e) = u;
}
// the values st_row4 stores, as fp32 (a copy of an updated row that must equal the stored row)
__device__ __forceinline__ f32x4 rounded_row4(f32x4 v, int e, bool bf, uint32_t seed) {
  if (!bf) return v;
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = __uint_as_float(f2bf_sr(v[j], fmix32(seed + 4u * e + j)) << 16);
  return r;
}
// rounding seed of (table row, optimizer step, which array: 0 = v, 1 / 2 = slots)
__device__ __forceinline__ uint32_t row_sr_seed(size_t row, int64_t step, uint32_t which) {
  return fmix32((uint32_t)row ^ fmix32((uint32_t)(row >> 32) ^ ((uint32_t)step * 0x9E3779B1u) ^
                                       (which * 0x85EBCA77u)));
}

// ---- OCP fp8 e4m3 (gfx950 v_cvt_pk_fp8_f32 is OCP e4m3fn, max 448; NOT MI300's fnuz) ----
constexpr float FP8_MAX = 448.f;
// 4 floats -> 4 e4m3 bytes (little-endian: a in byte 0), round-to-nearest-even, saturating
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, FP8_MAX, -FP8_MAX);
  b = __builtin_amdgcn_fmed3f(b, FP8_MAX, -FP8_MAX);
  c = __builtin_amdgcn_fmed3f(c, FP8_MAX, -FP8_MAX);
  d = __builtin_amdgcn_fmed3f(d, FP8_MAX, -FP8_MAX);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
// Power-of-two quantization scale s for a row / tensor of absolute max `amax`: amax * s lands
// in (224, 448], and s and its inverse are exact (dequantization adds no rounding).
__device__ __forceinline__ float fp8_pow2_scale(float amax) {
  if (!(amax > 1e-30f) || !(amax < 3.0e38f)) return 1.f;
  int e;
  frexpf(FP8_MAX / amax, &e);
  e = e > 100 ? 100 : e;
  return ldexpf(1.f, e - 1);
}

// Optimizer ids shared by the sparse/dense optimizer kernels (hipfm/ops/optim.py).
enum HfmOpt { OPT_ADAM = 0, OPT_ADAGRAD = 1, OPT_MOMENTUM = 2, OPT_FTRL = 3, OPT_GD = 4 };

struct OptHyper {
  float lr;        // base learning rate (already x world size)
  float l2;        // l2_reg added as l2*w to sparse-table grads (0 for dense MLP params)
  float b1, b2, eps;
  float momentum;  // Momentum
};

// TF1 Adam learning-rate correction with the beta powers of step t (1-based).
__device__ __forceinline__ float adam_lr_t(const OptHyper& h, int64_t t) {
  float b1p = powf(h.b1, (float)t), b2p = powf(h.b2, (float)t);
  return h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
}

// One optimizer update of a single element; s0/s1 are the optimizer slots.  Every
// multiply-add is an explicit fmaf and no product feeds a plain add/sub, so the rounding does not
// depend on which FMAs the compiler would form in the inlining context: the dense optimizer fused
// into the gradient finalize (fin_opt_apply) and the dense_opt sweep stay bitwise equal.
template <int OPT>
__device__ __forceinline__ void opt_update(float& p, float g, float& s0, float& s1,
                                           const OptHyper& h, float lr_t) {
  if (OPT == OPT_ADAM) {
    s0 = fmaf(s0, h.b1, (1.f - h.b1) * g);
    s1 = fmaf(s1, h.b2, (1.f - h.b2) * g * g);
    p -= lr_t * s0 / (sqrtf(s1) + h.eps);
  } else if (OPT == OPT_ADAGRAD) {
    s0 = fmaf(g, g, s0);
    p = fmaf(-h.lr * g, rsqrtf(s0), p);
  } else if (OPT == OPT_MOMENTUM) {
    s0 = fmaf(s0, h.momentum, g);
    p = fmaf(-h.lr, s0, p);
  } else if (OPT == OPT_FTRL) {  // lr_power=-0.5, l1=l2=0 (tf.train.FtrlOptimizer defaults)
    float a0 = s0, an = fmaf(g, g, a0);
    float sa = sqrtf(an);
    float sigma = (sa - sqrtf(a0)) / h.lr;
    s1 = fmaf(-sigma, p, s1 + g);
    s0 = an;
    p = -s1 / (sa / h.lr);
  } else {  // GD
    p = fmaf(-h.lr, g, p);
  }
}

// A weight matrix [rows, cols] inside the flat dense buffer with bf16 copies (MFMA operands).
struct ShadowSeg {
  long off;          // element offset in the flat buffer
  int rows, cols;
  bf16* w16;         // [rows, cols]
  bf16* wt16;        // [cols, rows]
};

// Dense optimizer applied by the thread that produces an element's final gradient (the
// single-GPU finalize + dense_opt fusion, mlp.hip): no second pass over the flat buffer.
struct FinOpt {
  float* p;
  float* g;          // flat gradient buffer; a finalize output outside [g, g + n) is no parameter
  float* s0;
  float* s1;
  long n;
  OptHyper h;
  int64_t* step;     // read by every block; the last block to finish advances it
  const ShadowSeg* segs;
  int nseg;
  unsigned* done_ctr;
};

// One element of the dense optimizer sweep (+ bf16 shadows): dense_opt_kernel and the merged
// owner-apply launch (shard.hip) share it, so their results are bitwise equal.
template <int OPT>
__device__ __forceinline__ void dense_opt_apply(float* __restrict__ p, float gi, float* __restrict__ s0,
                                                float* __restrict__ s1, long i, const OptHyper& h, float lr_t,
                                                const ShadowSeg* __restrict__ segs, int nseg) {
  float pi = p[i];
  float a = (OPT != OPT_GD) ? s0[i] : 0.f;
  float c = (OPT == OPT_ADAM || OPT == OPT_FTRL) ? s1[i] : 0.f;
  opt_update<OPT>(pi, gi, a, c, h, lr_t);
  p[i] = pi;
  if (OPT != OPT_GD) s0[i] = a;
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) s1[i] = c;
  for (int s = 0; s < nseg; ++s) {
    const long rel = i - segs[s].off;
    const long sz = (long)segs[s].rows * segs[s].cols;
    if (rel >= 0 && rel < sz) {
      const int r = (int)(rel / segs[s].cols), cc = (int)(rel % segs[s].cols);
      segs[s].w16[rel] = f2bf(pi);
      // (wt16 null: a large segment whose transposed shadow a tiled pass writes afterwards --
      // optim.hip shadow_transpose; one scattered 2-byte store per element cost 0.5 ms per
      // 4096x4096 step)
      if (segs[s].wt16) segs[s].wt16[(long)cc * segs[s].rows + r] = f2bf(pi);
    }
  }
}

template <int OPT>
__device__ __forceinline__ void dense_opt_elem(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ s0, float* __restrict__ s1, long i,
                                               const OptHyper& h, float lr_t, const ShadowSeg* __restrict__ segs,
                                               int nseg) {
  dense_opt_apply<OPT>(p, g[i], s0, s1, i, h, lr_t, segs, nseg);
}

template <int OPT>
__device__ __forceinline__ void fin_opt_apply(const FinOpt& o, float lr_t, const float* dst, float gv) {
  const long i = dst - o.g;
  if (i < 0 || i >= o.n) return;
  // gv arrives as an SSA product (slab sum * scale): pin it to a rounded fp32 register so the
  // update cannot contract that multiply into its own adds -- dense_opt reads g from memory, and
  // the fused path must stay bitwise equal to it (tests/test_gpu_kernels.py)
  asm volatile("" : "+v"(gv));
  float pi = o.p[i];
  float a = (OPT != OPT_GD) ? o.s0[i] : 0.f;
  float c = (OPT == OPT_ADAM || OPT == OPT_FTRL) ? o.s1[i] : 0.f;
  opt_update<OPT>(pi, gv, a, c, o.h, lr_t);
  o.p[i] = pi;
  if (OPT != OPT_GD) o.s0[i] = a;
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) o.s1[i] = c;
  for (int s = 0; s < o.nseg; ++s) {
    const long rel = i - o.segs[s].off;
    if (rel >= 0 && rel < (long)o.segs[s].rows * o.segs[s].cols) {
      const int r = (int)(rel / o.segs[s].cols), cc = (int)(rel % o.segs[s].cols);
      o.segs[s].w16[rel] = f2bf(pi);
      if (o.segs[s].wt16) o.segs[s].wt16[(long)cc * o.segs[s].rows + r] = f2bf(pi);
    }
  }
}
