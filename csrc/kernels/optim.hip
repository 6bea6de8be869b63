// K4 sparse_optim and K5 dense_optim.
//
// Embedding tables (fm_v [R,K], fm_w [R]) — two modes:
//  * lazy      : update only the unique rows of this step (one fused row-wise kernel; the
//                l2*w term of the whole-table l2_loss is applied to those rows only).
//  * tf1_dense : reference semantics.  TF1 aggregates the gather's IndexedSlices with the
//                dense gradient of l2_loss(fm_v) (= l2*fm_v) into IndexedSlices covering every
//                row, so Adam/Adagrad/... move EVERY row EVERY step.  Implemented as a scatter of
//                the unique row-gradients into a persistent zero-invariant gradient buffer,
//                then one streaming sweep that applies g = l2*w + G and re-zeroes G.
// Dense MLP parameters live in one flat fp32 buffer (one all-reduce bucket); the dense
// optimizer also refreshes the bf16 W and W^T copies the MFMA GEMMs read (mlp.hip).
//
// The optimizer step t is read from device memory (t = *step + 1), so one captured HIP graph
// replays correctly for every step.
#include "common.h"
#include "tf1_sweep.h"

template <int K>
struct alignas(16) GradRowO {
  float v[K];
  float w;
  float pad[3];
};

template <int OPT>
__device__ __forceinline__ float lr_t_of(const OptHyper& h, const int64_t* step) {
  return OPT == OPT_ADAM ? adam_lr_t(h, *step + 1) : h.lr;
}

// ------------------------------------------------------------------ lazy row update
template <int K, int OPT>
__global__ void __launch_bounds__(256) sparse_rows_kernel(
    const int* __restrict__ ukeys, const GradRowO<K>* __restrict__ UG, const int* __restrict__ num,
    int row_div, float* __restrict__ tv, float* __restrict__ tw, float* __restrict__ s0v,
    float* __restrict__ s1v, float* __restrict__ s0w, float* __restrict__ s1w, OptHyper h,
    const int64_t* __restrict__ step, long ldv, long ldw) {
  constexpr int LPS = K / 4;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int u = gt / LPS, sub = gt % LPS;
  if (u >= *num) return;
  const float lr_t = lr_t_of<OPT>(h, step);
  const size_t row = (size_t)(ukeys[u] / row_div);
  const size_t o = row * ldv + sub * 4;
  const size_t ow = row * ldw;
  f32x4 p = *reinterpret_cast<f32x4*>(tv + o);
  f32x4 g = *reinterpret_cast<const f32x4*>(&UG[u].v[sub * 4]);
  f32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
  if (OPT != OPT_GD) a = *reinterpret_cast<f32x4*>(s0v + o);
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) c = *reinterpret_cast<f32x4*>(s1v + o);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float gj = l2_grad(g[j], h.l2, p[j]);
    float pj = p[j], aj = a[j], cj = c[j];
    opt_update<OPT>(pj, gj, aj, cj, h, lr_t);
    p[j] = pj; a[j] = aj; c[j] = cj;
  }
  *reinterpret_cast<f32x4*>(tv + o) = p;
  if (OPT != OPT_GD) *reinterpret_cast<f32x4*>(s0v + o) = a;
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) *reinterpret_cast<f32x4*>(s1v + o) = c;
  if (sub == 0) {
    float pw = tw[ow];
    float gw = l2_grad(UG[u].w, h.l2, pw);
    float aw = (OPT != OPT_GD) ? s0w[ow] : 0.f;
    float cw = (OPT == OPT_ADAM || OPT == OPT_FTRL) ? s1w[ow] : 0.f;
    opt_update<OPT>(pw, gw, aw, cw, h, lr_t);
    tw[ow] = pw;
    if (OPT != OPT_GD) s0w[ow] = aw;
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) s1w[ow] = cw;
  }
}

// ------------------------------------------------------------------ tf1_dense
template <int K>
__global__ void scatter_rows_kernel(const int* __restrict__ ukeys, const GradRowO<K>* __restrict__ UG,
                                    const int* __restrict__ num, int row_div, float* __restrict__ Gv,
                                    float* __restrict__ Gw) {
  constexpr int LPS = K / 4;
  const int gt = blockIdx.x * blockDim.x + threadIdx.x;
  const int u = gt / LPS, sub = gt % LPS;
  if (u >= *num) return;
  const size_t row = (size_t)(ukeys[u] / row_div);
  *reinterpret_cast<f32x4*>(Gv + row * K + sub * 4) =
      *reinterpret_cast<const f32x4*>(&UG[u].v[sub * 4]);
  if (sub == 0) Gw[row] = UG[u].w;
}

template <int K, int OPT>
__global__ void __launch_bounds__(256) dense_sweep_kernel(
    long R, float* __restrict__ tv, float* __restrict__ tw, float* __restrict__ Gv,
    float* __restrict__ Gw, float* __restrict__ s0v, float* __restrict__ s1v,
    float* __restrict__ s0w, float* __restrict__ s1w, OptHyper h, const int64_t* __restrict__ step,
    long ldv, long ldw) {
  constexpr int LPS = K / 4;
  const float lr_t = lr_t_of<OPT>(h, step);
  const long total = R * LPS;
  for (long gt = blockIdx.x * (long)blockDim.x + threadIdx.x; gt < total;
       gt += (long)gridDim.x * blockDim.x) {
    const long row = gt / LPS;
    const int sub = (int)(gt % LPS);
    const size_t o = (size_t)row * ldv + sub * 4;     // table / slot rows (record stride)
    const size_t og = (size_t)row * K + sub * 4;      // gradient buffer rows (dense [R, K])
    const size_t ow = (size_t)row * ldw;
    f32x4 p = *reinterpret_cast<f32x4*>(tv + o);
    f32x4 g = *reinterpret_cast<f32x4*>(Gv + og);
    f32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (OPT != OPT_GD) a = *reinterpret_cast<f32x4*>(s0v + o);
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) c = *reinterpret_cast<f32x4*>(s1v + o);
    const bool touched = (g[0] != 0.f) | (g[1] != 0.f) | (g[2] != 0.f) | (g[3] != 0.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = l2_grad(g[j], h.l2, p[j]);
      float pj = p[j], aj = a[j], cj = c[j];
      opt_update<OPT>(pj, gj, aj, cj, h, lr_t);
      p[j] = pj; a[j] = aj; c[j] = cj;
    }
    *reinterpret_cast<f32x4*>(tv + o) = p;
    if (OPT != OPT_GD) *reinterpret_cast<f32x4*>(s0v + o) = a;
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) *reinterpret_cast<f32x4*>(s1v + o) = c;
    if (touched) *reinterpret_cast<f32x4*>(Gv + og) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (sub == 0) {
      float pw = tw[ow];
      float g0 = Gw[row];
      float gw = l2_grad(g0, h.l2, pw);
      float aw = (OPT != OPT_GD) ? s0w[ow] : 0.f;
      float cw = (OPT == OPT_ADAM || OPT == OPT_FTRL) ? s1w[ow] : 0.f;
      opt_update<OPT>(pw, gw, aw, cw, h, lr_t);
      tw[ow] = pw;
      if (OPT != OPT_GD) s0w[ow] = aw;
      if (OPT == OPT_ADAM || OPT == OPT_FTRL) s1w[ow] = cw;
      if (g0 != 0.f) Gw[row] = 0.f;
    }
  }
}

// ------------------------------------------------------------------ tf1_dense, split form
// The same TF1 update as scatter + dense_sweep, split by row set (one GPU, record layout):
//  * rows of this step's batch get their full update (g = G + l2*w) from the sparse kernel's
//    lazy mode -- the arithmetic is the sweep's, so the result is bitwise the same;
//  * every OTHER row gets g = 0 + l2*w here.  The sweep knows the batch's rows from a byte flag
//    per row (set from the sorted slot keys before the step, cleared by the sweep as it skips
//    the row), so it touches no row the step reads or writes and runs CONCURRENTLY with the
//    step's tower / sparse launches on a graph side branch (no Gv/Gw gradient table at all).
//  * the sweep keeps its OWN step counter (*sw_step + 1 = t; the last workgroup to finish
//    advances it): the main counter is advanced by the step's own last launch while the sweep
//    may still be running.
__global__ void __launch_bounds__(256) stamp_rows_kernel(const int* __restrict__ keys, int n,
                                                         int row_div, unsigned char* __restrict__ flags,
                                                         unsigned char val) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = keys[i];
  // sorted keys: one store per run (unsorted input is still correct: duplicates store alike)
  if (i == 0 || keys[i - 1] != k) flags[k / row_div] = val;
}

template <int K, int OPT>
__global__ void __launch_bounds__(256) tf1_sweep_kernel(
    long R, float* __restrict__ rec, int ld, unsigned char* __restrict__ flags, OptHyper h,
    int64_t* __restrict__ sw_step, unsigned* __restrict__ done_ctr) {
  // U rows per thread per pass, all loads issued before any update: on its own graph branch the
  // sweep shares the chip with the step's launches, so it runs on few workgroups and needs
  // memory-level parallelism per thread rather than more waves
  tf1_sweep_rows<K, OPT, K <= 8 ? 4 : (K <= 16 ? 2 : 1)>(rec, ld, R, flags, h, lr_t_of<OPT>(h, sw_step),
                                         blockIdx.x * (long)blockDim.x + threadIdx.x,
                                         (long)gridDim.x * blockDim.x);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(done_ctr, 1u);
    if (prev == gridDim.x - 1) {
      *sw_step += 1;
      *done_ctr = 0u;
    }
  }
}

// ------------------------------------------------------------------ dense flat params
// ShadowSeg: common.h

template <int OPT>
__global__ void __launch_bounds__(256) dense_opt_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ s0, float* __restrict__ s1,
    long n, OptHyper h, int64_t* __restrict__ step, const ShadowSeg* __restrict__ segs, int nseg,
    unsigned* __restrict__ done_ctr) {
  const float lr_t = lr_t_of<OPT>(h, step);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dense_opt_elem<OPT>(p, g, s0, s1, i, h, lr_t, segs, nseg);
  // the step counter advances once every block has read it (last block to finish does it):
  // replaces a separate 1-thread step_inc launch at the end of every training step
  if (done_ctr) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = atomicAdd(done_ctr, 1u);
      if (prev == gridDim.x - 1) {
        *step += 1;
        *done_ctr = 0u;
      }
    }
  }
}

// refresh bf16 shadows without an update (after init / checkpoint load)
__global__ void shadow_refresh_kernel(const float* __restrict__ p, long n,
                                      const ShadowSeg* __restrict__ segs, int nseg) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    for (int s = 0; s < nseg; ++s) {
      const long rel = i - segs[s].off;
      const long sz = (long)segs[s].rows * segs[s].cols;
      if (rel >= 0 && rel < sz) {
        const int r = (int)(rel / segs[s].cols), cc = (int)(rel % segs[s].cols);
        segs[s].w16[rel] = f2bf(p[i]);
        segs[s].wt16[(long)cc * segs[s].rows + r] = f2bf(p[i]);
      }
    }
  }
}

__global__ void step_inc_kernel(int64_t* step) { *step += 1; }

// Transposed bf16 shadows of large weight segments, wt16[c][r] = w16[r][c], through 64 x 64 LDS
// tiles (16-byte row reads, 16-byte column-chunk writes): the pass that replaces the dense
// optimizer's per-element scattered wt16 stores for those segments.  Block = one tile of one
// segment (tiles numbered segment by segment); edges handled element-wise.
__global__ void __launch_bounds__(256) shadow_transpose_kernel(const ShadowSeg* __restrict__ segs, int nseg) {
  __shared__ bf16 t[64][64 + 8];
  int b = blockIdx.x, s = 0;
  for (; s < nseg; ++s) {
    const int nt = ((segs[s].rows + 63) / 64) * ((segs[s].cols + 63) / 64);
    if (b < nt) break;
    b -= nt;
  }
  if (s >= nseg) return;
  const ShadowSeg g = segs[s];
  const int tcols = (g.cols + 63) / 64;
  const int r0 = (b / tcols) * 64, c0 = (b % tcols) * 64;
  const int tid = threadIdx.x;
  const bool full = r0 + 64 <= g.rows && c0 + 64 <= g.cols && (g.cols % 8) == 0 && (g.rows % 8) == 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {          // 64 rows x 8 chunks of 8 columns
    const int e = tid + 256 * k, r = e >> 3, q = e & 7;
    if (full) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(g.w16 + (size_t)(r0 + r) * g.cols + c0 + q * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[r][q * 8 + j] = v[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rr = r0 + r, cc = c0 + q * 8 + j;
        t[r][q * 8 + j] = (rr < g.rows && cc < g.cols) ? g.w16[(size_t)rr * g.cols + cc] : f2bf(0.f);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {          // 64 columns x 8 chunks of 8 rows
    const int e = tid + 256 * k, c = e >> 3, q = e & 7;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[q * 8 + j][c];
    if (full) {
      *reinterpret_cast<bf16x8*>(g.wt16 + (size_t)(c0 + c) * g.rows + r0 + q * 8) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rr = r0 + q * 8 + j, cc = c0 + c;
        if (rr < g.rows && cc < g.cols) g.wt16[(size_t)cc * g.rows + rr] = v[j];
      }
    }
  }
}

// ------------------------------------------------------------------ dispatch
#define HFM_OPT_DISPATCH(OPT, CALL)   \
  switch (OPT) {                      \
    case OPT_ADAM: CALL(OPT_ADAM); break;         \
    case OPT_ADAGRAD: CALL(OPT_ADAGRAD); break;   \
    case OPT_MOMENTUM: CALL(OPT_MOMENTUM); break; \
    case OPT_FTRL: CALL(OPT_FTRL); break;         \
    case OPT_GD: CALL(OPT_GD); break;             \
    default: return (int)hipErrorInvalidValue;    \
  }

template <int K>
static int sparse_rows_k(int opt, const int* ukeys, const void* UG, const int* num, int max_n,
                         int row_div, float* tv, float* tw, float* s0v, float* s1v, float* s0w,
                         float* s1w, OptHyper h, const int64_t* step, long ldv, long ldw,
                         hipStream_t st) {
  constexpr int LPS = K / 4;
  const long th = (long)max_n * LPS;
  const int grid = (int)((th + 255) / 256);
  if (grid == 0) return 0;
#define CALL(O)                                                                                   \
  hipLaunchKernelGGL((sparse_rows_kernel<K, O>), dim3(grid), dim3(256), 0, st, ukeys,             \
                     (const GradRowO<K>*)UG, num, row_div, tv, tw, s0v, s1v, s0w, s1w, h, step, ldv, ldw)
  HFM_OPT_DISPATCH(opt, CALL)
#undef CALL
  HFM_LAUNCH_CHECK();
}

template <int K>
static int scatter_k(const int* ukeys, const void* UG, const int* num, int max_n, int row_div,
                     float* Gv, float* Gw, hipStream_t st) {
  constexpr int LPS = K / 4;
  const long th = (long)max_n * LPS;
  const int grid = (int)((th + 255) / 256);
  if (grid == 0) return 0;
  hipLaunchKernelGGL(scatter_rows_kernel<K>, dim3(grid), dim3(256), 0, st, ukeys,
                     (const GradRowO<K>*)UG, num, row_div, Gv, Gw);
  HFM_LAUNCH_CHECK();
}

template <int K>
static int sweep_k(int opt, long R, float* tv, float* tw, float* Gv, float* Gw, float* s0v,
                   float* s1v, float* s0w, float* s1w, OptHyper h, const int64_t* step,
                   long ldv, long ldw, hipStream_t st) {
  constexpr int LPS = K / 4;
  const long th = R * LPS;
  long g = (th + 255) / 256;
  const int grid = (int)(g < 8192 ? g : 8192);
  if (grid == 0) return 0;
#define CALL(O)                                                                              \
  hipLaunchKernelGGL((dense_sweep_kernel<K, O>), dim3(grid), dim3(256), 0, st, R, tv, tw, Gv, \
                     Gw, s0v, s1v, s0w, s1w, h, step, ldv, ldw)
  HFM_OPT_DISPATCH(opt, CALL)
#undef CALL
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

HFM_API int hfm_sparse_rows_update(int K, int opt, const int* ukeys, const void* UG, const int* num,
                                   int max_n, int row_div, float* tv, float* tw, float* s0v,
                                   float* s1v, float* s0w, float* s1w, const OptHyper* h,
                                   const int64_t* step, long ldv, long ldw, hipStream_t st) {
#define CALL(KK) sparse_rows_k<KK>(opt, ukeys, UG, num, max_n, row_div, tv, tw, s0v, s1v, s0w, s1w, *h, step, ldv, ldw, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

HFM_API int hfm_scatter_rows(int K, const int* ukeys, const void* UG, const int* num, int max_n,
                             int row_div, float* Gv, float* Gw, hipStream_t st) {
#define CALL(KK) scatter_k<KK>(ukeys, UG, num, max_n, row_div, Gv, Gw, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

HFM_API int hfm_dense_sweep(int K, int opt, long R, float* tv, float* tw, float* Gv, float* Gw,
                            float* s0v, float* s1v, float* s0w, float* s1w, const OptHyper* h,
                            const int64_t* step, long ldv, long ldw, hipStream_t st) {
#define CALL(KK) sweep_k<KK>(opt, R, tv, tw, Gv, Gw, s0v, s1v, s0w, s1w, *h, step, ldv, ldw, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

HFM_API int hfm_stamp_rows(const int* keys, int n, int row_div, unsigned char* flags, int val,
                           hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(stamp_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, keys, n, row_div,
                     flags, (unsigned char)val);
  HFM_LAUNCH_CHECK();
}

template <int K>
static int tf1_sweep_k(int opt, long R, float* rec, int ld, unsigned char* flags, OptHyper h,
                       int64_t* sw_step, unsigned* done_ctr, int max_wg, hipStream_t st) {
  const int ns = opt == OPT_GD ? 0 : ((opt == OPT_ADAM || opt == OPT_FTRL) ? 2 : 1);
  const int used = K + 4 + ns * K;
  if (ld != (used <= 16 ? (used + 15) / 16 * 16 : (used + 31) / 32 * 32))
    return (int)hipErrorInvalidValue;       // not the record layout the kernel writes
  long g = (R + 255) / 256;
  const int grid = (int)(g < max_wg ? g : max_wg);
  if (grid == 0) return 0;
#define CALL(O)                                                                                   \
  hipLaunchKernelGGL((tf1_sweep_kernel<K, O>), dim3(grid), dim3(256), 0, st, R, rec, ld, flags, h, \
                     sw_step, done_ctr)
  HFM_OPT_DISPATCH(opt, CALL)
#undef CALL
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_tf1_sweep(int K, int opt, long R, float* rec, int ld, unsigned char* flags,
                          const OptHyper* h, int64_t* sw_step, unsigned* done_ctr, int max_wg,
                          hipStream_t st) {
  switch (K) {
    case 4: return tf1_sweep_k<4>(opt, R, rec, ld, flags, *h, sw_step, done_ctr, max_wg, st);
    case 8: return tf1_sweep_k<8>(opt, R, rec, ld, flags, *h, sw_step, done_ctr, max_wg, st);
    case 16: return tf1_sweep_k<16>(opt, R, rec, ld, flags, *h, sw_step, done_ctr, max_wg, st);
    case 32: return tf1_sweep_k<32>(opt, R, rec, ld, flags, *h, sw_step, done_ctr, max_wg, st);
    default: return (int)hipErrorInvalidValue;
  }
}

HFM_API int hfm_dense_opt(int opt, float* p, const float* g, float* s0, float* s1, long n,
                          const OptHyper* h, int64_t* step, const void* segs, int nseg,
                          unsigned* done_ctr, hipStream_t st) {
  long gg = (n + 255) / 256;
  const int grid = (int)(gg < 4096 ? gg : 4096);
#define CALL(O)                                                                                  \
  hipLaunchKernelGGL((dense_opt_kernel<O>), dim3(grid), dim3(256), 0, st, p, g, s0, s1, n, *h, step, \
                     (const ShadowSeg*)segs, nseg, done_ctr)
  HFM_OPT_DISPATCH(opt, CALL)
#undef CALL
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_shadow_refresh(const float* p, long n, const void* segs, int nseg, hipStream_t st) {
  long gg = (n + 255) / 256;
  const int grid = (int)(gg < 4096 ? gg : 4096);
  hipLaunchKernelGGL(shadow_refresh_kernel, dim3(grid), dim3(256), 0, st, p, n,
                     (const ShadowSeg*)segs, nseg);
  HFM_LAUNCH_CHECK();
}

// segs: device table of nseg segments, ntiles = sum over them of ceil(rows / 64) * ceil(cols / 64)
HFM_API int hfm_shadow_transpose(const void* segs, int nseg, int ntiles, hipStream_t st) {
  if (nseg <= 0 || ntiles <= 0) return 0;
  hipLaunchKernelGGL(shadow_transpose_kernel, dim3(ntiles), dim3(256), 0, st, (const ShadowSeg*)segs, nseg);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_step_inc(int64_t* step, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_shadow_seg_bytes() { return (int)sizeof(ShadowSeg); }
HFM_API int hfm_opt_hyper_bytes() { return (int)sizeof(OptHyper); }
