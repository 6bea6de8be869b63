// K8 auc_bucket and K9 l2_full.
//
// tf.metrics.auc (HVD:242) keeps TP/FN/TN/FP at 200 thresholds
//   t_0 = -1e-7, t_i = i/199 (i = 1..198), t_199 = 1 + 1e-7     (float32 compare `pred > t_i`)
// We histogram each prediction into bucket b = #{i : t_i < pred} (binary search of the same
// float32 thresholds -> bit-identical decisions), per label; TP[i] = sum_{b > i} pos[b] etc.
// is done on the host.  Histograms from every rank are all-reduced (distributed eval, Q10).
#include "common.h"

#define NTHR 200

__constant__ float c_thr[NTHR];

__global__ void __launch_bounds__(256) auc_hist_kernel(const float* __restrict__ pred,
                                                       const float* __restrict__ label, int n,
                                                       unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[2][NTHR + 1];
  for (int i = threadIdx.x; i < 2 * (NTHR + 1); i += blockDim.x) (&h[0][0])[i] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float p = pred[i];
    int lo = 0, hi = NTHR;  // count of thresholds < p
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (c_thr[mid] < p) lo = mid + 1; else hi = mid;
    }
    const int pos = label[i] > 0.5f ? 1 : 0;
    atomicAdd(&h[pos][lo], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * (NTHR + 1); i += blockDim.x) {
    const unsigned int v = (&h[0][0])[i];
    if (v) atomicAdd(&hist[i], (unsigned long long)v);
  }
}

static bool g_thr_init = false;

HFM_API int hfm_auc_hist(const float* pred, const float* label, int n, unsigned long long* hist,
                         hipStream_t st) {
  if (!g_thr_init) {
    float t[NTHR];
    t[0] = -1e-7f;
    for (int i = 1; i < NTHR - 1; ++i) t[i] = (float)((double)i / (double)(NTHR - 1));
    t[NTHR - 1] = 1.0f + 1e-7f;
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_thr), t, sizeof(t));
    if (e != hipSuccess) return (int)e;
    g_thr_init = true;
  }
  if (n <= 0) return 0;
  int grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(auc_hist_kernel, dim3(grid), dim3(256), 0, st, pred, label, n, hist);
  HFM_LAUNCH_CHECK();
}

// sum of squares of a large fp32 array (l2_loss value for logging), per-block partials.
__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ x, long n,
                                                    double* __restrict__ out) {
  __shared__ double red[256];
  double acc = 0.0;
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    acc += (double)(v[0] * v[0] + v[1] * v[1]) + (double)(v[2] * v[2] + v[3] * v[3]);
  }
  if (blockIdx.x == 0)
    for (long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) acc += (double)x[i] * x[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

HFM_API int hfm_sumsq_partials(const float* x, long n, double* out, int nblocks, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblocks), dim3(256), 0, st, x, n, out);
  HFM_LAUNCH_CHECK();
}
