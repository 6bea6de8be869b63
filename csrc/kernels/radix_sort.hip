// Stable LSD radix sort of non-negative int32 keys (slot ids) with their slot positions,
// specialised for the DeepFM batch-id sort.
//
// Why not hipCUB: at 16K-sample batches (n = 640K slots) rocPRIM dispatches a block-sort +
// merge-path sort (10 merge passes, ~140 us on MI355X, measured in profiles/); this sort does
// ceil(end_bit / 8) passes of {per-tile digit histogram, exclusive scan, stable scatter} and
// generates the position values itself in the first pass (no iota kernel, no final copy).
//
// Stable in-tile ranking (wave64): a lane's peers (same digit) are found with 8 ballots, its
// rank among earlier lanes is popcount(peers & lanemask_lt); per-wave counts are combined in
// wave order through LDS.  Items are striped (item k of lane l of wave w is tile element
// k*256 + w*64 + l), so (k, w, l) order == input order and the scatter is stable.
#include <hipcub/hipcub.hpp>
#include "common.h"

namespace {
constexpr int RS_BITS = 8;
constexpr int RS_RADIX = 1 << RS_BITS;
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
}  // namespace

__global__ void __launch_bounds__(RS_THREADS) rs_upsweep_kernel(const int* __restrict__ keys, int n,
                                                               int shift, int nblocks,
                                                               int* __restrict__ hist) {
  __shared__ int h[RS_RADIX];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int b0 = blockIdx.x * RS_TILE;
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & (RS_RADIX - 1)], 1);
  }
  __syncthreads();
  hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

__global__ void __launch_bounds__(RS_THREADS) rs_downsweep_kernel(
    const int* __restrict__ keys_in, const int* __restrict__ vals_in, int* __restrict__ keys_out,
    int* __restrict__ vals_out, int n, int shift, int nblocks, const int* __restrict__ offs) {
  __shared__ int cnt[RS_RADIX];
  __shared__ int wcnt[4][RS_RADIX];
  __shared__ int base[RS_RADIX];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  cnt[tid] = 0;
  wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
  base[tid] = offs[tid * nblocks + blockIdx.x];
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int b0 = blockIdx.x * RS_TILE;
  // issue every load of the tile up front (no load latency inside the ranking loop)
  int kr[RS_ITEMS], vr[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + tid;
    kr[k] = i < n ? keys_in[i] : 0;
    vr[k] = i < n ? (vals_in ? vals_in[i] : i) : 0;
  }
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + tid;
    const bool valid = i < n;
    const int key = kr[k];
    const int val = vr[k];
    const int d = (key >> shift) & (RS_RADIX - 1);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < RS_BITS; ++bit) {
      const bool bset = (d >> bit) & 1;
      const unsigned long long bal = __ballot(bset);
      peers &= bset ? bal : ~bal;
    }
    const int rk = __popcll(peers & lt);
    if (valid && rk == 0) wcnt[wv][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      int r = cnt[d] + rk;
      for (int w = 0; w < wv; ++w) r += wcnt[w][d];
      const int dst = base[d] + r;
      keys_out[dst] = key;
      vals_out[dst] = val;
    }
    __syncthreads();
    cnt[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    __syncthreads();
  }
}

static inline int rs_blocks(int n) { return (n + RS_TILE - 1) / RS_TILE; }

// workspace: [hist, offs: RADIX*nblocks ints each][ping keys n][ping vals n][scan temp]
HFM_API int hfm_radix_sort_temp_bytes(int n, size_t* bytes) {
  const int nb = rs_blocks(n);
  size_t scan_tb = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tb, (const int*)nullptr, (int*)nullptr,
                                                  RS_RADIX * nb);
  *bytes = (size_t)RS_RADIX * nb * 8 + (size_t)n * 8 + scan_tb + 1024;
  return (int)e;
}

// Sort keys (< 2^end_bit) ascending; perm_out[i] = input position of the i-th smallest (stable).
HFM_API int hfm_radix_sort_ids(const int* keys_in, int* keys_out, int* perm_out, int n, int end_bit,
                               void* temp, size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  const int nb = rs_blocks(n);
  const int passes = (end_bit + RS_BITS - 1) / RS_BITS;
  char* t = (char*)temp;
  int* hist = (int*)t;
  int* offs = hist + (size_t)RS_RADIX * nb;
  t += (size_t)RS_RADIX * nb * 8;
  t = (char*)(((uintptr_t)t + 255) & ~(uintptr_t)255);
  int* pk = (int*)t;
  int* pv = pk + n;
  t = (char*)(pv + n);
  t = (char*)(((uintptr_t)t + 255) & ~(uintptr_t)255);
  size_t scan_tb = temp_bytes - (size_t)(t - (char*)temp);
  // ping-pong so that the last pass lands in (keys_out, perm_out)
  const int* ki = keys_in;
  const int* vi = nullptr;
  for (int p = 0; p < passes; ++p) {
    const bool last = (p == passes - 1);
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    int* ko = to_out ? keys_out : pk;
    int* vo = to_out ? perm_out : pv;
    (void)last;
    const int shift = p * RS_BITS;
    hipLaunchKernelGGL(rs_upsweep_kernel, dim3(nb), dim3(RS_THREADS), 0, st, ki, n, shift, nb, hist);
    size_t tb = scan_tb;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(t, tb, hist, offs, RS_RADIX * nb, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(rs_downsweep_kernel, dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n,
                       shift, nb, offs);
    ki = ko;
    vi = vo;
  }
  HFM_LAUNCH_CHECK();
}
