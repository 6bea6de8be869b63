// K3 sparse_reduce and K10 shard_route helpers.
//
// TF1 deduplicates IndexedSlices with Unique + UnsortedSegmentSum (atomics, order-dependent).
// Here: hipCUB radix sort of (id, slot) pairs restricted to ceil(log2 V) bits, gradient rows
// materialised in sorted order (fm.hip), then ReduceByKey -> one row-gradient per unique id.
// Deterministic (bitwise reproducible), atomic-free, and robust to Zipf-hot ids (a hot id
// appearing in every sample is just a long run, load-balanced by the decoupled look-back scan).
#include <hipcub/hipcub.hpp>
#include "common.h"

template <int K>
struct alignas(16) GradRowS {
  float v[K];
  float w;
  float pad[3];
};

template <int K>
struct GradSum {
  __device__ __forceinline__ GradRowS<K> operator()(const GradRowS<K>& a, const GradRowS<K>& b) const {
    GradRowS<K> r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.v[k] = a.v[k] + b.v[k];
    r.w = a.w + b.w;
    r.pad[0] = r.pad[1] = r.pad[2] = 0.f;
    return r;
  }
};

__global__ void iota_kernel(int* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}

HFM_API int hfm_sort_pairs_temp_bytes(int n, int end_bit, size_t* bytes) {
  size_t tb = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const int*)nullptr, (int*)nullptr,
                                                    (const int*)nullptr, (int*)nullptr, n, 0, end_bit);
  *bytes = tb;
  return (int)e;
}

// keys_in -> keys_out (sorted), vals_out = permutation (original slot of each sorted key).
// vals_tmp is scratch for the iota (n ints).
HFM_API int hfm_sort_ids(const int* keys_in, int* keys_out, int* vals_tmp, int* perm_out, int n,
                         int end_bit, void* temp, size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, vals_tmp, n);
  size_t tb = temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, tb, keys_in, keys_out, vals_tmp, perm_out,
                                                    n, 0, end_bit, st);
  return (int)e;
}

template <int K>
static int rbk_temp(int n, size_t* bytes) {
  size_t tb = 0;
  hipError_t e = hipcub::DeviceReduce::ReduceByKey(
      nullptr, tb, (const int*)nullptr, (int*)nullptr, (const GradRowS<K>*)nullptr,
      (GradRowS<K>*)nullptr, (int*)nullptr, GradSum<K>(), n);
  *bytes = tb;
  return (int)e;
}

template <int K>
static int rbk_run(const int* keys, const void* G, int* ukeys, void* UG, int* num, int n,
                   void* temp, size_t tb, hipStream_t st) {
  hipError_t e = hipcub::DeviceReduce::ReduceByKey(
      temp, tb, keys, ukeys, (const GradRowS<K>*)G, (GradRowS<K>*)UG, num, GradSum<K>(), n, st);
  return (int)e;
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

HFM_API int hfm_reduce_by_key_temp_bytes(int K, int n, size_t* bytes) {
#define CALL(KK) rbk_temp<KK>(n, bytes)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

// Sum gradient rows G (sorted by key) per unique key.  num -> device int (count of uniques).
HFM_API int hfm_reduce_by_key(int K, const int* sorted_keys, const void* G, int* ukeys, void* UG,
                              int* num, int n, void* temp, size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return (int)hipMemsetAsync(num, 0, sizeof(int), st);
#define CALL(KK) rbk_run<KK>(sorted_keys, G, ukeys, UG, num, n, temp, temp_bytes, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
}

// ---------------------------------------------------------------- unique + inverse
// For the row-sharded table: unique ids of the batch and, for every slot, the index of its
// id in the unique list (the forward then gathers from a compact [U, K] buffer).
__global__ void head_flags_kernel(const int* __restrict__ sk, int* __restrict__ flags, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1 : 0;
}

__global__ void unique_scatter_kernel(const int* __restrict__ sk, const int* __restrict__ perm,
                                      const int* __restrict__ seg_incl, int n,
                                      int* __restrict__ uniq, int* __restrict__ inverse,
                                      int* __restrict__ num) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = seg_incl[i] - 1;
  inverse[perm[i]] = s;
  if (i == 0 || sk[i] != sk[i - 1]) uniq[s] = sk[i];
  if (i == n - 1) *num = s + 1;
}

HFM_API int hfm_scan_temp_bytes(int n, size_t* bytes) {
  size_t tb = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, tb, (const int*)nullptr, (int*)nullptr, n);
  *bytes = tb;
  return (int)e;
}

HFM_API int hfm_unique_inverse(const int* sorted_keys, const int* perm, int n, int* flags_tmp,
                               int* seg_tmp, int* uniq, int* inverse, int* num, void* temp,
                               size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return (int)hipMemsetAsync(num, 0, sizeof(int), st);
  const int g = (n + 255) / 256;
  hipLaunchKernelGGL(head_flags_kernel, dim3(g), dim3(256), 0, st, sorted_keys, flags_tmp, n);
  size_t tb = temp_bytes;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(temp, tb, flags_tmp, seg_tmp, n, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(unique_scatter_kernel, dim3(g), dim3(256), 0, st, sorted_keys, perm, seg_tmp,
                     n, uniq, inverse, num);
  HFM_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- owner routing (K10)
// owner(id) = id % world (mod sharding spreads Zipf-hot ids over ranks); local row = id / world.
// Produces per-owner counts and the ids grouped by owner (stable) for the all-to-all.
__global__ void owner_count_kernel(const int* __restrict__ uniq, const int* __restrict__ num,
                                   int world, int* __restrict__ counts) {
  __shared__ int lc[64];
  if (threadIdx.x < 64) lc[threadIdx.x] = 0;
  __syncthreads();
  const int n = *num;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&lc[uniq[i] % world], 1);
  __syncthreads();
  if (threadIdx.x < world) atomicAdd(&counts[threadIdx.x], lc[threadIdx.x]);
}

// Since uniq is sorted ascending and owner = id % world, a stable partition by owner is done
// with one pass per owner rank (world <= 64): position = offset[o] + rank among same-owner ids.
// Implemented as: key' = (id % world) << 27-bit shift is not safe for large V, so we sort by a
// composite key computed on the fly by the caller (hfm_sort_ids on owner-major keys).
__global__ void owner_key_kernel(const int* __restrict__ uniq, const int* __restrict__ num,
                                 int max_n, int world, int* __restrict__ okey) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= max_n) return;
  okey[i] = (i < *num) ? (uniq[i] % world) : world;  // padding sorts last
}

HFM_API int hfm_owner_keys(const int* uniq, const int* num, int max_n, int world, int* okey,
                           int* counts, hipStream_t st) {
  if (max_n <= 0) return 0;
  (void)hipMemsetAsync(counts, 0, sizeof(int) * world, st);
  hipLaunchKernelGGL(owner_key_kernel, dim3((max_n + 255) / 256), dim3(256), 0, st, uniq, num, max_n,
                     world, okey);
  hipLaunchKernelGGL(owner_count_kernel, dim3(64), dim3(256), 0, st, uniq, num, world, counts);
  HFM_LAUNCH_CHECK();
}

// out[i] = src[perm[i]] for i < n (int gather), used to permute ids / rows for the exchange.
__global__ void gather_i32_kernel(const int* __restrict__ src, const int* __restrict__ perm, int n,
                                  int* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[perm[i]];
}
// Streamed-input wire format (hfm_io.cpp Loader::next with a value mask, data/pipeline.py
// _DeviceRing): a batch's values arrive as [rows, nc] -- only the nc fields of ``mask`` whose values
// are not all 1.0 -- and are expanded here, on the copy stream, into the [rows, F] layout every
// kernel reads.  One thread per output element; the shipped column of field f is the popcount of
// the mask bits below f.
__global__ __launch_bounds__(256) void expand_vals_kernel(const float* __restrict__ vc, int nc,
                                                          unsigned long long mask, int F, long n,
                                                          float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long b = i / F;
  const int f = (int)(i - b * F);
  float v = 1.0f;
  if ((mask >> f) & 1ull) v = vc[b * nc + __popcll(mask & ((1ull << f) - 1ull))];
  out[i] = v;
}

HFM_API int hfm_expand_vals(const float* vc, int nc, unsigned long long mask, int F, long rows, float* out,
                            hipStream_t st) {
  if (rows <= 0) return 0;
  if (F <= 0 || F > 64 || nc != __builtin_popcountll(mask) || (F < 64 && (mask >> F) != 0)) return (int)hipErrorInvalidValue;
  const long n = rows * F;
  hipLaunchKernelGGL(expand_vals_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, vc, nc, mask, F, n,
                     out);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_gather_i32(const int* src, const int* perm, int n, int* out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_i32_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, perm, n, out);
  HFM_LAUNCH_CHECK();
}
