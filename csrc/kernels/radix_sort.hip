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
#include <stdlib.h>

namespace {
constexpr int RS_BITS = 8;
constexpr int RS_RADIX = 1 << RS_BITS;
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
}  // namespace

// LSD passes use digits of DB = ceil(end_bit / passes) bits with passes = ceil(end_bit / 11):
// 30-bit ids (882.8M-row table) sort in 3 passes of 10 bits, 21-bit ids in 2 passes of 11 bits.
template <int DB>
__global__ void __launch_bounds__(RS_THREADS) rs_upsweep_kernel(const int* __restrict__ keys, int n,
                                                               int shift, int nblocks,
                                                               int* __restrict__ hist) {
  constexpr int RADIX = 1 << DB;
  __shared__ int h[RADIX];
  for (int d = threadIdx.x; d < RADIX; d += RS_THREADS) h[d] = 0;
  __syncthreads();
  const int b0 = blockIdx.x * RS_TILE;
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & (RADIX - 1)], 1);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < RADIX; d += RS_THREADS) hist[d * nblocks + blockIdx.x] = h[d];
}

// Downsweep: stable in-tile ranking, then the tile is reordered by digit in LDS and written
// out in LDS order, so consecutive threads store consecutive addresses of one digit's run
// (coalesced) instead of 2 scattered 4-B stores per key.
template <int DB>
__global__ void __launch_bounds__(RS_THREADS) rs_downsweep_kernel(
    const int* __restrict__ keys_in, const int* __restrict__ vals_in, int* __restrict__ keys_out,
    int* __restrict__ vals_out, int n, int shift, int nblocks, const int* __restrict__ offs) {
  constexpr int RADIX = 1 << DB;
  static_assert(RADIX == RS_THREADS, "one thread per digit");
  __shared__ int cnt[RADIX];
  __shared__ int wcnt[4][RADIX];
  __shared__ int gbase[RADIX];   // global offset of this tile's run of digit d
  __shared__ int lbase[RADIX];   // local (in-tile) exclusive offset of digit d
  __shared__ int lk[RS_TILE];
  __shared__ int lv[RS_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  cnt[tid] = 0;
  wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
  gbase[tid] = offs[tid * nblocks + blockIdx.x];
  lbase[tid] = 0;
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int b0 = blockIdx.x * RS_TILE;
  const int nloc = min(RS_TILE, n - b0);
  int kr[RS_ITEMS], vr[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + tid;
    kr[k] = i < n ? keys_in[i] : 0;
    vr[k] = i < n ? (vals_in ? vals_in[i] : i) : 0;
    if (i < n) atomicAdd(&lbase[(kr[k] >> shift) & (RADIX - 1)], 1);
  }
  __syncthreads();
  {  // exclusive scan of the tile histogram (Hillis-Steele over 256 digits)
    const int own = lbase[tid];
    for (int off = 1; off < RADIX; off <<= 1) {
      const int v = tid >= off ? lbase[tid - off] : 0;
      __syncthreads();
      lbase[tid] += v;
      __syncthreads();
    }
    lbase[tid] -= own;
    __syncthreads();
  }
  int lpos[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int i = b0 + k * RS_THREADS + tid;
    const bool valid = i < n;
    const int d = (kr[k] >> shift) & (RADIX - 1);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < DB; ++bit) {
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
      lpos[k] = lbase[d] + r;
    }
    __syncthreads();
    cnt[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
    wcnt[0][tid] = wcnt[1][tid] = wcnt[2][tid] = wcnt[3][tid] = 0;
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    if (b0 + k * RS_THREADS + tid < n) {
      lk[lpos[k]] = kr[k];
      lv[lpos[k]] = vr[k];
    }
  }
  __syncthreads();
  for (int j = tid; j < nloc; j += RS_THREADS) {
    const int key = lk[j];
    const int d = (key >> shift) & (RADIX - 1);
    const int dst = gbase[d] + (j - lbase[d]);
    keys_out[dst] = key;
    vals_out[dst] = lv[j];
  }
}

static inline int rs_blocks(int n) { return (n + RS_TILE - 1) / RS_TILE; }
static inline int rs_digit_bits(int end_bit, int* passes) {
  // 8-bit digits measured fastest on MI355X (tools/bench_sort.py): wider digits cost more in
  // the per-tile ranking than the saved pass
  int p = (end_bit + 7) / 8;
  if (p < 1) p = 1;
  *passes = p;
  return 8;
}

// workspace: [hist, offs: RADIX*nblocks ints each][ping keys n][ping vals n][scan temp]
HFM_API int hfm_radix_sort_temp_bytes(int n, size_t* bytes) {
  const int nb = rs_blocks(n);
  const size_t R = 2048;  // largest digit (11 bits)
  size_t scan_tb = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tb, (const int*)nullptr, (int*)nullptr,
                                                  (int)(R * nb));
  *bytes = R * nb * 8 + (size_t)n * 8 + scan_tb + 2048;
  return (int)e;
}

template <int DB>
static int lsd_pass(const int* ki, const int* vi, int* ko, int* vo, int n, int shift, int nb,
                    int* hist, int* offs, void* t, size_t scan_tb, hipStream_t st) {
  constexpr int RADIX = 1 << DB;
  hipLaunchKernelGGL(rs_upsweep_kernel<DB>, dim3(nb), dim3(RS_THREADS), 0, st, ki, n, shift, nb, hist);
  size_t tb = scan_tb;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(t, tb, hist, offs, RADIX * nb, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rs_downsweep_kernel<DB>, dim3(nb), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n,
                     shift, nb, offs);
  return 0;
}

// Sort keys (< 2^end_bit) ascending; perm_out[i] = input position of the i-th smallest (stable).
HFM_API int hfm_radix_sort_ids(const int* keys_in, int* keys_out, int* perm_out, int n, int end_bit,
                               void* temp, size_t temp_bytes, hipStream_t st) {
  if (n <= 0) return 0;
  const int nb = rs_blocks(n);
  int passes;
  const int db = rs_digit_bits(end_bit, &passes);
  char* t = (char*)temp;
  int* hist = (int*)t;
  int* offs = hist + (size_t)2048 * nb;
  t += (size_t)2048 * nb * 8;
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
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    int* ko = to_out ? keys_out : pk;
    int* vo = to_out ? perm_out : pv;
    const int shift = p * db;
    int rc;
    (void)db;
    rc = lsd_pass<8>(ki, vi, ko, vo, n, shift, nb, hist, offs, t, scan_tb, st);
    if (rc) return rc;
    ki = ko;
    vi = vo;
  }
  HFM_LAUNCH_CHECK();
}

// =============================================================================================
// Onesweep variant: ONE global-histogram kernel for all digit passes + ONE kernel per pass that
// ranks its tile, finds its per-digit offset with a decoupled look-back over the earlier tiles,
// and scatters.  4 passes (30-bit ids) = 1 memset + 5 launches instead of 16: inside a HIP graph
// every kernel boundary costs a few us (L2 release/acquire across the 8 XCDs, measured with
// tools/bench_launch.py), so launch count matters as much as bandwidth at this size.
//
// Inter-workgroup protocol (guide §6 Guideline 16, "R2: the data IS the flag"): each tile
// publishes, per digit, one 32-bit word {2-bit state | 30-bit count} with a relaxed agent-scope
// atomic store — state 1 = this tile's own count (aggregate), 2 = inclusive prefix through this
// tile.  A tile resolves its exclusive prefix by polling earlier tiles' words (relaxed agent
// loads) back to the first inclusive one.  Tiles are handed out by an atomic ticket, so a tile
// only ever waits on tiles already owned by running workgroups (no dispatch-order assumption).
// Spins are bounded; a timeout sets an error word instead of hanging the GPU.
// The status words and tickets are zeroed by a hipMemsetAsync node before every sort.
namespace {
constexpr int OS_ITEMS = 16;
constexpr int OS_TILE = RS_THREADS * OS_ITEMS;      // 4096 keys per tile (156 tiles at n = 640K)
constexpr unsigned OS_AGG = 1u << 30, OS_INC = 2u << 30, OS_VAL = (1u << 30) - 1;
constexpr int OS_MAX_PASSES = 4;
constexpr int OS_HIST_BLOCKS = 128;
}  // namespace

// key_lim > 0: a key outside [0, key_lim) is counted (and, in pass 0, sorted) as key_lim - 1 and
// sets *key_err -- the sorted ids then index the table in bounds and the host raises on the flag
__device__ __forceinline__ int os_clamp(int k, unsigned lim) {
  return (lim && (unsigned)k >= lim) ? (int)(lim - 1) : k;
}

__global__ void __launch_bounds__(RS_THREADS) os_hist_kernel(const int* __restrict__ keys, int n,
                                                            int passes, unsigned* __restrict__ ghist,
                                                            unsigned key_lim, unsigned* __restrict__ key_err) {
  __shared__ unsigned h[OS_MAX_PASSES][RS_RADIX];
  for (int p = 0; p < OS_MAX_PASSES; ++p) h[p][threadIdx.x] = 0;
  __syncthreads();
  bool bad = false;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int k0 = keys[i];
    const int k = os_clamp(k0, key_lim);
    bad |= k != k0;
    for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(k >> (p * RS_BITS)) & (RS_RADIX - 1)], 1u);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0 && key_err) atomicOr(key_err, 1u);
  __syncthreads();
  for (int p = 0; p < passes; ++p)
    if (h[p][threadIdx.x]) atomicAdd(&ghist[p * RS_RADIX + threadIdx.x], h[p][threadIdx.x]);
}

__global__ void __launch_bounds__(256) os_zero_kernel(unsigned* __restrict__ p, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L)
    __hip_atomic_store(&p[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive scan of one value per thread (256 threads) -> returns the exclusive prefix and
// leaves the block total in *total.  Wave-level shuffles + one LDS exchange of 4 wave sums.
__device__ __forceinline__ int block_excl_scan256(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int pre = 0;
  for (int w = 0; w < wv; ++w) pre += wsum[w];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  return pre + x - v;
}

// One onesweep pass.  Ranking is wave-private: wave w owns the contiguous quarter
// [w*64*IT, (w+1)*64*IT) of the tile and walks it 64 keys at a time, keeping running per-digit
// counts in its own LDS row (no block barrier inside the loop; a lane's rank among same-digit
// lanes comes from 8 ballots).  One barrier then turns the 4 wave rows into wave-exclusive
// offsets and the tile histogram, which is published for the look-back before the tile's
// global base is resolved.  Keys are reordered in LDS so the global stores are runs of one
// digit.
template <int IT>
__global__ void __launch_bounds__(RS_THREADS) os_pass_kernel(
    const int* __restrict__ keys_in, const int* __restrict__ vals_in, int* __restrict__ keys_out,
    int* __restrict__ vals_out, int n, int shift, const unsigned* __restrict__ ghist_p,
    unsigned* __restrict__ status, unsigned* __restrict__ ticket, unsigned* __restrict__ err,
    int debug_nolb, unsigned key_lim) {
  constexpr int TILE = RS_THREADS * IT;
  __shared__ int whist[4][RS_RADIX];
  __shared__ int lbase[RS_RADIX];
  __shared__ int gbase[RS_RADIX];
  __shared__ int wsum[4];
  __shared__ int lk[TILE];
  __shared__ int lv[TILE];
  __shared__ unsigned tile_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) tile_s = atomicAdd(ticket, 1u);
  whist[0][tid] = whist[1][tid] = whist[2][tid] = whist[3][tid] = 0;
  __syncthreads();
  const int tile = (int)tile_s;
  const int b0 = tile * TILE;
  const int w0 = b0 + wv * 64 * IT;
  int kr[IT], vr[IT], rr[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int i = w0 + k * 64 + lane;
    kr[k] = i < n ? os_clamp(keys_in[i], key_lim) : -1;
    vr[k] = i < n ? (vals_in ? vals_in[i] : i) : 0;
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  int* wh = whist[wv];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const bool valid = kr[k] >= 0;
    const int d = (kr[k] >> shift) & (RS_RADIX - 1);
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < RS_BITS; ++bit) {
      const bool bset = (d >> bit) & 1;
      const unsigned long long bal = __ballot(bset);
      peers &= bset ? bal : ~bal;
    }
    const int rk = __popcll(peers & lt);
    const int old = wh[d];                 // LDS ops of one wave execute in order: every lane
    rr[k] = old + rk;                      // reads before the leader's update below lands
    if (valid && rk == 0) wh[d] = old + __popcll(peers);
  }
  __syncthreads();
  // per digit (thread tid): wave-exclusive offsets + tile count
  const int c0 = whist[0][tid], c1 = whist[1][tid], c2 = whist[2][tid], c3 = whist[3][tid];
  const int mine = c0 + c1 + c2 + c3;
  unsigned* st = status + (size_t)tile * RS_RADIX;
  __hip_atomic_store(&st[tid], (tile == 0 ? OS_INC : OS_AGG) | (unsigned)mine, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  whist[0][tid] = 0;
  whist[1][tid] = c0;
  whist[2][tid] = c0 + c1;
  whist[3][tid] = c0 + c1 + c2;
  int tot;
  lbase[tid] = block_excl_scan256(mine, wsum, &tot);
  __syncthreads();
  // ghist was built with device atomics by os_hist_kernel: read it coherently (agent scope,
  // bypassing a possibly stale L2 line left by an earlier sort's plain read on this XCD)
  const int g = (int)__hip_atomic_load(&ghist_p[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int gex = block_excl_scan256(g, wsum + 0, &tot);
  // decoupled look-back for digit tid.  Every tile publishes its aggregate right after ranking,
  // so predecessors' words are read in batches of W independent loads (one memory round trip
  // per batch) and only a still-unpublished word is re-polled; the walk stops at the first
  // inclusive prefix.
  unsigned prefix = 0;
  if (tile > 0 && !debug_nolb) {
    constexpr int W = 64;
    int j = tile - 1;
    bool done = false;
    while (!done && j >= 0) {
      unsigned w[W];
#pragma unroll
      for (int q = 0; q < W; ++q)
        w[q] = (j - q >= 0) ? __hip_atomic_load(&status[(size_t)(j - q) * RS_RADIX + tid],
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : 0u;
#pragma unroll
      for (int q = 0; q < W; ++q) {
        if (done || j - q < 0) continue;
        unsigned v = w[q];
        unsigned spins = 0;
        while ((v & ~OS_VAL) == 0u) {
          if (++spins > (1u << 22)) { atomicExch(err, 1u); v = OS_INC; break; }
          __builtin_amdgcn_s_sleep(1);
          v = __hip_atomic_load(&status[(size_t)(j - q) * RS_RADIX + tid], __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
        }
        prefix += v & OS_VAL;
        if ((v & ~OS_VAL) == OS_INC) done = true;
      }
      j -= W;
    }
  }
  if (tile > 0)
    __hip_atomic_store(&st[tid], OS_INC | (prefix + (unsigned)mine), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  gbase[tid] = gex + (int)prefix;
  __syncthreads();
  // reorder the tile by digit in LDS, then store runs of one digit
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    if (kr[k] >= 0) {
      const int d = (kr[k] >> shift) & (RS_RADIX - 1);
      const int lp = lbase[d] + wh[d] + rr[k];
      lk[lp] = kr[k];
      lv[lp] = vr[k];
    }
  }
  __syncthreads();
  const int nloc = min(TILE, n - b0);
  for (int j = tid; j < nloc; j += RS_THREADS) {
    const int key = lk[j];
    const int d = (key >> shift) & (RS_RADIX - 1);
    const int dst = gbase[d] + (j - lbase[d]);
    keys_out[dst] = key;
    vals_out[dst] = lv[j];
  }
}

static inline int os_tiles(int n) { return (n + OS_TILE - 1) / OS_TILE; }

// workspace: [zeroed block: ghist P*256 | tickets P | err 1 | pad][status P*tiles*256][ping k][ping v]
HFM_API int hfm_onesweep_temp_bytes(int n, size_t* bytes) {
  const size_t tiles = os_tiles(n);
  *bytes = 8192 + (size_t)OS_MAX_PASSES * tiles * RS_RADIX * 4 + (size_t)n * 8 + 1024;
  return 0;
}

HFM_API int hfm_onesweep_sort_ids(const int* keys_in, int* keys_out, int* perm_out, int n, int end_bit,
                                  void* temp, size_t temp_bytes, unsigned key_lim, unsigned* key_err,
                                  hipStream_t st) {
  if (n <= 0) return 0;
  if (key_lim && key_lim - 1 >= (1u << end_bit)) return (int)hipErrorInvalidValue;
  const int tiles = os_tiles(n);
  const int passes = (end_bit + RS_BITS - 1) / RS_BITS;
  if (passes > OS_MAX_PASSES) return (int)hipErrorInvalidValue;
  size_t need;
  hfm_onesweep_temp_bytes(n, &need);
  if (temp_bytes < need) return (int)hipErrorInvalidValue;
  char* t = (char*)temp;
  unsigned* ghist = (unsigned*)t;                          // P*256
  unsigned* tickets = ghist + OS_MAX_PASSES * RS_RADIX;    // P
  unsigned* err = tickets + OS_MAX_PASSES;                 // 1
  unsigned* status = (unsigned*)(t + 8192);
  const size_t status_words = (size_t)passes * tiles * RS_RADIX;
  int* pk = (int*)(((uintptr_t)(status + (size_t)OS_MAX_PASSES * tiles * RS_RADIX) + 255) & ~(uintptr_t)255);
  int* pv = pk + n;
  // one zeroing kernel clears histogram, tickets, error word and this sort's status words (a
  // kernel, not a memset node: inside a HIP graph a memset node may be executed by a DMA
  // engine, outside the L2 coherence path the look-back relies on)
  // HIPFM_OS_DEBUG_NOLB=1: skip the look-back (WRONG order; only to time its share)
  static const int debug_nolb = getenv("HIPFM_OS_DEBUG_NOLB") ? atoi(getenv("HIPFM_OS_DEBUG_NOLB")) : 0;
  {
    const size_t words = (8192 + status_words * 4) / 4;
    int zg = (int)((words + 1023) / 1024);
    if (zg > 1024) zg = 1024;
    hipLaunchKernelGGL(os_zero_kernel, dim3(zg), dim3(256), 0, st, (unsigned*)t, (long)words);
  }
  int hg = (n + RS_THREADS - 1) / RS_THREADS;
  if (hg > OS_HIST_BLOCKS) hg = OS_HIST_BLOCKS;
  hipLaunchKernelGGL(os_hist_kernel, dim3(hg), dim3(RS_THREADS), 0, st, keys_in, n, passes, ghist, key_lim,
                     key_err);
  const int* ki = keys_in;
  const int* vi = nullptr;
  for (int p = 0; p < passes; ++p) {
    const bool to_out = ((passes - 1 - p) % 2) == 0;
    int* ko = to_out ? keys_out : pk;
    int* vo = to_out ? perm_out : pv;
    hipLaunchKernelGGL(os_pass_kernel<OS_ITEMS>, dim3(tiles), dim3(RS_THREADS), 0, st, ki, vi, ko, vo, n,
                       p * RS_BITS, ghist + p * RS_RADIX, status + (size_t)p * tiles * RS_RADIX,
                       tickets + p, err, debug_nolb, p == 0 ? key_lim : 0u);
    ki = ko;
    vi = vo;
  }
  HFM_LAUNCH_CHECK();
}

// error word of the last onesweep sort in `temp` (1 = a look-back spin timed out)
HFM_API int hfm_onesweep_error_offset() { return (OS_MAX_PASSES * RS_RADIX + OS_MAX_PASSES) * 4; }
