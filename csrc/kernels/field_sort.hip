// Field-partitioned slot-id sort: ONE launch, one workgroup per field, sorted entirely in LDS
// (SURVEY §2.5 row 19, K3 — the "Unique + UnsortedSegmentSum" of TF1's sparse apply needs the
// B*F slot ids grouped by id, deterministically).
//
// CTR data gives every field its own id range (Criteo: 13 integer fields + 26 categorical
// vocabularies; the reference's libsvm ids, PS:74, and the per-field hashing behind
// feature_size).  When the ranges [lo_f, hi_f) are disjoint and increasing in f, the globally
// sorted slot list is the concatenation of F per-field sorted lists, each of only B keys of
// ceil(log2(hi_f - lo_f)) bits.  So instead of 4 global LSD passes over n = B*F keys (6 launches,
// each pass a decoupled look-back across the whole chip), each field is sorted by one 1024-thread
// workgroup holding its B <= 16384 (key, row) pairs in 128 KB of LDS:
//
//   * single-id fields (Criteo's integer fields: one id each) are written out directly;
//   * other fields run ceil(bits / 8) stable LSD passes of 8-bit digits in LDS.  Item k of lane l
//     of wave w is element w*64*IT + k*64 + l, so (w, k, l) order is input order.  A lane's rank
//     among same-digit lanes of its wave comes from 8 ballots; running per-digit counts live in the
//     wave's own LDS row (no block barrier inside the ranking loop); one barrier then turns the 16
//     wave rows into wave-exclusive digit offsets.  Rows beyond B carry the all-ones sentinel
//     (every digit 255) and, being last in input order, stay last.
//
// The output is bit-identical to the stable global sort (ties keep slot order b*F+f, i.e. row
// order within a field), so every downstream kernel and test is unchanged.  An id outside its
// field's declared range sets *err (the host raises on it): the concatenation would then not be
// globally sorted.
#include "common.h"

namespace {
constexpr int FS_THREADS = 1024;
constexpr int FS_WAVES = FS_THREADS / 64;
constexpr int FS_IT = 16;
constexpr int FS_MAXB = FS_THREADS * FS_IT;  // rows per field
constexpr int FS_LDS = (2 * FS_MAXB + FS_WAVES * 256 + 256 + 16) * 4;
}  // namespace

// fr: per field {lo, hi, bits}
__global__ void __launch_bounds__(FS_THREADS) field_sort_kernel(const int* __restrict__ ids, int B, int F,
                                                               const int* __restrict__ fr,
                                                               int* __restrict__ sorted_keys,
                                                               int* __restrict__ perm,
                                                               unsigned* __restrict__ err) {
  extern __shared__ __align__(16) unsigned char fs_lds_raw[];
  unsigned* lk = reinterpret_cast<unsigned*>(fs_lds_raw);  // [FS_MAXB]
  unsigned* lv = lk + FS_MAXB;                              // [FS_MAXB]
  unsigned* wc = lv + FS_MAXB;                              // [FS_WAVES][256]
  unsigned* dbase = wc + FS_WAVES * 256;                    // [256]
  unsigned* wsum = dbase + 256;                             // [4]
  const int f = blockIdx.x;
  const int lo = fr[3 * f], hi = fr[3 * f + 1], bits = fr[3 * f + 2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int* sko = sorted_keys + (size_t)f * B;
  int* pko = perm + (size_t)f * B;
  bool bad = false;
  if (bits == 0) {
    for (int b = tid; b < B; b += FS_THREADS) {
      const int id = ids[(size_t)b * F + f];
      bad |= id != lo;
      sko[b] = id;
      pko[b] = b * F + f;
    }
    if (__any(bad) && lane == 0) atomicOr(err, 1u);
    return;
  }
  const int base = wv * 64 * FS_IT;
  unsigned key[FS_IT], val[FS_IT];
#pragma unroll
  for (int k = 0; k < FS_IT; ++k) {
    const int p = base + k * 64 + lane;
    val[k] = (unsigned)p;
    key[k] = 0xFFFFFFFFu;
    if (p < B) {
      const int id = ids[(size_t)p * F + f];
      bad |= (id < lo) | (id >= hi);
      key[k] = (unsigned)(id - lo) & ((1u << bits) - 1u);
    }
  }
  if (__any(bad) && lane == 0) atomicOr(err, 1u);
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned* wh = wc + wv * 256;
  const int passes = (bits + 7) >> 3;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = pass * 8;
#pragma unroll
    for (int d = lane; d < 256; d += 64) wh[d] = 0u;
#pragma unroll
    for (int k = 0; k < FS_IT; ++k) {
      const unsigned d = (key[k] >> shift) & 255u;
      unsigned long long peers = ~0ull;
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const bool bset = (d >> bit) & 1u;
        const unsigned long long bal = __ballot(bset);
        peers &= bset ? bal : ~bal;
      }
      const unsigned rk = (unsigned)__popcll(peers & lt);
      const unsigned old = wh[d];  // a wave's LDS ops execute in order: every lane reads before
      val[k] |= (old + rk) << 16;  // the leader's update below lands.  rank < 1024, row < 2^16
      if (rk == 0) wh[d] = old + (unsigned)__popcll(peers);
    }
    __syncthreads();
    unsigned tot = 0, x = 0;
    if (tid < 256) {  // digit tid: wave-exclusive offsets, tile total
#pragma unroll
      for (int w = 0; w < FS_WAVES; ++w) {
        const unsigned c = wc[w * 256 + tid];
        wc[w * 256 + tid] = tot;
        tot += c;
      }
      x = tot;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) wsum[wv] = x;
    }
    __syncthreads();
    if (tid < 256) {
      unsigned pre = 0;
      for (int w = 0; w < wv; ++w) pre += wsum[w];
      dbase[tid] = pre + x - tot;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FS_IT; ++k) {
      const unsigned d = (key[k] >> shift) & 255u;
      const unsigned p = dbase[d] + wh[d] + (val[k] >> 16);
      lk[p] = key[k];
      lv[p] = val[k] & 0xFFFFu;
    }
    __syncthreads();
    {
      // one base address per array + immediate offsets (lv sits 64 KB in: beyond the DS offset
      // field, so per-item addresses would otherwise be hoisted into 16 registers and spilled)
      const unsigned* lkp = lk + base + lane;
      const unsigned* lvp = lv + base + lane;
#pragma unroll
      for (int k = 0; k < FS_IT; ++k) {
        key[k] = lkp[k * 64];
        val[k] = lvp[k * 64];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < FS_IT; ++k) {
    const int p = base + k * 64 + lane;
    if (p < B) {
      sko[p] = lo + (int)key[k];
      pko[p] = (int)val[k] * F + f;
    }
  }
}

HFM_API int hfm_field_sort_max_rows() { return FS_MAXB; }

// ids: [B, F] int32 (row-major slots); fr_dev: [F][3] {lo, hi, bits} on the device; outputs are
// the n = B*F sorted keys and their slot positions (field f occupies [f*B, (f+1)*B)).
HFM_API int hfm_field_sort(const int* ids, int B, int F, const int* fr_dev, int* sorted_keys, int* perm,
                           unsigned* err, hipStream_t st) {
  if (B <= 0 || F <= 0) return 0;
  if (B > FS_MAXB) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(field_sort_kernel, dim3(F), dim3(FS_THREADS), FS_LDS, st, ids, B, F, fr_dev,
                     sorted_keys, perm, err);
  HFM_LAUNCH_CHECK();
}
