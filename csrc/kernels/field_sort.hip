// Field-partitioned slot-id sort (SURVEY §2.5 row 19, K3 — the "Unique + UnsortedSegmentSum"
// of TF1's sparse apply needs the B*F slot ids grouped by id, deterministically).
//
// CTR data gives every field its own id range (Criteo: 13 integer fields + 26 categorical
// vocabularies; the reference's libsvm ids, PS:74, and the per-field hashing behind
// feature_size).  When the ranges [lo_f, hi_f) are disjoint and increasing in f, the globally
// sorted slot list is the concatenation of F per-field sorted lists of B keys of
// bits_f = ceil(log2(hi_f - lo_f)) bits each.  Instead of 4 global LSD passes over n = B*F keys
// (6 launches, each pass a decoupled look-back across the chip), two launches sort everything:
//
//   fs_transpose: ids [B, F] -> field-major [F, B] (coalesced reads for every field's workgroups)
//   fs_sort:      field f is split into P_f = 2^pb_f MSD partitions by the top pb_f key bits
//                 (pb_f = min(bits_f, max_pb), chosen by the host); one 1024-thread workgroup per
//                 (field, partition):
//       1. reads all B keys of the field, counts the keys of lower partitions (= its output
//          offset) and stably compacts its own keys into LDS (ballot ranks, wave order);
//       2. sorts its m keys by the remaining bits_f - pb bits with stable LSD passes of 8-bit
//          digits in LDS: a lane's rank among same-digit lanes of its wave from 8 ballots, running
//          per-digit counts in the wave's own LDS row, one barrier to turn the 16 wave rows into
//          wave-exclusive offsets.  The m keys are striped over all 16 waves (csz = m/16 rounded
//          up to 64), so a partition of 1K keys costs each wave one 64-key step per pass;
//       3. writes its run at the partition offset.
// Batches above FS_MAXB rows per field are cut into row chunks of FS_MAXB: every (field,
// partition, chunk) workgroup sorts its chunk as above into a scratch run, then fs_merge places
// each key by merge-path ranks (its index in its own run plus, per other run, a binary-search
// count of the keys that precede it: <= for earlier chunks, < for later ones -- stable).
// Ballot ranking is VALU-bound (~10 instructions per key bit), so spreading a field over 16
// CUs instead of one is what makes the sort fast when it is on the critical path (the multi-GPU
// step, max_pb = 4: 405 workgroups at the Criteo-1TB shape); when it runs on a side stream
// concurrently with the forward (single GPU), max_pb = 0 keeps it on 39 CUs so the tower keeps
// the rest of the chip.  Single-id fields (Criteo's integer fields) need no ranking at all.
//
// Output is bit-identical to the stable global sort (ties keep row order b, i.e. slot order
// b*F+f).  An id outside its field's declared range sets *err (the host raises on it).
#include "common.h"
#include "fsort_run.h"

namespace {
constexpr int FS_THREADS = 1024;
constexpr int FS_WAVES = FS_THREADS / 64;
// 8K rows per workgroup: its LDS (2 x 32 KB keys / positions + 16 KB digit counts) leaves room
// for two tower workgroups on the same CU, so the next batch's sort co-runs with the step instead
// of waiting for whole CUs to drain (at 16K rows a 148 KB sort workgroup needed an EMPTY CU)
constexpr int FS_IT = 8;
constexpr int FS_MAXB = FS_THREADS * FS_IT;  // rows per field
constexpr int FS_PBMAX = 4;                   // up to 16 partitions per field
constexpr int FS_MAXCHUNK = 32;               // row chunks per field (batches up to 256K)
constexpr int FS_LDS = (2 * FS_MAXB + FS_WAVES * 256 + 256 + 64) * 4;
}  // namespace

__global__ void __launch_bounds__(256) fs_transpose_kernel(const int* __restrict__ ids, int B, int F,
                                                          int* __restrict__ idsT) {
  __shared__ int t[64][65];
  const int b0 = blockIdx.x * 64;
  const int nb = min(64, B - b0);
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int nf = min(64, F - f0);
    for (int e = threadIdx.x; e < nb * nf; e += 256) {
      const int b = e / nf, f = e - b * nf;
      t[f][b] = ids[(size_t)(b0 + b) * F + f0 + f];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * nf; e += 256) {
      const int f = e / nb, b = e - f * nb;
      idsT[(size_t)(f0 + f) * B + b0 + b] = t[f][b];
    }
    __syncthreads();
  }
}

// fr: per field {lo, hi, bits, pb}; work: per workgroup {field, partition, chunk}; ids are
// field-major [F, B]; outputs land at [f * B + chunk * FS_MAXB, ...) (the final arrays when there
// is one chunk, the runs fs_merge reads otherwise).
__global__ void __launch_bounds__(FS_THREADS) fs_sort_kernel(const int* __restrict__ ids, int Btot, int F,
                                                            const int* __restrict__ fr,
                                                            const int* __restrict__ work,
                                                            int* __restrict__ sorted_keys,
                                                            int* __restrict__ perm,
                                                            unsigned* __restrict__ err) {
  extern __shared__ __align__(16) unsigned char fs_lds_raw[];
  unsigned* lk = reinterpret_cast<unsigned*>(fs_lds_raw);  // [FS_MAXB]
  unsigned* lv = lk + FS_MAXB;                              // [FS_MAXB]
  unsigned* wc = lv + FS_MAXB;                              // [FS_WAVES][256]
  unsigned* dbase = wc + FS_WAVES * 256;                    // [256]
  unsigned* wsum = dbase + 256;                             // [16]
  unsigned* wlow = wsum + 16;                               // [16]
  const int f = work[3 * blockIdx.x], part = work[3 * blockIdx.x + 1];
  const int row0 = work[3 * blockIdx.x + 2] * FS_MAXB;
  const int B = min(FS_MAXB, Btot - row0);
  const int lo = fr[4 * f], hi = fr[4 * f + 1], bits = fr[4 * f + 2], pb = fr[4 * f + 3];
  const int rb = bits - pb;  // bits sorted inside the partition
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int* sko = sorted_keys + (size_t)f * Btot + row0;
  int* pko = perm + (size_t)f * Btot + row0;
  const int* src = ids + (size_t)f * Btot + row0;
  bool bad = false;
  if (bits == 0) {
    for (int b = tid; b < B; b += FS_THREADS) {
      const int id = src[b];
      bad |= id != lo;
      sko[b] = id;
      pko[b] = (row0 + b) * F + f;
    }
    if (__any(bad) && lane == 0) atomicOr(err, 1u);
    return;
  }
  // ---- 1. partition: count lower partitions, stably compact this partition's keys
  const int base = wv * 64 * FS_IT;
  unsigned key[FS_IT];
  unsigned mine_bits = 0;
  unsigned my_cnt = 0, low_cnt = 0;
#pragma unroll
  for (int k = 0; k < FS_IT; ++k) {
    const int p = base + k * 64 + lane;
    key[k] = 0u;
    int kp = 1 << 30;
    if (p < B) {
      const int id = src[p];
      bad |= (id < lo) | (id >= hi);
      key[k] = (unsigned)(id - lo) & ((1u << bits) - 1u);
      kp = (int)(key[k] >> rb);
    }
    const unsigned long long bm = __ballot(kp == part);
    const unsigned long long bl = __ballot(kp < part);
    if (kp == part) mine_bits |= 1u << k;
    my_cnt += (unsigned)__popcll(bm);
    low_cnt += (unsigned)__popcll(bl);
  }
  if (__any(bad) && lane == 0) atomicOr(err, 1u);
  if (lane == 0) {
    wsum[wv] = my_cnt;
    wlow[wv] = low_cnt;
  }
  __syncthreads();
  unsigned woff = 0, m = 0, out_base = 0;
  for (int w = 0; w < FS_WAVES; ++w) {
    const unsigned c = wsum[w];
    if (w < wv) woff += c;
    m += c;
    out_base += wlow[w];
  }
  {
    unsigned run = woff;
#pragma unroll
    for (int k = 0; k < FS_IT; ++k) {
      const bool mine = (mine_bits >> k) & 1u;
      const unsigned long long bm = __ballot(mine);
      if (mine) {
        const unsigned q = run + (unsigned)__popcll(bm & lt);
        lk[q] = key[k] & ((1u << rb) - 1u);
        lv[q] = (unsigned)(base + k * 64 + lane);
      }
      run += (unsigned)__popcll(bm);
    }
  }
  __syncthreads();
  // ---- 2. LSD passes over the rb low bits; the m keys striped over all waves
  const int csz = (((int)m + FS_WAVES * 64 - 1) / (FS_WAVES * 64)) * 64;  // keys per wave (x64)
  const int its = csz / 64;
  const int wb = wv * csz;
  unsigned val[FS_IT];
  {
    const unsigned* lkp = lk + wb + lane;
    const unsigned* lvp = lv + wb + lane;
#pragma unroll
    for (int k = 0; k < FS_IT; ++k) {
      const bool in = k < its && wb + k * 64 + lane < (int)m;
      key[k] = in ? lkp[k * 64] : 0xFFFFFFFFu;
      val[k] = in ? lvp[k * 64] : 0u;
    }
  }
  unsigned* wh = wc + wv * 256;
  const int passes = (rb + 7) >> 3;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = pass * 8;
    __syncthreads();  // everyone's previous reloads are done before the LDS arrays are rewritten
#pragma unroll
    for (int d = lane; d < 256; d += 64) wh[d] = 0u;
#pragma unroll
    for (int k = 0; k < FS_IT; ++k) {
      if (k >= its) break;  // wave-uniform
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
      val[k] |= (old + rk) << 16;  // the update below lands (all peers store the same value).
      wh[d] = old + (unsigned)__popcll(peers);  // rank < 1024, row < 2^16
    }
    __syncthreads();
    unsigned tot = 0, x = 0;
    if (tid < 256) {  // digit tid: wave-exclusive offsets, total
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
      if (k >= its) break;
      const unsigned d = (key[k] >> shift) & 255u;
      const unsigned p = dbase[d] + wh[d] + (val[k] >> 16);
      lk[p] = key[k];
      lv[p] = val[k] & 0xFFFFu;
    }
    __syncthreads();
    {
      const unsigned* lkp = lk + wb + lane;
      const unsigned* lvp = lv + wb + lane;
#pragma unroll
      for (int k = 0; k < FS_IT; ++k) {
        if (k >= its) break;
        key[k] = lkp[k * 64];
        val[k] = lvp[k * 64];
      }
    }
  }
  // ---- 3. write the partition's run (sentinels sort last, so [0, m) are the real keys)
  const int kbase = lo + (part << rb);
#pragma unroll
  for (int k = 0; k < FS_IT; ++k) {
    if (k >= its) break;
    const int q = wb + k * 64 + lane;
    if (q < (int)m) {
      sko[out_base + q] = min(kbase + (int)key[k], hi - 1);   // (out-of-field ids: flagged, kept valid)
      pko[out_base + q] = (row0 + (int)(val[k] & 0xFFFFu)) * F + f;
    }
  }
}

// runs of FS_MAXB sorted keys per field (the last one shorter) -> one sorted list per field
__global__ void __launch_bounds__(256) fs_merge_kernel(const int* __restrict__ rk, const int* __restrict__ rp,
                                                      int B, int* __restrict__ sko, int* __restrict__ pko) {
  const int f = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= B) return;
  const int* keys = rk + (size_t)f * B;
  const int c = e / FS_MAXB;
  const int k = keys[e];
  int pos = e - c * FS_MAXB;
  const int nrun = (B + FS_MAXB - 1) / FS_MAXB;
  for (int r = 0; r < nrun; ++r) {
    if (r == c) continue;
    const int* run = keys + r * FS_MAXB;
    int lo = 0, hi = min(FS_MAXB, B - r * FS_MAXB);
    while (lo < hi) {  // first index whose key is > k (earlier runs) or >= k (later runs)
      const int mid = (lo + hi) >> 1;
      const int v = run[mid];
      if (r < c ? v <= k : v < k) lo = mid + 1; else hi = mid;
    }
    pos += lo;
  }
  sko[(size_t)f * B + pos] = k;
  pko[(size_t)f * B + pos] = rp[(size_t)f * B + e];
}

// Run-level sort (fsort_run.h): items are (job, work item) pairs over the run's batches
__global__ void __launch_bounds__(FS2_THREADS) fs2_sort_run_kernel(const FsJob* __restrict__ jobs,
                                                                   const int* __restrict__ items) {
  extern __shared__ __align__(16) unsigned char lds[];
  const FsJob J = jobs[items[2 * blockIdx.x]];
  fs2_sort_item(J, items[2 * blockIdx.x + 1], lds);
}

__global__ void __launch_bounds__(FSM_THREADS) fs2_merge_run_kernel(const FsJob* __restrict__ jobs,
                                                                    const int* __restrict__ items) {
  extern __shared__ int stage[];
  const FsJob J = jobs[items[2 * blockIdx.x]];
  fs2_merge_item(J, items[2 * blockIdx.x + 1], stage);
}

// jobs: [njobs] device FsJobs (one per batch; B <= 8 chunks); items: [nitems][2] {job, sort item};
// mitems: [nmitems][2] {job, merge workgroup}
HFM_API int hfm_field_sort_run(const FsJob* jobs, const int* items, int nitems, const int* mitems, int nmitems,
                               hipStream_t st) {
  if (!jobs || !items || nitems <= 0 || nmitems < 0 || (nmitems && !mitems)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fs2_sort_run_kernel, dim3(nitems), dim3(FS2_THREADS), FS2_LDS, st, jobs, items);
  if (nmitems)
    hipLaunchKernelGGL(fs2_merge_run_kernel, dim3(nmitems), dim3(FSM_THREADS), FS2_MAXB * 4, st, jobs, mitems);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_fs_job_bytes() { return (int)sizeof(FsJob); }

HFM_API int hfm_fs2_chunk_rows() { return FS2_MAXB; }

HFM_API int hfm_fs2_merge_wgs_per_run() { return FSM_WPR; }

HFM_API int hfm_field_sort_max_rows() { return FS_MAXB * FS_MAXCHUNK; }

HFM_API int hfm_field_sort_chunk_rows() { return FS_MAXB; }

HFM_API int hfm_field_sort_max_pb() { return FS_PBMAX; }

// the sort of field-major ids [F, B]: one launch, plus the merge when B > FS_MAXB (runs in rk/rp,
// [F, B] each; unused otherwise)
static int fs_sort_launch(const int* idsT, int B, int F, const int* fr_dev, const int* work_dev, int nwork,
                          int* rk, int* rp, int* sorted_keys, int* perm, unsigned* err, hipStream_t st) {
  const bool merge = B > FS_MAXB;
  if (merge && (!rk || !rp)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fs_sort_kernel, dim3(nwork), dim3(FS_THREADS), FS_LDS, st, idsT, B, F, fr_dev, work_dev,
                     merge ? rk : sorted_keys, merge ? rp : perm, err);
  if (merge)
    hipLaunchKernelGGL(fs_merge_kernel, dim3((B + 255) / 256, F), dim3(256), 0, st, rk, rp, B, sorted_keys, perm);
  HFM_LAUNCH_CHECK();
}

// ids: [B, F] int32 (row-major slots); fr_dev: [F][4] {lo, hi, bits, pb}; work_dev: [nwork][3]
// {field, partition, chunk}; idsT: [F, B] scratch; rk / rp: [F, B] scratch runs (B > FS_MAXB).
// Outputs: the n = B*F sorted keys and their slot positions (field f occupies [f*B, (f+1)*B)).
HFM_API int hfm_field_sort(const int* ids, int B, int F, const int* fr_dev, const int* work_dev, int nwork,
                           int* idsT, int* rk, int* rp, int* sorted_keys, int* perm, unsigned* err,
                           hipStream_t st) {
  if (B <= 0 || F <= 0) return 0;
  if (B > FS_MAXB * FS_MAXCHUNK) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(fs_transpose_kernel, dim3((B + 63) / 64), dim3(256), 0, st, ids, B, F, idsT);
  return fs_sort_launch(idsT, B, F, fr_dev, work_dev, nwork, rk, rp, sorted_keys, perm, err, st);
}

// Same sort from ids the FM forward already wrote field-major (hfm_fm_fwd's idsT).
HFM_API int hfm_field_sort_pre(const int* idsT, int B, int F, const int* fr_dev, const int* work_dev,
                               int nwork, int* rk, int* rp, int* sorted_keys, int* perm, unsigned* err,
                               hipStream_t st) {
  if (B <= 0 || F <= 0) return 0;
  if (B > FS_MAXB * FS_MAXCHUNK) return (int)hipErrorInvalidValue;
  return fs_sort_launch(idsT, B, F, fr_dev, work_dev, nwork, rk, rp, sorted_keys, perm, err, st);
}
