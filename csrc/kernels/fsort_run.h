// Run-level per-field slot sort (field_sort.hip has the algorithm and the
// per-step side-stream form): the slot sorts of ALL batches of a multi-step graph as two launches
// at the graph's start, so the steps that follow run back to back on one queue.
//
// Why: on one GPU the next batch's sort ran on a graph side branch next to each step.  Its kernels
// share the CUs with the latency-bound tower and sparse launches, and joining the branch back
// costs the step ~10 us: the next step's first kernel waits on a cross-queue barrier packet even
// when the branch finished earlier (profiles/r3c_side_kernels.md: 10.3 us from one step's end to
// the next tower; ~0 between two kernels of one queue).  Sorting the steps' batches inside the
// steps' own launches instead removes the gap but the sort workgroups then stretch the launch
// that hosts them by more (tower +9 us, or sparse +45 us: profiles/r3c_inl_kernels.md) -- a
// sort workgroup co-running with a full launch gets a fraction of its SIMDs and its ballot / LDS
// chains are latency-bound.  Up front, the run's sorts have the chip to themselves.
//
//   sort launch:   one 1024-thread workgroup per (batch, field, 16K-row chunk): stable LSD passes
//                  of 4-bit digits in LDS with per-(digit, thread) counter ranks (fs2_sort_item;
//                  the round-3 8-bit wave-ballot form, fs2_sort_item_ballot, stays for A/B), ids
//                  read row-major or field-major (no transpose launch).  A single chunk (B <= 16K)
//                  or a single-id field writes the final arrays; else the chunk's run.
//   merge launch:  (B > 16K only) FSM_WPR 256-thread workgroups per (batch, multi-id field, chunk
//                  run): merge-path placement of
//                  every key (fs_merge_kernel's rule: own index + per other run the count of keys
//                  before it, <= for earlier runs, < for later ones -- stable), the other runs
//                  staged in LDS one at a time.
// Output is bit-identical to the per-step field sort (and to the stable global sort).
#pragma once
#include <type_traits>
#include "common.h"

// sort: 1024-thread workgroups over 16K-row chunks (one workgroup per CU -- the run's sort has the
// chip to itself), so a batch of up to 16K rows needs no merge at all
constexpr int FS2_THREADS = 1024;
constexpr int FS2_WAVES = FS2_THREADS / 64;
constexpr int FS2_MAXB = 16384;
constexpr int FS2_IT = FS2_MAXB / FS2_THREADS;      // keys per thread
constexpr int FS2_WROWS = FS2_MAXB / FS2_WAVES;     // positions per wave (ballot form)
// counter-rank form (fs2_sort_item): 4-bit digits; LDS: keys u32 [16K], row indices u16 [16K]
// (both position-swizzled), per-(digit, thread) counters u16 [16][1024], wave sums u32 [16]
constexpr int FS2_RB = 4;
constexpr int FS2_ND = 1 << FS2_RB;
constexpr int FS2_LDS = FS2_MAXB * 4 + FS2_MAXB * 2 + FS2_ND * FS2_THREADS * 2 + FS2_WAVES * 4;
// ballot form (fs2_sort_item_ballot, kept for tools/fsbench A/B): 8-bit digits; keys u32 [16K],
// row indices u16 [16K], per-wave digit counts u16 [16][256], digit bases u16 [256], wave sums u32 [4]
constexpr int FS2_LDS_BALLOT = FS2_MAXB * 4 + FS2_MAXB * 2 + FS2_WAVES * 256 * 2 + 256 * 2 + 4 * 4;
// merge (batches above one chunk): 256-thread workgroups, 8 keys per thread each
constexpr int FSM_THREADS = 256;
constexpr int FSM_EPT = 8;
constexpr int FSM_WPR = FS2_MAXB / (FSM_THREADS * FSM_EPT);  // merge workgroups per chunk run

struct FsJob {
  const int* ids;    // batch ids: row-major [B, F] (ld = 0) or field-major (ld = a field's stride)
  int ld;
  int B, F;
  const int* fr;     // [F][4] {lo, hi, bits, pb} (pb unused here)
  const int* work;   // [nwork][2] {field, chunk}: one sort workgroup each
  int nwork;
  int* rk;           // [F, B] chunk runs of FS2_MAXB rows (B > FS2_MAXB)
  int* rp;
  int* keys;         // [F * B] sorted keys (field f at [f*B, (f+1)*B))
  int* perm;         // [F * B] slot position b*F + f of each sorted key
  unsigned* err;     // set when an id lies outside its field's range
  const int* mfields;  // fields that need the merge (bits > 0, B > FS2_MAXB)
  int nmf;
  int mwpf;          // merge workgroups per field (FSM_WPR per chunk run)
  int* inv;          // [F][B] or null: sorted index of slot (b, f) at inv[f * B + b] (the inverse
                     // of perm, field-major: each sort workgroup's writes stay inside its field's
                     // B ints; the tower writes each slot's gradient row to its sorted position)
};

// one (field, chunk) work item, ballot ranks; lds: FS2_LDS_BALLOT bytes.  The keys live in LDS
// between passes and each pass holds at most 16 keys + 16 packed (row, position) words per lane.
// Each 8-bit pass ranks a key among the same-digit keys of its wave with 8 ballots (~6 VALU per
// key bit): 12 us per pass per workgroup, 55 us for a 28-bit field (profiles/r3f_fs2_bench.log).
__device__ __forceinline__ void fs2_sort_item_ballot(const FsJob& J, int item, unsigned char* lds) {
  unsigned* lk = reinterpret_cast<unsigned*>(lds);
  unsigned short* lv = reinterpret_cast<unsigned short*>(lk + FS2_MAXB);
  unsigned short* wc = lv + FS2_MAXB;
  unsigned short* dbase = wc + FS2_WAVES * 256;
  unsigned* wsum = reinterpret_cast<unsigned*>(dbase + 256);
  const int f = J.work[2 * item], row0 = J.work[2 * item + 1] * FS2_MAXB;
  const int B = min(FS2_MAXB, J.B - row0);
  if (B <= 0) return;
  const int F = J.F;
  const int lo = J.fr[4 * f], hi = J.fr[4 * f + 1], bits = J.fr[4 * f + 2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int* src = J.ld ? J.ids + (size_t)f * J.ld + row0 : J.ids + (size_t)row0 * F + f;
  const int sst = J.ld ? 1 : F;
  bool bad = false;
  if (bits == 0) {  // single-id field: row order is the sorted order; final arrays directly
    int* sk = J.keys + (size_t)f * J.B + row0;
    int* pk = J.perm + (size_t)f * J.B + row0;
    int idv[FS2_IT];
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int b = k * FS2_THREADS + tid;
      idv[k] = b < B ? src[(size_t)b * sst] : lo;
    }
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int b = k * FS2_THREADS + tid;
      if (b < B) {
        bad |= idv[k] != lo;
        sk[b] = idv[k];
        pk[b] = (row0 + b) * F + f;
        if (J.inv) J.inv[(size_t)f * J.B + row0 + b] = f * J.B + row0 + b;
      }
    }
    if (__any(bad) && lane == 0) atomicOr(J.err, 1u);
    return;
  }
  const bool direct = J.B <= FS2_MAXB;
  int* sko = (direct ? J.keys : J.rk) + (size_t)f * J.B + row0;
  int* pko = (direct ? J.perm : J.rp) + (size_t)f * J.B + row0;
  const unsigned mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int wb = wv * FS2_WROWS;  // this wave's block of positions (row order)
  // keys into LDS in row order (sentinels past B sort last: their digit is 255 in every pass and
  // they start after every real key -- field_sort.hip)
  {
    // every load in flight before the first LDS store (a load-store loop waited out one HBM
    // round trip per iteration: ~60 us per workgroup instead of ~15)
    int idv[FS2_IT];
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int p = k * FS2_THREADS + tid;
      idv[k] = p < B ? src[(size_t)p * sst] : lo;
    }
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int p = k * FS2_THREADS + tid;
      unsigned key = 0xFFFFFFFFu;
      if (p < B) {
        bad |= (idv[k] < lo) | (idv[k] >= hi);
        key = (unsigned)(idv[k] - lo) & mask;
      }
      lk[p] = key;
      lv[p] = (unsigned short)p;
    }
  }
  if (__any(bad) && lane == 0) atomicOr(J.err, 1u);
  unsigned short* wh = wc + wv * 256;
  const int passes = (bits + 7) >> 3;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = pass * 8;
    __syncthreads();  // the key arrays are complete (initial fill / previous scatter)
#pragma unroll
    for (int d = lane; d < 256; d += 64) wh[d] = 0;
    // 1. ranks among same-digit keys of the wave block, in position order (8 ballots per key)
    unsigned rk2[FS2_IT / 2];  // two 16-bit ranks per register
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const unsigned d = (lk[wb + k * 64 + lane] >> shift) & 255u;
      unsigned long long peers = ~0ull;
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const bool bset = (d >> bit) & 1u;
        const unsigned long long bal = __ballot(bset);
        peers &= bset ? bal : ~bal;
      }
      const unsigned old = wh[d];  // (a wave's LDS ops run in order; all peers store one value)
      const unsigned r = old + (unsigned)__popcll(peers & lt);
      if (k & 1) rk2[k >> 1] |= r << 16;
      else rk2[k >> 1] = r;
      wh[d] = (unsigned short)(old + (unsigned)__popcll(peers));
    }
    __syncthreads();
    // 2. digit tid (the first 4 waves): wave-exclusive offsets and the digit total, then bases
    unsigned tot = 0, x = 0;
    if (tid < 256) {
#pragma unroll
      for (int w = 0; w < FS2_WAVES; ++w) {
        const unsigned c = wc[w * 256 + tid];
        wc[w * 256 + tid] = (unsigned short)tot;
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
      dbase[tid] = (unsigned short)(pre + x - tot);
    }
    __syncthreads();
#pragma unroll
    for (int d = lane; d < 256; d += 64) wh[d] = (unsigned short)(wh[d] + dbase[d]);  // own row

    // 3. read the block, then (after everyone has read) scatter it to its new positions
    unsigned key[FS2_IT], vp[FS2_IT];
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int q = wb + k * 64 + lane;
      key[k] = lk[q];
      const unsigned d = (key[k] >> shift) & 255u;
      const unsigned r = (k & 1) ? (rk2[k >> 1] >> 16) : (rk2[k >> 1] & 0xFFFFu);
      vp[k] = (unsigned)lv[q] | (((unsigned)wh[d] + r) << 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const unsigned p = vp[k] >> 16;
      lk[p] = key[k];
      lv[p] = (unsigned short)(vp[k] & 0xFFFFu);
    }
  }
  __syncthreads();
  for (int q = tid; q < B; q += FS2_THREADS) {  // sentinels sit past B
    sko[q] = min(lo + (int)lk[q], hi - 1);   // (an id outside its field -- flagged above -- stays a valid row)
    pko[q] = (row0 + (int)lv[q]) * F + f;
    if (direct && J.inv) J.inv[(size_t)f * J.B + row0 + (int)lv[q]] = f * J.B + row0 + q;
  }
}

// inclusive wave64 prefix sum in DPP steps: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast 15 / 31 carry the row totals up (no LDS round trips, unlike a shuffle scan)
__device__ __forceinline__ unsigned fs2_wave_incl_scan(unsigned x) {
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// LDS word of sort position p: rotated inside its 16-word block by p / 64, so that the blocked
// reads below (thread t reads positions 16 t + j, j fixed per instruction) hit 64 distinct banks
__device__ __forceinline__ int fs2_swz(int p) { return (p & ~15) | ((p + (p >> 6)) & 15); }

// one (field, chunk) work item, counter ranks; lds: FS2_LDS bytes.  Stable LSD passes of 4-bit
// digits over a blocked arrangement: thread t holds the keys at positions [t ipt, t ipt + ipt)
// (ipt = keys per thread, the smallest power of two with 1024 ipt >= B).  Per pass:
//   count:   each key increments its thread's counter for its digit (a column of the [16 digits]
//            [1024 threads] u16 counter table no other thread touches); the value before the
//            increment is the key's rank among its thread's earlier same-digit keys;
//   scan:    one exclusive scan of the table in (digit, thread) order -- thread t rakes 16
//            consecutive counters, a wave scan and the 16 wave sums;
//   scatter: key -> counter (now: # keys of lower digits + same-digit keys of lower threads) +
//            its rank; then the blocked keys are read back for the next pass.
// A key costs ~4 VALU and 6 LDS accesses per 4-bit pass instead of ~48 VALU of ballots per 8-bit
// pass.  Output is bit-identical to the ballot form (both are the stable sort).
__device__ __forceinline__ void fs2_sort_item(const FsJob& J, int item, unsigned char* lds) {
  unsigned* lk = reinterpret_cast<unsigned*>(lds);
  unsigned short* lv = reinterpret_cast<unsigned short*>(lk + FS2_MAXB);
  unsigned short* cnt = lv + FS2_MAXB;                       // [FS2_ND][FS2_THREADS]
  unsigned* wsum = reinterpret_cast<unsigned*>(cnt + FS2_ND * FS2_THREADS);
  const int f = J.work[2 * item], row0 = J.work[2 * item + 1] * FS2_MAXB;
  const int B = min(FS2_MAXB, J.B - row0);
  if (B <= 0) return;
  const int F = J.F;
  const int lo = J.fr[4 * f], hi = J.fr[4 * f + 1], bits = J.fr[4 * f + 2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int* src = J.ld ? J.ids + (size_t)f * J.ld + row0 : J.ids + (size_t)row0 * F + f;
  const int sst = J.ld ? 1 : F;
  bool bad = false;
  if (bits == 0) {  // single-id field: row order is the sorted order; final arrays directly
    int* sk = J.keys + (size_t)f * J.B + row0;
    int* pk = J.perm + (size_t)f * J.B + row0;
    int idv[FS2_IT];
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int b = k * FS2_THREADS + tid;
      idv[k] = b < B ? src[(size_t)b * sst] : lo;
    }
#pragma unroll
    for (int k = 0; k < FS2_IT; ++k) {
      const int b = k * FS2_THREADS + tid;
      if (b < B) {
        bad |= idv[k] != lo;
        sk[b] = idv[k];
        pk[b] = (row0 + b) * F + f;
        if (J.inv) J.inv[(size_t)f * J.B + row0 + b] = f * J.B + row0 + b;
      }
    }
    if (__any(bad) && lane == 0) atomicOr(J.err, 1u);
    return;
  }
  const bool direct = J.B <= FS2_MAXB;
  int* sko = (direct ? J.keys : J.rk) + (size_t)f * J.B + row0;
  int* pko = (direct ? J.perm : J.rp) + (size_t)f * J.B + row0;
  const unsigned mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  const int ipt = B <= 1024 ? 1 : B <= 2048 ? 2 : B <= 4096 ? 4 : B <= 8192 ? 8 : 16;
  const int np = ((B + ipt - 1) / ipt) * ipt;   // positions in use (sentinels in [B, np))
  const bool act = tid * ipt < np;              // this thread holds keys
  const int p0 = tid * ipt;
  unsigned short* mc = cnt + tid;               // this thread's counter column (stride FS2_THREADS)
  const int passes = (bits + FS2_RB - 1) / FS2_RB;
  // PACK (keys of <= 18 bits): key and row index travel as one word (key << 14 | row), so a pass
  // moves one LDS array instead of two; else keys u32 in lk, row indices u16 in lv.
  auto body = [&](auto pack_tag) {
    constexpr bool PACK = decltype(pack_tag)::value;
    constexpr int KS = PACK ? 14 : 0;           // key bit offset inside an element
    // keys (coalesced, row order) into LDS; sentinels past B sort last: their digit is all ones
    // in every pass, and they start after every real key.  Counters zeroed.
    {
      int idv[FS2_IT];
#pragma unroll
      for (int k = 0; k < FS2_IT; ++k) {
        const int p = k * FS2_THREADS + tid;
        idv[k] = p < B ? src[(size_t)p * sst] : lo;
      }
#pragma unroll
      for (int k = 0; k < FS2_IT; ++k) {
        const int p = k * FS2_THREADS + tid;
        if (p < np) {
          unsigned e = 0xFFFFFFFFu;
          if (p < B) {
            bad |= (idv[k] < lo) | (idv[k] >= hi);
            e = PACK ? ((((unsigned)(idv[k] - lo) & mask) << KS) | (unsigned)p) : ((unsigned)(idv[k] - lo) & mask);
          }
          lk[fs2_swz(p)] = e;
          if (!PACK) lv[fs2_swz(p)] = (unsigned short)p;
        }
      }
      uint4* cz = reinterpret_cast<uint4*>(cnt);
      for (int i = tid; i < FS2_ND * FS2_THREADS / 8; i += FS2_THREADS) cz[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (__any(bad) && lane == 0) atomicOr(J.err, 1u);
    __syncthreads();
    unsigned kr[FS2_IT], vr[FS2_IT];
#pragma unroll
    for (int j = 0; j < FS2_IT; ++j) {
      kr[j] = 0xFFFFFFFFu;
      vr[j] = 0u;
      if (act && j < ipt) {
        kr[j] = lk[fs2_swz(p0 + j)];
        vr[j] = (unsigned)(p0 + j);
      }
    }
    for (int pass = 0; pass < passes; ++pass) {
      const int shift = KS + pass * FS2_RB;
      // 1. count (own column only: the read-increment-write of one thread's keys run in order)
      unsigned lr[FS2_IT];
#pragma unroll
      for (int j = 0; j < FS2_IT; ++j) {
        lr[j] = 0u;
        if (act && j < ipt) {
          const unsigned d = (kr[j] >> shift) & (FS2_ND - 1);
          const unsigned c = mc[d * FS2_THREADS];
          lr[j] = c;
          mc[d * FS2_THREADS] = (unsigned short)(c + 1u);
        }
      }
      __syncthreads();
      // 2. exclusive scan of the table in (digit, thread) order: thread t owns counters [16 t, 16 t + 16)
      {
        uint4* cw = reinterpret_cast<uint4*>(cnt) + 2 * tid;
        const uint4 a = cw[0], b = cw[1];
        const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        unsigned sum = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += (w[i] & 0xFFFFu) + (w[i] >> 16);
        const unsigned x = fs2_wave_incl_scan(sum);
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        unsigned run = x - sum;
        const uint4* ws4 = reinterpret_cast<const uint4*>(wsum);
#pragma unroll
        for (int v4 = 0; v4 < FS2_WAVES / 4; ++v4) {
          const uint4 q = ws4[v4];   // (one address for the whole wave: a broadcast read)
          run += (4 * v4 < wv ? q.x : 0u) + (4 * v4 + 1 < wv ? q.y : 0u) + (4 * v4 + 2 < wv ? q.z : 0u) +
                 (4 * v4 + 3 < wv ? q.w : 0u);
        }
        unsigned o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned e0 = run, e1 = run + (w[i] & 0xFFFFu);
          run = e1 + (w[i] >> 16);
          o[i] = e0 | (e1 << 16);   // offsets <= 16384
        }
        cw[0] = make_uint4(o[0], o[1], o[2], o[3]);
        cw[1] = make_uint4(o[4], o[5], o[6], o[7]);
      }
      __syncthreads();
      // 3. scatter to the new positions, then clear this thread's column for the next pass
      if (act) {
#pragma unroll
        for (int j = 0; j < FS2_IT; ++j) {
          if (j < ipt) {
            const unsigned d = (kr[j] >> shift) & (FS2_ND - 1);
            const int q = fs2_swz((int)(mc[d * FS2_THREADS] + lr[j]));
            lk[q] = kr[j];
            if (!PACK) lv[q] = (unsigned short)vr[j];
          }
        }
      }
      // (every thread, holding keys or not: the scan wrote offsets into every column)
#pragma unroll
      for (int d = 0; d < FS2_ND; ++d) mc[d * FS2_THREADS] = 0;
      __syncthreads();
      if (act && pass + 1 < passes) {
#pragma unroll
        for (int j = 0; j < FS2_IT; ++j) {
          if (j < ipt) {
            const int q = fs2_swz(p0 + j);
            kr[j] = lk[q];
            if (!PACK) vr[j] = lv[q];
          }
        }
      }
    }
    for (int q = tid; q < B; q += FS2_THREADS) {  // sentinels sit past B
      const int sq = fs2_swz(q);
      const unsigned e = lk[sq];
      const int key = (int)(e >> KS), row = PACK ? (int)(e & 0x3FFFu) : (int)lv[sq];
      sko[q] = min(lo + key, hi - 1);   // (an id outside its field -- flagged above -- stays a valid row)
      pko[q] = (row0 + row) * F + f;
      if (direct && J.inv) J.inv[(size_t)f * J.B + row0 + row] = f * J.B + row0 + q;
    }
  };
  if (bits <= 32 - 14) body(std::true_type{});
  else body(std::false_type{});
}

// merge workgroup `wg` of the multi-chunk fields: half of run c of field mfields[wg / (2 nrun)] (runs in
// rk / rp -> final keys / perm).  Each other run is staged in LDS (`lds`: FS2_MAXB ints, the
// caller's static array) and searched there: a binary search over an L2-resident run costs a
// dependent L2 round trip per step, one in LDS ~100 cycles.
__device__ __forceinline__ void fs2_merge_item(const FsJob& J, int wg, int* lds) {
  // FSM_WPR workgroups per run: 8 keys per thread, all 8 searches interleaved
  constexpr int EPT = FSM_EPT;
  constexpr int IL = EPT;
  const int B = J.B;
  const int nrun = (B + FS2_MAXB - 1) / FS2_MAXB;
  const int mi = wg / (FSM_WPR * nrun), cw = wg - mi * FSM_WPR * nrun, c = cw / FSM_WPR;
  const int part = cw - c * FSM_WPR;
  const int f = J.mfields[mi];
  const int* keys = J.rk + (size_t)f * B;
  const int* rperm = J.rp + (size_t)f * B;
  int* sko = J.keys + (size_t)f * B;
  int* pko = J.perm + (size_t)f * B;
  const int c0 = c * FS2_MAXB, clen = min(FS2_MAXB, B - c0);
  const int tid = threadIdx.x;
  int k[EPT], pos[EPT];
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = (j * FSM_WPR + part) * FSM_THREADS + tid;  // index in run c
    k[j] = e < clen ? keys[c0 + e] : 0;
    pos[j] = e;
  }
  for (int r = 0; r < nrun; ++r) {
    if (r == c) continue;
    const int len = min(FS2_MAXB, B - r * FS2_MAXB);
    __syncthreads();  // the previous run's searches are done
    for (int i = tid; i < len; i += FSM_THREADS) lds[i] = keys[r * FS2_MAXB + i];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < EPT; h += IL) {
      int lo[IL], hi[IL];
#pragma unroll
      for (int j = 0; j < IL; ++j) {
        lo[j] = 0;
        hi[j] = len;
      }
      for (int step = len; step > 0; step >>= 1) {  // ceil(log2(len + 1)) rounds
#pragma unroll
        for (int j = 0; j < IL; ++j) {
          if (lo[j] < hi[j]) {
            const int mid = (lo[j] + hi[j]) >> 1;
            const int v = lds[mid];
            // the key's rank among run r: keys <= it (earlier runs) or < it (later runs)
            if (r < c ? v <= k[h + j] : v < k[h + j]) lo[j] = mid + 1;
            else hi[j] = mid;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < IL; ++j) pos[h + j] += lo[j];
    }
  }
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    const int e = (j * FSM_WPR + part) * FSM_THREADS + tid;
    if (e < clen) {
      sko[pos[j]] = k[j];
      pko[pos[j]] = rperm[c0 + e];
      if (J.inv) J.inv[(size_t)f * B + rperm[c0 + e] / J.F] = f * B + pos[j];
    }
  }
}
