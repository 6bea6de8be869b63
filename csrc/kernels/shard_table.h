// Owner-side request table and row serve of the row-sharded exchange (shard.hip has the
// protocol); a header so the serve can also run as extra workgroups of the tower launch (the
// run-routed step serves the NEXT batch's rows inside the current step's tower launch).
#pragma once
#include "common.h"

// hash table of the owner's requested rows: key[slot] = {stamp, row}, pos[slot][p] = {stamp, c}
struct ShTable {
  unsigned long long* key;  // [slots]
  unsigned long long* pos;  // [slots][N]
  unsigned mask;            // slots - 1 (power of two)
  int pad;
};

__device__ __forceinline__ unsigned sh_hash(unsigned row) {
  unsigned h = row * 0x9E3779B1u;
  return h ^ (h >> 15);
}

// insert `row` (requested by rank p at position c) for the step `stamp`; returns nothing: the
// position is recorded in the row's slot.  Stale slots (older stamps) count as empty.
__device__ __forceinline__ void sh_insert(const ShTable& T, int N, unsigned row, int p, unsigned c,
                                          unsigned stamp) {
  const unsigned long long want = ((unsigned long long)stamp << 32) | row;
  unsigned s = sh_hash(row) & T.mask;
  for (unsigned probe = 0; probe <= T.mask; ++probe, s = (s + 1) & T.mask) {
    unsigned long long cur = T.key[s];
    if (cur != want) {
      if ((unsigned)(cur >> 32) == stamp) continue;  // taken by another row this step
      const unsigned long long prev = atomicCAS(T.key + s, cur, want);
      if (prev != cur && prev != want) {  // lost the slot to another row: re-examine it
        if ((unsigned)(prev >> 32) == stamp) continue;
        --probe;
        s = (s - 1) & T.mask;
        continue;
      }
    }
    T.pos[(size_t)s * N + p] = ((unsigned long long)stamp << 32) | c;
    return;
  }
}

__device__ __forceinline__ const unsigned long long* sh_find(const ShTable& T, int N, unsigned row,
                                                             unsigned stamp) {
  const unsigned long long want = ((unsigned long long)stamp << 32) | row;
  unsigned s = sh_hash(row) & T.mask;
  for (unsigned probe = 0; probe <= T.mask; ++probe, s = (s + 1) & T.mask) {
    const unsigned long long cur = T.key[s];
    if (cur == want) return T.pos + (size_t)s * N;
    if ((unsigned)(cur >> 32) != stamp) return nullptr;  // an empty slot ends the probe chain
  }
  return nullptr;
}

// request e = p*C + c of the received ids: [N][C] blocks (rstride == C, or 0 = contiguous), or
// a column of a packed buffer / the all-gathered [N][N][C] requests (base + p*rstride + c)
__device__ __forceinline__ int sh_rid(const int* __restrict__ r, int e, int C, int rstride) {
  return rstride > C ? r[(size_t)(e / C) * rstride + e % C] : r[e];
}

struct ShServeArgs {
  const int* recv_ids;
  int total, N, C, rstride;
  const float* tv;
  const float* tw;
  long ldv, ldw;
  float* rows;            // [total][sh_row_words<K>(rbf16)] (see sh_row_words)
  const int64_t* step;
  ShTable T;              // key == null: eval-style fetch (no request recorded)
  int stamp_off;          // 1: served at its own step's start; 2: served ahead (previous step)
  int vbf16;              // the TABLE's v rows are bf16
  int rbf16;              // served rows carry v as bf16 (compact rows)
  int rdiv;               // local row = id / rdiv (0: N, the row-sharded owner; 1: a replicated table)
  unsigned char* rflag;   // tf1_dense split form: byte flag of every row requested this step (the
                          // owner launch's sweep skips and clears it), or null
};

// Exchanged rows.  Served rows: fp32 {v[K], w, 0, 0, 0} (K + 4 words, 16-B aligned v), or compact
// {v as K bf16 (round to nearest), w, 0} (K/2 + 2 words: 24 B at K = 8 instead of 48; 8-B aligned,
// so a 4-element bf16 group is one 8-B load).  Gradient rows: {g_v[K], g_w} (K + 1 words, dword
// loads / stores).
template <int K>
__host__ __device__ constexpr int sh_row_words(int rbf16) { return rbf16 ? K / 2 + 2 : K + 4; }
template <int K>
__host__ __device__ constexpr int sh_grad_words() { return K + 1; }

// write the 4 v elements [4*sub, 4*sub + 4) of a served row (and w, on sub 0)
template <int K>
__device__ __forceinline__ void sh_put_row(float* o, int sub, f32x4 v, float w, bool rbf) {
  if (rbf) {
    const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, f2bf(v[0])) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, f2bf(v[1])) << 16);
    const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, f2bf(v[2])) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, f2bf(v[3])) << 16);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(o) + sub * 4) = uint2{lo, hi};
    if (sub == 0) *reinterpret_cast<float2*>(o + K / 2) = float2{w, 0.f};
  } else {
    *reinterpret_cast<f32x4*>(o + sub * 4) = v;
    if (sub == 0) *reinterpret_cast<f32x4*>(o + K) = f32x4{w, 0.f, 0.f, 0.f};
  }
}

// tag only (rows == null; the replicated exchange's run steps): request gt of this step recorded
// in the table, one thread per request
__device__ __forceinline__ void sh_tag_elem(const ShServeArgs& A, int gt) {
  if (gt >= A.total || !A.T.key) return;
  const int id = sh_rid(A.recv_ids, gt, A.C, A.rstride);
  if (id < 0) return;
  const unsigned row = (unsigned)(id / (A.rdiv > 0 ? A.rdiv : A.N));
  sh_insert(A.T, A.N, row, gt / A.C, (unsigned)(gt % A.C), (unsigned)(*A.step + A.stamp_off));
  if (A.rflag) A.rflag[row] = 1;
}

// thread gt of a serve: request gt / (K/4), f32x4 column gt % (K/4)
template <int K>
__device__ __forceinline__ void sh_serve_elem(const ShServeArgs& A, int gt) {
  constexpr int LPS = K / 4;
  const int e = gt / LPS, sub = gt % LPS;
  if (e >= A.total) return;
  const int id = sh_rid(A.recv_ids, e, A.C, A.rstride);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  float w = 0.f;
  if (id >= 0) {
    const size_t row = (size_t)(id / (A.rdiv > 0 ? A.rdiv : A.N));
    v = ld_row4(A.tv + row * A.ldv, sub * 4, A.vbf16);
    if (sub == 0) {
      w = A.tw[row * A.ldw];
      if (A.T.key) {
        sh_insert(A.T, A.N, (unsigned)row, e / A.C, (unsigned)(e % A.C), (unsigned)(*A.step + A.stamp_off));
        if (A.rflag) A.rflag[row] = 1;
      }
    }
  }
  sh_put_row<K>(A.rows + (size_t)e * sh_row_words<K>(A.rbf16), sub, v, w, A.rbf16 != 0);
}
