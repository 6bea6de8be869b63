// Fused embedding backward + row optimizer over the sorted slots (single rank / tf1_dense
// scatter): K2 (per-slot FM + MLP-input gradient), K3 (sum per unique id) and K4 (lazy row
// optimizer, or the tf1_dense gradient scatter) in ONE launch.
// SURVEY §2.5 rows 17-20, §7.4 item 1; the reference's update is TF1 Adam._apply_sparse on the
// IndexedSlices of embedding_lookup (HVD:170-176, HVD:252-263).
//
// Per slot (b, f) with id r and value x (see sparse_bwd.hip for the derivation):
//     a = x*(dX0[b, f] + dy_b*S_b),  g_w = dy_b*x,  c = x^2*dy_b;   d fm_v[r] = sum(a) - V[r]*sum(c)
//
// Tile kernel (one workgroup per TP consecutive sorted slots):
//   1. per-slot [a | g_w | c] rows into LDS;
//   2. segmented sums without serial walks over long runs: the tile is cut into CH-slot chunks;
//      one thread per (chunk, column) sums each run piece inside its chunk (in place at the
//      run's head) and the chunk's leading piece (slots before its first head);
//   3. every run head adds the leading pieces of the following chunks up to the chunk holding
//      the next head.  A run that closes inside the tile is applied right here (optimizer on the
//      row, or scatter); the one run that continues into the next tile leaves its partial in
//      ctail[tile].  The tile's own leading piece (continuation of an earlier run) goes to
//      lead[tile], with a flag when the tile has no head at all.
//   4. the tile publishes (lead, ctail, run info) and, if its leading piece closes a run that
//      started in an earlier tile (first slot not a head, and the run ends in this tile), one
//      wave looks back over the predecessors, 64 tiles per round: the run total
//      = own lead + leads of the headless tiles in between + ctail of the origin tile, applied
//      right there (sync.h hand-off; predecessors have lower ids, so the wait always ends).
// Every sum has a fixed order: bitwise reproducible, atomic-free.  Long runs (Criteo's integer
// fields: one id in every row) cost one parallel lead read per 64 tiles they span.
#include "sync.h"

// slots per tile (K = 8, same-box: 256 -> 0.1116, 512 -> 0.1120, 1024 -> 0.1158 ms/step; 1024 drops
// the merged launch to 3 workgroups per CU)
#ifndef HFM_SF_TP8
#define HFM_SF_TP8 512     // (diagnostic variants: HIPFM_BUILD_VARIANT=<tag>:HFM_SF_TP8=<slots>)
#endif
__host__ __device__ constexpr int sf_tile_slots(int K) { return K <= 16 ? HFM_SF_TP8 : (K == 32 ? 256 : 128); }
// K = 32 with few slots (the reference workload, B = 1024: 40K slots) -- every sparse launch
// takes 128-slot tiles: twice the tiles, half the run heads per tile, so a tile's serial
// record round trips halve (0.0766 -> 0.0695 ms/step there; at B = 16384 the 256-slot tiles stay
// faster, 0.2585 vs 0.2734: profiles/r6_sf_tile32_ab.log).  Tile buffers are sized for 128.
constexpr int SF_SMALL_N32 = 131072;

template <int K, int TPS = sf_tile_slots(K)>
struct SfCfg {
  static constexpr int TP = TPS;  // slots per tile
  static constexpr int LPS = K / 4;                                    // lanes per slot (f32x4 each)
  static constexpr int PPP = 256 / LPS;                                // slots per pass
  static constexpr int PASSES = TP / PPP;
  static constexpr int C = K + 2;  // columns: a[K], g_w, c
  static constexpr int CP = C | 1; // LDS row stride (odd: the chunk walk's lanes spread over banks)
  static constexpr int CH = 16;    // chunk length of the segmented sums
  static constexpr int NCH = TP / CH;
  static constexpr int RS = K + 4;  // ctail / lead row stride (16-B aligned)
};

struct SfArgs {
  const int* sorted_keys;
  const int* perm;  // slot position b*F + f of each sorted slot
  const float* vals;
  const float* dlogit;
  const bf16* dX0;  // [B, KP] bf16
  const float* S;   // [B, K]
  int n, F, KP, row_div;
  float* ctail;  // [tiles][RS]
  float* lead;   // [tiles][RS]
  int* tinfo;    // [tiles][4]: {headless, open-run key or -1, open-run head position, pad}
  float *tv, *tw, *s0v, *s1v, *s0w, *s1w;
  float *Gv, *Gw;
  OptHyper h;
  const int64_t* step;
  long ldv, ldw;  // table row strides (record layout: both = record floats)
  // MODE 2 (row-sharded exchange): gradient row of unique u -> gout[upos[u]] ({g_v[K], g_w}), V from
  // the received rows (tv = rows_in, ldv = their words, vbf16 = their format); u = sid[head] - 1
  const int* sid;
  const int* upos;
  float* gout;
  int step_off;     // 1: *step is this step's index - 1 (the dense optimizer advances it later);
                    // 0: the dense optimizer already ran and advanced it (single-GPU early mode)
  unsigned* flags;  // [tiles] publication flags: the step's 1-based index (*step + step_off)
  unsigned* sync;   // {pad, pad, error bits, pad}
  int v_by_key;     // MODE 2: 1 = V rows from the local table row key / row_div (replicated-table
                    // exchange), 0 = from the received rows at upos (row-sharded exchange)
  int vbf16;        // table v rows and v slots are bf16 (mixed-precision embeddings; MODE 0 / 2)
  // or null: [n][K + 2] per-slot rows {a[K], g_w, c} already in SORTED order (written by the
  // tower straight to each slot's sorted position): step 1 streams them instead of gathering
  // perm -> vals / dlogit / S / dX0 per slot
  const float* grow;
  int grow_perm;    // 1: grow rows are in SLOT order (b*F + f): gathered through perm, one 40-B row per slot
};

// one row's record as the lazy optimizer reads it (the f32x4 column group `sub` of v and its
// slots; w and its slots on sub 0)
struct SfRec {
  f32x4 p, s0, s1;
  float pw, aw, cw;
};
template <int K, int OPT>
__device__ __forceinline__ SfRec sf_load_rec(const SfArgs& A, int key, int sub);
template <int K, int OPT>
__device__ __forceinline__ void sf_apply_rec(const SfArgs& A, int key, int sub, f32x4 a, float w, float c,
                                             float lr_t, SfRec R);

// MODE 0: lazy optimizer OPT on the row; 1: tf1_dense scatter of the row gradient;
// 2: compact gradient row for the owner exchange
template <int K, int MODE, int OPT>
__device__ __forceinline__ void sf_apply_row(const SfArgs& A, int key, int hpos, int sub, f32x4 a, float w,
                                             float c, float lr_t) {
  if (MODE == 2) {
    const int r = A.upos[A.sid[hpos] - 1];
    if (r < 0) return;  // capacity overflow (flagged by the bucketing kernel)
    // v from the local table (replicated) or the received row r (row-sharded: vbf16 = the
    // received rows' format, fp32 or compact bf16)
    const f32x4 pv = ld_row4(A.tv + (A.v_by_key ? (size_t)(key / A.row_div) : (size_t)r) * A.ldv, sub * 4,
                             A.vbf16);
    float* go = A.gout + (size_t)r * (K + 1);      // {g_v[K], g_w}: dword stores
    const f32x4 gv = row_grad4(a, pv, c);
#pragma unroll
    for (int j = 0; j < 4; ++j) go[sub * 4 + j] = gv[j];
    if (sub == 0) go[K] = w;
    return;
  }
  const size_t row = (size_t)(key / A.row_div);
  const size_t rb = row * A.ldv;  // the row's record (v, and the v slots at their offsets)
  const bool bf = MODE == 0 && A.vbf16;
  if (MODE == 1) {
    const f32x4 p = ld_row4(A.tv + rb, sub * 4, bf);
    *reinterpret_cast<f32x4*>(A.Gv + row * K + sub * 4) = row_grad4(a, p, c);
    if (sub == 0) A.Gw[row] = w;
    return;
  }
  sf_apply_rec<K, OPT>(A, key, sub, a, w, c, lr_t, sf_load_rec<K, OPT>(A, key, sub));
}

template <int K, int OPT>
__device__ __forceinline__ SfRec sf_load_rec(const SfArgs& A, int key, int sub) {
  const size_t row = (size_t)(key / A.row_div);
  const size_t rb = row * A.ldv, ow = row * A.ldw;
  const bool bf = A.vbf16;
  SfRec r;
  r.p = ld_row4(A.tv + rb, sub * 4, bf);
  r.s0 = r.s1 = f32x4{0, 0, 0, 0};
  r.pw = r.aw = r.cw = 0.f;
  if (OPT != OPT_GD) r.s0 = ld_row4(A.s0v + rb, sub * 4, bf);
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) r.s1 = ld_row4(A.s1v + rb, sub * 4, bf);
  if (sub == 0) {
    r.pw = A.tw[ow];
    if (OPT != OPT_GD) r.aw = A.s0w[ow];
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) r.cw = A.s1w[ow];
  }
  return r;
}

// the lazy optimizer on one row whose record ``R`` was loaded (sf_load_rec) -- possibly early, by
// the tile that owns the row's update (no other workgroup writes it in this launch)
template <int K, int OPT>
__device__ __forceinline__ void sf_apply_rec(const SfArgs& A, int key, int sub, f32x4 a, float w, float c,
                                             float lr_t, SfRec R) {
  const size_t row = (size_t)(key / A.row_div);
  const size_t rb = row * A.ldv;
  const size_t ow = row * A.ldw;
  const bool bf = A.vbf16;
  f32x4 p = R.p, s0 = R.s0, s1 = R.s1;
  const f32x4 gv = row_grad4(a, p, c);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float gj = l2_grad(gv[j], A.h.l2, p[j]);
    float pj = p[j], aj = s0[j], cj = s1[j];
    opt_update<OPT>(pj, gj, aj, cj, A.h, lr_t);
    p[j] = pj;
    s0[j] = aj;
    s1[j] = cj;
  }
  const int64_t st = *A.step;
  st_row4(A.tv + rb, sub * 4, p, bf, bf ? row_sr_seed(row, st, 0) : 0u);
  if (OPT != OPT_GD) st_row4(A.s0v + rb, sub * 4, s0, bf, bf ? row_sr_seed(row, st, 1) : 0u);
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) st_row4(A.s1v + rb, sub * 4, s1, bf, bf ? row_sr_seed(row, st, 2) : 0u);
  if (sub == 0) {
    float pw = R.pw;
    float gw = l2_grad(w, A.h.l2, pw);
    float aw = R.aw;
    float cw = R.cw;
    opt_update<OPT>(pw, gw, aw, cw, A.h, lr_t);
    A.tw[ow] = pw;
    if (OPT != OPT_GD) A.s0w[ow] = aw;
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) A.s1w[ow] = cw;
  }
}

template <int OPT>
__device__ __forceinline__ float sf_lr_t(const SfArgs& A) {
  return OPT == OPT_ADAM ? adam_lr_t(A.h, *A.step + A.step_off) : A.h.lr;
}

// One wave: the run that started in an earlier tile and closes in tile `tile` (see step 4).
template <int K, int MODE, int OPT>
__device__ __forceinline__ void sf_lookback(const SfArgs& A, int tile, unsigned tag, const float* own,
                                            float lr_t) {
  using T = SfCfg<K>;
  constexpr int NV = T::RS / 4;  // f32x4 per lead row: a[K], w, c, pad, pad
  const int lane = threadIdx.x & 63;
  f32x4 tot[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 4; ++j) tot[v][j] = (4 * v + j < T::C) ? own[4 * v + j] : 0.f;
  for (int t0 = tile - 1; t0 >= 0; t0 -= 64) {
    const int t2 = t0 - lane;  // lane 0 = the nearest predecessor
    const bool valid = t2 >= 0;
    unsigned spins = 0;
    while (!__all(!valid || hx_load(A.flags + t2) == tag)) {
      if (++spins >= HFM_SPIN_LIMIT) {
        if (lane == 0) atomicOr(A.sync + 2, 1u);
        return;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // agent-scope acquire after the poll matched (cdna guide §6 G16): the handed-off words below
    // are written sc1 and read sc1, but that fence-free form is only validated for one workgroup
    // per CU -- this kernel runs several, and without the acquire a look-back read stale partial
    // sums now and then (wrong hot-row gradients, not bitwise reproducible across runs)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool has_head = valid && !hx_ldi(A.tinfo + t2 * 4);
    const unsigned long long stop = __ballot(has_head);
    const int first = stop ? __ffsll((long long)stop) - 1 : 64;  // the run's origin tile (lane)
    f32x4 p[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      p[v] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (valid && lane < first) {
        const float* lp = A.lead + (size_t)t2 * T::RS + 4 * v;
        p[v] = f32x4{hx_ldf(lp), hx_ldf(lp + 1), hx_ldf(lp + 2), hx_ldf(lp + 3)};
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        p[v][0] += __shfl_xor(p[v][0], o, 64);
        p[v][1] += __shfl_xor(p[v][1], o, 64);
        p[v][2] += __shfl_xor(p[v][2], o, 64);
        p[v][3] += __shfl_xor(p[v][3], o, 64);
      }
      tot[v] += p[v];
    }
    if (!stop) continue;
    const int org = t0 - first;
    const int key = hx_ldi(A.tinfo + org * 4 + 1), hpos = hx_ldi(A.tinfo + org * 4 + 2);
    if (key < 0) {  // an origin tile always leaves its last run open: inconsistent publication
      if (lane == 0) atomicOr(A.sync + 2, 2u);
      return;
    }
    const int sub = lane;
    if (sub >= T::LPS) return;
    const float* ct = A.ctail + (size_t)org * T::RS;
    f32x4 av = {hx_ldf(ct + sub * 4), hx_ldf(ct + sub * 4 + 1), hx_ldf(ct + sub * 4 + 2), hx_ldf(ct + sub * 4 + 3)};
    float w = hx_ldf(ct + K), c = hx_ldf(ct + K + 1);
    f32x4 ad = {0.f, 0.f, 0.f, 0.f};
    float wd = 0.f, cd = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (v == sub) ad = tot[v];
      if (v == K / 4) {
        wd = tot[v][0];
        cd = tot[v][1];
      }
    }
    av += ad;
    w += wd;
    c += cd;
    sf_apply_row<K, MODE, OPT>(A, key, hpos, sub, av, w, c, lr_t);
    return;
  }
  if (lane == 0) atomicOr(A.sync + 2, 4u);  // no origin before tile 0: impossible
}

template <int K, int TPS = sf_tile_slots(K)>
struct SfSmem {
  using T = SfCfg<K, TPS>;
  float g[T::TP][T::CP];
  int skl[T::TP];
  float lead[T::NCH][T::CP];
  int fh[T::NCH];  // offset of the first head in the chunk (CH: none)
  unsigned hb[T::NCH];  // head bits of the chunk's CH slots (bit q: slot j*CH + q heads a run)
  int hl[T::TP];   // head positions, ascending
  int wcount[4];
  int open_key_s, open_pos_s;
  float own_lead[T::C];
};

HFM_STAMP_BUF(hfm_st_sf)
#define SF_ST(k) HFM_STAMP(hfm_st_sf, blockIdx.x, k)

// tile `tile` of the sparse backward (the sf_tile_kernel workgroup, or one of sfwg_kernel's)
template <int K, int MODE, int OPT, int TPS = sf_tile_slots(K)>
__device__ __forceinline__ void sf_tile_body(const SfArgs& A, const int tile, SfSmem<K, TPS>& sm) {
  using T = SfCfg<K, TPS>;
  constexpr int CH = T::CH;
  auto& g = sm.g;
  auto& skl = sm.skl;
  auto& lead = sm.lead;
  auto& fh = sm.fh;
  auto& hb = sm.hb;
  auto& hl = sm.hl;
  auto& wcount = sm.wcount;
  int& open_key_s = sm.open_key_s;
  int& open_pos_s = sm.open_pos_s;
  auto& own_lead = sm.own_lead;
  // publication tag of this step: its 1-based index (unique per training step; the host zeroes
  // the flags whenever the step counter is rewritten)
  const unsigned tag = (unsigned)(*A.step + A.step_off);
  const int b0 = tile * T::TP;
  const int nloc = min(T::TP, A.n - b0);
  const int nch = (nloc + CH - 1) / CH;
  const int tid = threadIdx.x, sub = tid % T::LPS, lane = tid & 63, wv = tid >> 6;
  const int prev_key = b0 > 0 ? A.sorted_keys[b0 - 1] : -1;
  const int next_key = (b0 + nloc < A.n) ? A.sorted_keys[b0 + nloc] : -1;
  if (tid == 0) open_key_s = open_pos_s = -1;
  SF_ST(0);
  // 1. per-slot contributions
  if (A.grow) {  // sorted rows from the tower: coalesced streams, no per-slot gather
#pragma unroll
    for (int ps = 0; ps < T::PASSES; ++ps) {
      const int p = ps * T::PPP + tid / T::LPS;
      if (p < nloc) {
        const float* gr = A.grow + (size_t)(A.grow_perm ? A.perm[b0 + p] : b0 + p) * grow_stride(K);
        const f32x4 av = *reinterpret_cast<const f32x4a8*>(gr + sub * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) g[p][sub * 4 + j] = av[j];
        if (sub == 0) {
          const f32x2a8 wc = *reinterpret_cast<const f32x2a8*>(gr + K);
          g[p][K] = wc.x;
          g[p][K + 1] = wc.y;
          skl[p] = A.sorted_keys[b0 + p];
        }
      }
    }
  } else {
#pragma unroll
  for (int ps = 0; ps < T::PASSES; ++ps) {
    const int p = ps * T::PPP + tid / T::LPS;
    if (p < nloc) {
      const int i = b0 + p;
      const int q = A.perm[i];
      const int b = q / A.F, f = q - b * A.F;
      const float x = A.vals[q];
      const float dy = A.dlogit[b];
      const f32x4 s = *reinterpret_cast<const f32x4*>(A.S + (size_t)b * K + sub * 4);
      const bf16x4 dxh = *reinterpret_cast<const bf16x4*>(A.dX0 + (size_t)b * A.KP + f * K + sub * 4);
      const f32x4 dx = {bf2f(dxh[0]), bf2f(dxh[1]), bf2f(dxh[2]), bf2f(dxh[3])};
      const f32x4 av = sf_slot_a(dx, dy, s, x);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[p][sub * 4 + j] = av[j];
      if (sub == 0) {
        g[p][K] = sf_slot_gw(dy, x);
        g[p][K + 1] = sf_slot_c(dy, x);
        skl[p] = A.sorted_keys[i];
      }
    }
  }
  }
  __syncthreads();
  SF_ST(1);
  // head flags -> compacted head list (ascending), per-chunk head bits and first head (the
  // ballot of 64 consecutive slots holds the bits of 64 / CH whole chunks)
  static_assert(64 % CH == 0, "a chunk's slots sit in one wave's ballot");
  int nh = 0;
  for (int r = 0; r < T::TP; r += 256) {
    const int p = r + tid;
    bool head = false;
    if (p < nloc) head = (p == 0) ? (skl[0] != prev_key) : (skl[p] != skl[p - 1]);
    const unsigned long long bal = __ballot(head);
    if (lane == 0) wcount[wv] = __popcll(bal);
    if (lane % CH == 0 && p < T::TP) {  // (TP < 256 for K >= 32: the upper lanes hold no slot)
      const unsigned bits = (unsigned)(bal >> lane) & ((1u << CH) - 1u);
      hb[p / CH] = bits;
      fh[p / CH] = bits ? __builtin_ctz(bits) : CH;
    }
    __syncthreads();
    int off = nh;
    for (int w = 0; w < wv; ++w) off += wcount[w];
    if (head) hl[off + __popcll(bal & ((1ull << lane) - 1ull))] = p;
    nh += wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
  }
  SF_ST(2);
  // the record of this thread's first run head, loaded now: its HBM round trip overlaps the chunk
  // sums below instead of following them (used if that run closes in this tile)
  // (also at K = 32, where it holds 15 registers across the chunk sums: A/B on the reference
  // workload 0.0961-0.0979 ms/step with, 0.0976-0.0979 without; profiles/r4p_ref_ab.log)
  const int pre_u = tid / T::LPS;
  constexpr bool PRE = MODE == 0;
  SfRec pre;
  if (PRE && pre_u < nh) pre = sf_load_rec<K, OPT>(A, skl[hl[pre_u]], sub);
  // 2. chunk-local run pieces: in place at the head, leading piece into lead[j]
  for (int t = tid; t < T::NCH * T::C; t += 256) {
    const int j = t / T::C, c = t - j * T::C;
    const int p0 = j * CH, p1 = min(p0 + CH, nloc);
    const unsigned bits = hb[j];
    float s = 0.f;
    int h = -1;
    for (int p = p0; p < p1; ++p) {
      const bool head = (bits >> (p - p0)) & 1u;
      if (head) {
        if (h < 0) lead[j][c] = s;
        else g[h][c] = s;
        s = 0.f;
        h = p;
      }
      s += g[p][c];
    }
    if (h < 0) lead[j][c] = s;
    else g[h][c] = s;
  }
  __syncthreads();
  SF_ST(3);
  // tile leading piece (continuation of an earlier tile's run) + headless flag
  if (tid < T::C) {
    float s = 0.f;
    bool any = false;
    for (int j = 0; j < nch; ++j) {
      s += lead[j][tid];
      if (fh[j] < CH) {
        any = true;
        break;
      }
    }
    hx_stf(A.lead + (size_t)tile * T::RS + tid, s);      // handed off: write-through stores
    own_lead[tid] = s;
    if (tid == 0) hx_sti(A.tinfo + tile * 4, any ? 0 : 1);
  }
  // 3. finish every run headed in this tile
  const float lr_t = sf_lr_t<OPT>(A);
  for (int u = tid / T::LPS; u < nh; u += T::PPP) {
    const int hp = hl[u];
    const int key = skl[hp];
    const int j = hp / CH;
    f32x4 a = {g[hp][sub * 4], g[hp][sub * 4 + 1], g[hp][sub * 4 + 2], g[hp][sub * 4 + 3]};
    float w = g[hp][K], c = g[hp][K + 1];
    bool closed = (u + 1 < nh) && (hl[u + 1] / CH == j);
    if (!closed) {
      for (int jj = j + 1; jj < nch; ++jj) {
        a += f32x4{lead[jj][sub * 4], lead[jj][sub * 4 + 1], lead[jj][sub * 4 + 2], lead[jj][sub * 4 + 3]};
        w += lead[jj][K];
        c += lead[jj][K + 1];
        if (fh[jj] < CH) {
          closed = true;
          break;
        }
      }
      if (!closed) closed = (next_key != key);
    }
    if (closed) {
      if (PRE && u == pre_u)
        sf_apply_rec<K, OPT>(A, key, sub, a, w, c, lr_t, pre);
      else
        sf_apply_row<K, MODE, OPT>(A, key, b0 + hp, sub, a, w, c, lr_t);
    } else {
      float* ct = A.ctail + (size_t)tile * T::RS;
#pragma unroll
      for (int j = 0; j < 4; ++j) hx_stf(ct + sub * 4 + j, a[j]);
      if (sub == 0) {
        hx_stf(ct + K, w);
        hx_stf(ct + K + 1, c);
        open_key_s = key;
        open_pos_s = b0 + hp;
      }
    }
  }
  __syncthreads();
  SF_ST(4);
  if (tid == 0) {
    hx_sti(A.tinfo + tile * 4 + 1, open_key_s);
    hx_sti(A.tinfo + tile * 4 + 2, open_pos_s);
  }
  // 4. publish this tile, then close the run that continues into it (if any)
  hx_drain();
  __syncthreads();
  if (tid == 0) hx_flag(A.flags + tile, tag);
  SF_ST(5);
  // the leading piece continues an earlier run; it ends inside this tile (at the first head) or,
  // for a headless tile, at the tile's end when the next tile starts a new id (or there is none)
  const bool closes = nloc > 0 && skl[0] == prev_key && (nh > 0 || next_key != skl[nloc - 1]);
  if (closes && wv == 0) sf_lookback<K, MODE, OPT>(A, tile, tag, own_lead, lr_t);
  SF_ST(6);
}

template <int K, int MODE, int OPT, int TPS>
__global__ void __launch_bounds__(256) sf_tile_kernel(SfArgs A) {
  __shared__ SfSmem<K, TPS> sm;
  sf_tile_body<K, MODE, OPT, TPS>(A, blockIdx.x, sm);
}

// ---------------------------------------------------------------------------------------------
// sfwg: the sparse backward (lazy rows) and the fused tower's wgfin work (wgfin.h: weight
// gradients, split-K combine, dense optimizer) in ONE launch.  The two are independent -- the
// sparse tiles need dX0 / S / dlogit from the tower, wgfin needs its dZ^T / H^T -- and both are
// latency-bound, so sharing the chip hides most of wgfin under the sparse tiles instead of
// running them back to back behind a kernel boundary.  wgfin workgroups take the LOWEST ids
// (dispatched first: they never wait on anyone); the sparse tiles keep their look-back order
// among themselves.  Every workgroup reads the step counter before it arrives on `done`; the last
// arrival (any grid size: it resets the counter) advances it, so both halves use this step's
// index (sparse: step_off = 1; wgfin: *step + 1).
#include "wgfin.h"
#include "tf1_sweep.h"
#include "shard_table.h"

// the wgfin half's register footprint must not cut the sparse tiles' occupancy (6 waves / SIMD)
constexpr int SFWG_PF = 2;
constexpr int SFWG_MAXNS = 4;
// combine tail one element at a time: 84 VGPRs (4 waves / SIMD) vs 113 (3) for all 4 at once;
// same-box bf16 0.1109-0.1114 (1) / 0.1120-0.1128 (2) / 0.1169-0.1171 (4) ms/step
constexpr int SFWG_TQ = 1;

template <int K, int TPS = sf_tile_slots(K)>
union SfwgSmem {
  SfSmem<K, TPS> sf;
  WgfSmem wg;
};

// (forcing 6 waves / SIMD at K = 8 spills 22 VGPRs and measured slower: 0.1139 vs 0.1110 ms)
// SWEEP (tf1_dense split form): S.nblk more workgroups, dispatched after the sparse tiles, give
// every row outside the batch its l2-only update (tf1_sweep.h) -- disjoint rows, same step t
// (a waves-per-SIMD floor of 5 -- 5 tile workgroups per CU at K <= 8, 8 VGPRs spilled in the
// wgfin half -- did not hold up in a 3 x 3 A/B: profiles/r4zz_sfwg_occupancy_confirm.log)
template <int K, int OPT, bool SWEEP, int TPS>
__global__ void __launch_bounds__(256) sfwg_kernel(SfArgs A, WgFinArgs W, unsigned* done, SweepArgs S) {
  __shared__ SfwgSmem<K, TPS> sm;
  const int nw = W.tile_wgs + 1;
  const int ntile = (A.n + TPS - 1) / TPS;
  // (the wgfin workgroups first: with the sparse tiles first and wgfin in the tail the launch
  // measured 0.1202-0.1213 vs 0.1032-0.1043 ms/step)
  const int bid = (int)blockIdx.x;
  if (bid < nw) {
    SF_ST(8);
    wgfin_body<OPT, SFWG_PF, SFWG_MAXNS, SFWG_TQ>(W, bid, sm.wg);
    SF_ST(9);
  } else if (!SWEEP || bid < nw + ntile) {
    sf_tile_body<K, 0, OPT, TPS>(A, bid - nw, sm.sf);
  } else if (SWEEP) {
    const int sb = bid - nw - ntile;
    // (2 rows per thread per pass: 98 VGPRs, 0.1596-0.1598 vs 0.1565-0.1619 ms -- no gain)
    tf1_sweep_rows<K, OPT, 1>(S.rec, S.ld, S.R, S.flags, A.h, sf_lr_t<OPT>(A),
                              (long)sb * blockDim.x + threadIdx.x, (long)S.nblk * blockDim.x);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(done, 1u, HFM_RLX_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(done, 0u, HFM_RLX_AGENT);
      const int64_t t = *W.o.step + 1;
      *W.o.step = t;
      if (SWEEP) *S.sw_step = t;      // keeps the branch sweep's counter in step
    }
  }
  SF_ST(7);
}

template <int K, int OPT, int TPS>
static void sfwg_launch(const SfArgs& A, const WgFinArgs& W, unsigned* done, const SweepArgs& S,
                        hipStream_t st) {
  const dim3 g(W.tile_wgs + 1 + (A.n + TPS - 1) / TPS + S.nblk), blk(256);
  if constexpr (K <= 32) {
    if (S.nblk) {
      hipLaunchKernelGGL((sfwg_kernel<K, OPT, true, TPS>), g, blk, 0, st, A, W, done, S);
      return;
    }
  }
  hipLaunchKernelGGL((sfwg_kernel<K, OPT, false, TPS>), g, blk, 0, st, A, W, done, S);
}

template <int K, int TPS = sf_tile_slots(K)>
static int sfwg_dispatch(int opt, const SfArgs& A, const WgFinArgs& W, unsigned* done,
                         const SweepArgs& S, hipStream_t st) {
  switch (opt) {
    case OPT_ADAM: sfwg_launch<K, OPT_ADAM, TPS>(A, W, done, S, st); break;
    case OPT_ADAGRAD: sfwg_launch<K, OPT_ADAGRAD, TPS>(A, W, done, S, st); break;
    case OPT_MOMENTUM: sfwg_launch<K, OPT_MOMENTUM, TPS>(A, W, done, S, st); break;
    case OPT_FTRL: sfwg_launch<K, OPT_FTRL, TPS>(A, W, done, S, st); break;
    case OPT_GD: sfwg_launch<K, OPT_GD, TPS>(A, W, done, S, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  return 0;
}

// Row-sharded step: the sparse backward's gradient rows for the owner exchange (MODE 2) and the
// wgfin gradient work (no optimizer: the dense gradient is exchanged first) in one launch.
// Run-routed steps: `S.total` > 0 adds workgroups AFTER the sparse tiles that serve the NEXT step's
// rows (shard_table.h sh_serve_elem, stamped step + 2; this step's owner update patches what it
// changes).  The highest block indices are dispatched last: they fill the CUs the tiles' look-back
// tail leaves idle, instead of competing with the tower's workgroups in its launch.
template <int K, int TPS>
__global__ void __launch_bounds__(256) sfwg_x_kernel(SfArgs A, WgFinArgs W, ShServeArgs S, int tiles) {
  __shared__ SfwgSmem<K, TPS> sm;
  const int nw = W.tile_wgs + 1;
  if ((int)blockIdx.x < nw) wgfin_body<-1, SFWG_PF, SFWG_MAXNS, SFWG_TQ>(W, blockIdx.x, sm.wg);
  else if ((int)blockIdx.x < nw + tiles) sf_tile_body<K, 2, 0, TPS>(A, (int)blockIdx.x - nw, sm.sf);
  else if (S.rows) sh_serve_elem<K>(S, ((int)blockIdx.x - nw - tiles) * 256 + (int)threadIdx.x);
  else sh_tag_elem(S, ((int)blockIdx.x - nw - tiles) * 256 + (int)threadIdx.x);   // (replicated run step)
}

HFM_API int hfm_sparse_wgfin_x(int K, const SfArgs* A, const WgFinArgs* W, const ShServeArgs* S,
                               hipStream_t st) {
  if (A->n <= 0 || !A->flags || !A->sync || !A->gout || W->opt_on || W->ns < 1 || W->ns > SFWG_MAXNS ||
      W->kchunk % 32 || W->ldk != W->ns * 4 * W->kchunk || W->L + 2 > WGF_MAXC || !W->tile_ctr)
    return (int)hipErrorInvalidValue;
  const ShServeArgs sv = S ? *S : ShServeArgs{};
  // serve workgroups: the next step's rows (stamp 2), or -- rows == null -- this step's requests
  // tagged for the owner update that follows (stamp 1: the replicated exchange's run steps)
  if (S && (!sv.recv_ids || !sv.step || !sv.T.key || sv.total <= 0 || sv.stamp_off != (sv.rows ? 2 : 1) ||
            (sv.T.mask & (sv.T.mask + 1)) != 0 || sv.T.mask + 1 < 2u * (unsigned)sv.total))
    return (int)hipErrorInvalidValue;
  const long sth = S ? (long)sv.total * (sv.rows ? K / 4 : 1) : 0;
  const int swg = (int)((sth + 255) / 256);
#define X_(KK, TT)                                                                                \
  hipLaunchKernelGGL((sfwg_x_kernel<KK, TT>), dim3(W->tile_wgs + 1 + (A->n + TT - 1) / TT + swg),   \
                     dim3(256), 0, st, *A, *W, sv, (A->n + TT - 1) / TT)
  switch (K) {
    case 4: X_(4, sf_tile_slots(4)); break;
    case 8: X_(8, sf_tile_slots(8)); break;
    case 16: X_(16, sf_tile_slots(16)); break;
    case 32:
      if (A->n <= SF_SMALL_N32) X_(32, 128);
      else X_(32, sf_tile_slots(32));
      break;
    case 64: X_(64, sf_tile_slots(64)); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef X_
  HFM_LAUNCH_CHECK();
}

// lazy sparse rows (optimizer `opt`) + wgfin with the same dense optimizer; `done`: [1] arrival
// counter, zero between launches.  A.step_off must be 1 (the step advances at the launch's end).
HFM_API int hfm_sparse_wgfin(int K, int opt, const SfArgs* A, const WgFinArgs* W, unsigned* done,
                             const SweepArgs* sweep, hipStream_t st) {
  SweepArgs S{};
  if (sweep && sweep->nblk > 0) {
    const int ns = opt == OPT_GD ? 0 : ((opt == OPT_ADAM || opt == OPT_FTRL) ? 2 : 1);
    const int used = K + 4 + ns * K;
    if (K > 32 || !sweep->rec || !sweep->flags || !sweep->sw_step || sweep->R <= 0 ||
        sweep->ld != (used <= 16 ? (used + 15) / 16 * 16 : (used + 31) / 32 * 32))
      return (int)hipErrorInvalidValue;
    S = *sweep;
  }
  if (A->n <= 0 || !A->flags || !A->sync || !done || A->step_off != 1 || !W->opt_on || W->ns < 1 ||
      W->ns > SFWG_MAXNS || W->kchunk % 32 || W->ldk != W->ns * 4 * W->kchunk || W->L + 2 > WGF_MAXC ||
      !W->tile_ctr || (const void*)W->o.step != (const void*)A->step)
    return (int)hipErrorInvalidValue;
  int rc;
  switch (K) {
    case 4: rc = sfwg_dispatch<4>(opt, *A, *W, done, S, st); break;
    case 8: rc = sfwg_dispatch<8>(opt, *A, *W, done, S, st); break;
    case 16: rc = sfwg_dispatch<16>(opt, *A, *W, done, S, st); break;
    case 32:
      rc = A->n <= SF_SMALL_N32 ? sfwg_dispatch<32, 128>(opt, *A, *W, done, S, st)
                                : sfwg_dispatch<32>(opt, *A, *W, done, S, st);
      break;
    case 64: rc = sfwg_dispatch<64>(opt, *A, *W, done, S, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_sparse_fused_tiles(int K, int n) {
  const int tp = K == 32 ? 128 : sf_tile_slots(K);     // (an upper bound for either K = 32 tile)
  return (n + tp - 1) / tp;
}

template <int K, int MODE, int OPT>
static void sf_launch(const SfArgs& A, hipStream_t st) {
  // (K = 32 with few slots: the small tiles of every sparse launch, so all update forms sum each
  // run in the same tile grouping -- bitwise equal to each other)
  if constexpr (K == 32) {
    if (A.n <= SF_SMALL_N32) {
      hipLaunchKernelGGL((sf_tile_kernel<K, MODE, OPT, 128>), dim3((A.n + 127) / 128), dim3(256), 0, st, A);
      return;
    }
  }
  constexpr int TP = sf_tile_slots(K);
  hipLaunchKernelGGL((sf_tile_kernel<K, MODE, OPT, TP>), dim3((A.n + TP - 1) / TP), dim3(256), 0, st, A);
}

template <int K>
static int sf_dispatch(int mode, int opt, const SfArgs& A, hipStream_t st) {
  if (mode == 1 || mode == 2) {
    if (mode == 1) sf_launch<K, 1, 0>(A, st);
    else sf_launch<K, 2, 0>(A, st);
    return 0;
  }
  switch (opt) {
    case OPT_ADAM: sf_launch<K, 0, OPT_ADAM>(A, st); break;
    case OPT_ADAGRAD: sf_launch<K, 0, OPT_ADAGRAD>(A, st); break;
    case OPT_MOMENTUM: sf_launch<K, 0, OPT_MOMENTUM>(A, st); break;
    case OPT_FTRL: sf_launch<K, 0, OPT_FTRL>(A, st); break;
    case OPT_GD: sf_launch<K, 0, OPT_GD>(A, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  return 0;
}

// mode 0: lazy optimizer `opt` on every unique row; 1: tf1_dense scatter into (Gv, Gw);
// 2: gradient rows for the row-sharded owner exchange (gout[upos[u]])
HFM_API int hfm_sparse_fused(int K, int mode, int opt, const SfArgs* A, hipStream_t st) {
  if (A->n <= 0) return 0;
  if (!A->flags || !A->sync) return (int)hipErrorInvalidValue;
  int rc;
  switch (K) {
    case 4: rc = sf_dispatch<4>(mode, opt, *A, st); break;
    case 8: rc = sf_dispatch<8>(mode, opt, *A, st); break;
    case 16: rc = sf_dispatch<16>(mode, opt, *A, st); break;
    case 32: rc = sf_dispatch<32>(mode, opt, *A, st); break;
    case 64: rc = sf_dispatch<64>(mode, opt, *A, st); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_sparse_fused_args_bytes() { return (int)sizeof(SfArgs); }
