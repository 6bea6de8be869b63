// Row-sharded embedding exchange with FIXED per-peer capacity (SURVEY P1/P4, §2.6 row-sharded
// mode; the reference's parameter servers pull rows and push gradients over gRPC, PS:414-442).
//
// owner(id) = id % N, local row = id / N.  Every exchange moves N blocks of exactly C entries
// (unused entries carry id -1), so all-to-alls need no host-side split sizes and the whole step
// is one capturable stream sequence without a host synchronisation:
//
//   requester                                        owner
//   sorted uniques -> sh_scatter: send_ids[o][c]  -- a2a -->  recv_ids[p][c]
//   (upos[u] = o*C + c)                                       sh_serve: rows[p][c] = {v, w},
//                                                             request table: row -> c per p
//   rows_in[o][c]                                 <-- a2a --
//   sh_slot_rows: slot -> rows_in row; fm_fwd / tower / sparse_fused (MODE 2: gradient rows
//   g_u written at send_g[upos[u]], V taken from rows_in)
//   send_g[o][c]                                  -- a2a -->  recv_g[p][c]
//                                                             sh_owner_apply: the lowest requesting
//                                                             rank sums the rows of all requesters
//                                                             in rank order, applies the optimizer
//
// The request table replaces a sort of the received ids: an open-addressing hash table of the
// rows requested this step (>= 2x the N*C request slots, so at most half full; keys and the per-
// requester positions carry the step stamp {step+1} in their high word, so nothing is cleared
// between steps).  A row requested by several ranks is found in O(1), and its lead requester
// sums the rows of all requesters in rank order: bitwise reproducible.  Its size follows the
// exchange (N*C), not the table: tens of MB per rank instead of the 8*R*N bytes a direct-
// addressed [R_local][N] tag array costs (7 GB per rank at the Criteo-1TB shape).
// A bucket larger than C sets err bit 2 (the host raises).
#include "common.h"

#include "shard_table.h"
#include "tf1_sweep.h"

namespace {
constexpr int SH_THREADS = 256;
constexpr int SH_ITEMS = 16;
constexpr int SH_TILE = SH_THREADS * SH_ITEMS;
constexpr int SH_MAXN = 64;  // ranks
}  // namespace

__global__ void __launch_bounds__(SH_THREADS) sh_count_kernel(const int* __restrict__ ukeys,
                                                             const int* __restrict__ num_u, int N,
                                                             int* __restrict__ cnt) {
  __shared__ int h[SH_MAXN];
  if (threadIdx.x < N) h[threadIdx.x] = 0;
  __syncthreads();
  const int U = *num_u;
  const int b0 = blockIdx.x * SH_TILE;
#pragma unroll 4
  for (int k = 0; k < SH_ITEMS; ++k) {
    const int u = b0 + k * SH_THREADS + threadIdx.x;
    if (u < U) atomicAdd(&h[ukeys[u] % N], 1);
  }
  __syncthreads();
  if (threadIdx.x < N) cnt[blockIdx.x * N + threadIdx.x] = h[threadIdx.x];
}

// Stable bucketing of the (id-sorted) unique list by owner: send_ids[o*C + c] and upos[u].
__global__ void __launch_bounds__(SH_THREADS) sh_scatter_kernel(
    const int* __restrict__ ukeys, const int* __restrict__ num_u, int N, int nbits, int C,
    const int* __restrict__ cnt, int nb, int* __restrict__ send_ids, int* __restrict__ upos,
    int* __restrict__ send_cnt, unsigned* __restrict__ err) {
  __shared__ int off[SH_MAXN];
  __shared__ int tot[SH_MAXN];
  __shared__ int wc[4][SH_MAXN];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int U = *num_u;
  if (tid < SH_MAXN) off[tid] = tot[tid] = wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
  __syncthreads();
  // owner offsets of this block (counts of the blocks before it) and totals: every count loaded
  // by some thread at once (integer sums: order-free) -- a per-owner serial loop over the nb
  // blocks cost one load latency per block (~47 us at nb = 156)
  for (int e = tid; e < nb * N; e += SH_THREADS) {
    const int b = e / N, o = e - b * N;
    const int c = cnt[e];
    if (b < (int)blockIdx.x) atomicAdd(&off[o], c);
    atomicAdd(&tot[o], c);
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < N) {
    send_cnt[tid] = tot[tid];
    if (tot[tid] > C) atomicOr(err, 2u);
  }
  const int w0 = blockIdx.x * SH_TILE + wv * 64 * SH_ITEMS;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int own[SH_ITEMS], rnk[SH_ITEMS];
#pragma unroll
  for (int k = 0; k < SH_ITEMS; ++k) {
    const int u = w0 + k * 64 + lane;
    const bool valid = u < U;
    const int o = valid ? ukeys[u] % N : 0;
    unsigned long long peers = __ballot(valid);
    for (int bit = 0; bit < nbits; ++bit) {
      const bool bset = (o >> bit) & 1;
      const unsigned long long bal = __ballot(bset);
      peers &= bset ? bal : ~bal;
    }
    const int rk = __popcll(peers & lt);
    const int old = wc[wv][o];  // in-order LDS ops of one wave: all lanes read before the update
    own[k] = o;
    rnk[k] = old + rk;
    if (valid && rk == 0) wc[wv][o] = old + __popcll(peers);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SH_ITEMS; ++k) {
    const int u = w0 + k * 64 + lane;
    if (u >= U) continue;
    const int o = own[k];
    int pos = off[o] + rnk[k];
    for (int w = 0; w < wv; ++w) pos += wc[w][o];
    if (pos < C) {
      send_ids[o * C + pos] = ukeys[u];
      upos[u] = o * C + pos;
    } else {
      upos[u] = -1;
      atomicOr(err, 2u);
    }
  }
}

// Routing of the sorted slot ids in TWO launches (replaces segments + bucket: 7 launches).
// The sorted list is cut into tiles of RT_TILE slots; a slot heads a run when its id differs from
// the previous slot's.  sh_route_count: heads per owner and in total, per tile.  sh_route_scatter:
// each tile sums the counts of the tiles before it (every count loaded at once), then ranks its
// heads per owner within each wave (ballots on the owner bits; wave-contiguous slot chunks keep the
// id order), so owner bucket o holds this rank's unique ids of owner o in id order -- the layout
// segments + sh_bucket produced.  Outputs: sid_incl[i] (1-based unique index of slot i's id),
// send_ids[o][c] (-1 past the bucket's count), upos[u] = o*C + c, send_cnt[o], num_u.
constexpr int RT_ITEMS = 16;

// global-address-space access: the run kernels take their pointers from device descriptors, which
// makes them flat -- and a flat load shares lgkmcnt with the LDS counters, so every LDS step of the
// ranking waited on it (vmcnt(0) after each key load: the scatter measured 146 us vs 52)
__device__ __forceinline__ int gld(const int* p) { return *(const __attribute__((address_space(1))) int*)p; }
__device__ __forceinline__ void gst(int* p, int v) { *(__attribute__((address_space(1))) int*)p = v; }
constexpr int RT_TILE = SH_THREADS * RT_ITEMS;

// Per-tile head counts per owner.  Heads are counted per wave with ballots (lanes of one owner
// found by nbits bit-ballots, as in sh_route_scatter_kernel): one LDS atomic per (wave, owner)
// instead of one per head -- at N = 1 every head of a tile hit the same LDS word.
__device__ __forceinline__ void sh_route_count_body(const int* __restrict__ sk, int n, int N, int nbits,
                                                    int* __restrict__ tcnt, int bx) {
  __shared__ int h[SH_MAXN + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid <= N) h[tid] = 0;
  __syncthreads();
  const int i0 = bx * RT_TILE;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int nh = 0;
  int ky[RT_ITEMS], kp[RT_ITEMS];
#pragma unroll
  for (int k = 0; k < RT_ITEMS; ++k) {     // all loads first (clamped: no branches around them)
    const int ic = min(i0 + k * SH_THREADS + tid, n - 1);
    ky[k] = gld(sk + ic);
    kp[k] = gld(sk + max(ic - 1, 0));
  }
#pragma unroll
  for (int k = 0; k < RT_ITEMS; ++k) {
    const int i = i0 + k * SH_THREADS + tid;
    const bool head = i < n && (i == 0 || ky[k] != kp[k]);
    const int o = head ? ky[k] % N : 0;
    const unsigned long long hb = __ballot(head);
    unsigned long long peers = hb;
    for (int bit = 0; bit < nbits; ++bit) {
      const bool bset = (o >> bit) & 1;
      const unsigned long long bal = __ballot(bset);
      peers &= bset ? bal : ~bal;
    }
    if (head && (peers & lt) == 0) atomicAdd(&h[o], __popcll(peers));   // the owner group's leader
    if (lane == 0) nh += __popcll(hb);
  }
  if (lane == 0) atomicAdd(&h[N], nh);
  __syncthreads();
  if (tid <= N) gst(tcnt + bx * (N + 1) + tid, h[tid]);
}

__global__ void __launch_bounds__(SH_THREADS) sh_route_count_kernel(const int* __restrict__ sk, int n, int N,
                                                                   int nbits, int* __restrict__ tcnt) {
  sh_route_count_body(sk, n, N, nbits, tcnt, blockIdx.x);
}

// tile bx of the scatter (grid of nt tiles per batch)
__device__ __forceinline__ void sh_route_scatter_body(
    const int* __restrict__ sk, int n, int N, int nbits, int C, const int* __restrict__ tcnt, int nt,
    int* __restrict__ sid_incl, int* __restrict__ send_ids, int* __restrict__ upos, int* __restrict__ send_cnt,
    int* __restrict__ num_u, unsigned* __restrict__ err, int bx, int ostride,
    const int* __restrict__ perm = nullptr, int* __restrict__ slot_row = nullptr, int F = 1, int ld = 0) {
  __shared__ int off[SH_MAXN + 1];
  __shared__ int tot[SH_MAXN + 1];
  __shared__ int wc[4][SH_MAXN + 1];  // per wave: heads per owner, [N]: all heads
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid <= SH_MAXN) off[tid] = tot[tid] = wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
  __syncthreads();
  for (int e = tid; e < nt * (N + 1); e += SH_THREADS) {
    const int b = e / (N + 1), o = e - b * (N + 1);
    const int c = gld(tcnt + e);
    if (b < bx) atomicAdd(&off[o], c);
    atomicAdd(&tot[o], c);
  }
  __syncthreads();
  if (bx == 0) {
    if (tid < N) {
      gst(send_cnt + tid, tot[tid]);
      if (tot[tid] > C) atomicOr(err, 2u);
    }
    if (tid == 0) gst(num_u, tot[N]);
  }
  for (int e = bx * SH_THREADS + tid; e < N * C; e += nt * SH_THREADS) {
    const int o = e / C, c = e - o * C;
    if (c >= tot[o]) gst(send_ids + (size_t)o * ostride + c, -1);  // unused capacity: padding entries
  }
  const int w0 = bx * RT_TILE + wv * 64 * RT_ITEMS;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int key[RT_ITEMS], own[RT_ITEMS], rnk[RT_ITEMS], hin[RT_ITEMS], pq[RT_ITEMS], kp[RT_ITEMS];
  // every load first, unconditional (clamped indices): branch-free, all in flight at once
#pragma unroll
  for (int k = 0; k < RT_ITEMS; ++k) {
    const int ic = min(w0 + k * 64 + lane, n - 1);
    key[k] = gld(sk + ic);
    kp[k] = gld(sk + max(ic - 1, 0));
    pq[k] = slot_row ? gld(perm + ic) : 0;
  }
  unsigned hmask = 0;
  int run = 0;  // heads in this wave's earlier chunks (wave-uniform)
#pragma unroll
  for (int k = 0; k < RT_ITEMS; ++k) {
    const int i = w0 + k * 64 + lane;
    const bool valid = i < n;
    const bool head = valid && (i == 0 || key[k] != kp[k]);
    const unsigned long long hb = __ballot(head);
    hin[k] = run + __popcll(hb & (lt | (1ull << lane)));  // heads up to and including slot i
    run += __popcll(hb);
    // every slot's owner (not only the heads'): a slot's run head is the last head before it, so
    // the last head of ITS owner -- its rank among this wave's heads of that owner is rk - 1
    const int o = valid ? key[k] % N : 0;
    unsigned long long peers = hb;
    for (int bit = 0; bit < nbits; ++bit) {
      const bool bset = (o >> bit) & 1;
      const unsigned long long bal = __ballot(bset);
      peers &= bset ? bal : ~bal;
    }
    const int rk = __popcll(peers & lt);
    const int old = wc[wv][o];  // in-order LDS ops of one wave: all lanes read before the update
    own[k] = o;
    rnk[k] = old + rk;
    if (head) hmask |= 1u << k;
    if (head && rk == 0) wc[wv][o] = old + __popcll(peers);
  }
  if (lane == 0) wc[wv][N] = run;
  __syncthreads();
  int hw = off[N];
  for (int w = 0; w < wv; ++w) hw += wc[w][N];
#pragma unroll
  for (int k = 0; k < RT_ITEMS; ++k) {
    const int i = w0 + k * 64 + lane;
    if (i >= n) continue;
    gst(sid_incl + i, hw + hin[k]);
    const bool head = (hmask >> k) & 1u;
    const int o = own[k], u = hw + hin[k] - 1;
    int pos = off[o] + rnk[k];
    for (int w = 0; w < wv; ++w) pos += wc[w][o];
    if (slot_row) {
      // the slot -> received-row map (was sh_slot_rows_run: its dependent sid_incl -> upos reads);
      // a run continuing from an earlier tile resolves to off[o] - 1, that tile's last head of o
      const int rp = head ? pos : pos - 1;
      const int q = pq[k];
      gst(slot_row + (ld ? (size_t)(q % F) * ld + q / F : (size_t)q), rp < C ? o * C + rp : 0);
    }
    if (!head) continue;
    if (pos < C) {
      gst(send_ids + (size_t)o * ostride + pos, key[k]);
      gst(upos + u, o * C + pos);
    } else {
      gst(upos + u, -1);
      atomicOr(err, 2u);
    }
  }
}

__global__ void __launch_bounds__(SH_THREADS) sh_route_scatter_kernel(
    const int* __restrict__ sk, int n, int N, int nbits, int C, const int* __restrict__ tcnt, int nt,
    int* __restrict__ sid_incl, int* __restrict__ send_ids, int* __restrict__ upos, int* __restrict__ send_cnt,
    int* __restrict__ num_u, unsigned* __restrict__ err) {
  sh_route_scatter_body(sk, n, N, nbits, C, tcnt, nt, sid_incl, send_ids, upos, send_cnt, num_u, err, blockIdx.x, C);
}

// fm_fwd row index of every slot: the received row of its unique id
__global__ void sh_slot_rows_kernel(const int* __restrict__ perm, const int* __restrict__ sid_incl,
                                    const int* __restrict__ upos, int n, int* __restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = upos[sid_incl[i] - 1];
  idx[perm[i]] = r < 0 ? 0 : r;
}

// Run-level routing (the row-sharded analogue of fsort_run.h): the routing of EVERY batch of a
// multi-step graph in three launches at its start (blockIdx.y = batch), so the steps that follow
// carry no routing branch and no cross-queue join.  One descriptor per batch (its routing set).
struct ShRouteBatch {
  const int* sk;    // sorted slot ids [n]
  const int* perm;  // their slot positions [n]
  int* tcnt;        // [tiles][N + 1]
  int* sid_incl;
  int* send_ids;    // owner o's block at send_ids + o * ostride (the run's ids travel packed
                    // [N][G][C]: ONE all-to-all for the whole run)
  int* upos;
  int* send_cnt;
  int* num_u;
  int* slot_row;    // [n] fm_fwd row index of every slot
};

__global__ void __launch_bounds__(SH_THREADS) sh_route_count_run_kernel(const ShRouteBatch* __restrict__ rb, int n,
                                                                       int N, int nbits) {
  const ShRouteBatch R = rb[blockIdx.y];
  sh_route_count_body(R.sk, n, N, nbits, R.tcnt, blockIdx.x);
}

__global__ void __launch_bounds__(SH_THREADS) sh_route_scatter_run_kernel(const ShRouteBatch* __restrict__ rb, int n,
                                                                         int N, int nbits, int C, int nt,
                                                                         unsigned* __restrict__ err, int ostride,
                                                                         int F, int ld, int slot_rows) {
  const ShRouteBatch R = rb[blockIdx.y];
  sh_route_scatter_body(R.sk, n, N, nbits, C, R.tcnt, nt, R.sid_incl, R.send_ids, R.upos, R.send_cnt, R.num_u,
                        err, blockIdx.x, ostride, R.perm, slot_rows ? R.slot_row : nullptr, F, ld);
}

// Owner: rows[e] = the served row of each requested id (sh_row_words; zeros for padding entries)
// Training steps (tags != null) also stamp the owner-side request tags here, at the start of the
// step: the requests of the backward exchange are this step's requests, so the owner update at
// the end of the step needs no separate tagging launch on the critical path.
// Stamp = counter + stamp_off: 1 when served at the start of its own step; 2 when SERVED AHEAD
// during the previous step (whose counter is one lower) -- that step's owner update then patches
// the served rows it changes (sh_owner_apply_elem), so the fetch leaves the critical path.
template <int K>
__global__ void sh_serve_kernel(const int* __restrict__ recv_ids, int total, int N, int C, int rstride,
                                const float* __restrict__ tv, const float* __restrict__ tw, long ldv,
                                long ldw, float* __restrict__ rows, const int64_t* __restrict__ step,
                                ShTable T, int stamp_off, int vbf16, int rbf16, unsigned char* rflag) {
  const ShServeArgs A{recv_ids, total, N, C, rstride, tv, tw, ldv, ldw, rows, step, T, stamp_off, vbf16, rbf16,
                      0, rflag};
  sh_serve_elem<K>(A, blockIdx.x * blockDim.x + threadIdx.x);
}

__global__ void sh_owner_tag_kernel(const int* __restrict__ recv_ids, int total, int N, int C, int rstride,
                                    const int64_t* __restrict__ step, ShTable T, int rdiv,
                                    unsigned char* __restrict__ rflag) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int id = sh_rid(recv_ids, e, C, rstride);
  if (id < 0) return;
  sh_insert(T, N, (unsigned)(id / rdiv), e / C, (unsigned)(e % C), (unsigned)(*step + 1));
  if (rflag) rflag[id / rdiv] = 1;        // tf1_dense split form: this step's row (see the sweep)
}

// MODE 0: lazy optimizer OPT on the owner's row; 1: tf1_dense scatter into (Gv, Gw)
template <int K, int MODE, int OPT>
__device__ __forceinline__ void sh_owner_apply_elem(int gt, const int* __restrict__ recv_ids, int total, int N,
                                                    int C, int rstride, const float* __restrict__ recv_g,
                                                    ShTable T, float* tv, float* tw, float* s0v, float* s1v,
                                                    float* s0w, float* s1w, long ldv, long ldw, float* Gv,
                                                    float* Gw, OptHyper h, const int64_t* __restrict__ step,
                                                    const ShTable& NT, float* __restrict__ next_rows,
                                                    int rdiv, int vbf16, int rbf16) {
  constexpr int LPS = K / 4, RWG = sh_grad_words<K>();
  const int e = gt / LPS, sub = gt % LPS;
  if (e >= total) return;
  const int id = sh_rid(recv_ids, e, C, rstride);
  if (id < 0) return;
  const int p = e / C;
  const size_t row = (size_t)(id / rdiv);
  const unsigned cur = (unsigned)(*step + 1);
  // the owner's record (row, slots) is loaded up front, beside the request-table probes: its
  // HBM round trip overlaps theirs instead of following them (a non-lead requester's copy of the
  // loads is simply dropped)
  const size_t rb = row * ldv, ow = row * ldw;
  const bool bf = vbf16 != 0;
  f32x4 pv = {0, 0, 0, 0}, a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
  float pw = 0.f, aw = 0.f, cw = 0.f;
  if (MODE == 0) {
    pv = ld_row4(tv + rb, sub * 4, bf);
    if (OPT != OPT_GD) a = ld_row4(s0v + rb, sub * 4, bf);
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) c = ld_row4(s1v + rb, sub * 4, bf);
    if (sub == 0) {
      pw = tw[ow];
      if (OPT != OPT_GD) aw = s0w[ow];
      if (OPT == OPT_ADAM || OPT == OPT_FTRL) cw = s1w[ow];
    }
  }
  f32x4 g = {0.f, 0.f, 0.f, 0.f};
  float gw = 0.f;
  const unsigned long long* tr = sh_find(T, N, (unsigned)row, cur);
  if (!tr) return;  // cannot happen: every received row was inserted by this step's serve / tag
  for (int q = 0; q < p; ++q)
    if ((unsigned)(tr[q] >> 32) == cur) return;  // a lower rank also requested it: it leads
  for (int q = p; q < N; ++q) {
    const unsigned long long t = tr[q];
    if ((unsigned)(t >> 32) != cur) continue;
    const float* src = recv_g + ((size_t)q * C + (unsigned)t) * RWG;   // (dword-aligned rows)
    g += f32x4{src[sub * 4], src[sub * 4 + 1], src[sub * 4 + 2], src[sub * 4 + 3]};
    gw += src[K];
  }
  if (MODE == 1) {
    *reinterpret_cast<f32x4*>(Gv + row * K + sub * 4) = g;
    if (sub == 0) Gw[row] = gw;
    return;
  }
  const float lr_t = OPT == OPT_ADAM ? adam_lr_t(h, *step + 1) : h.lr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float gj = l2_grad(g[j], h.l2, pv[j]);
    float pj = pv[j], aj = a[j], cj = c[j];
    opt_update<OPT>(pj, gj, aj, cj, h, lr_t);
    pv[j] = pj;
    a[j] = aj;
    c[j] = cj;
  }
  const int64_t st = *step;
  const uint32_t sv_seed = bf ? row_sr_seed(row, st, 0) : 0u;
  st_row4(tv + rb, sub * 4, pv, bf, sv_seed);
  pv = rounded_row4(pv, sub * 4, bf, sv_seed);   // (bf16) the stored value, for the served-ahead patch
  if (OPT != OPT_GD) st_row4(s0v + rb, sub * 4, a, bf, bf ? row_sr_seed(row, st, 1) : 0u);
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) st_row4(s1v + rb, sub * 4, c, bf, bf ? row_sr_seed(row, st, 2) : 0u);
  float wnew = 0.f;
  if (sub == 0) {
    float g1 = l2_grad(gw, h.l2, pw);
    opt_update<OPT>(pw, g1, aw, cw, h, lr_t);
    tw[ow] = pw;
    if (OPT != OPT_GD) s0w[ow] = aw;
    if (OPT == OPT_ADAM || OPT == OPT_FTRL) s1w[ow] = cw;
    wnew = pw;
  }
  if (NT.key) {
    // the next step's requests were served ahead (before this update): refresh the rows this
    // update changed in every requester's block of the next fetch
    const unsigned long long* nr = sh_find(NT, N, (unsigned)row, cur + 1);
    if (nr) {
      for (int q = 0; q < N; ++q) {
        const unsigned long long t = nr[q];
        if ((unsigned)(t >> 32) != cur + 1) continue;
        sh_put_row<K>(next_rows + ((size_t)q * C + (unsigned)t) * sh_row_words<K>(rbf16), sub, pv, wnew,
                      rbf16 != 0);
      }
    }
  }
}

template <int K, int MODE, int OPT>
__global__ void sh_owner_apply_kernel(const int* __restrict__ recv_ids, int total, int N, int C, int rstride,
                                      const float* __restrict__ recv_g, ShTable T, float* tv, float* tw,
                                      float* s0v, float* s1v, float* s0w, float* s1w, long ldv, long ldw,
                                      float* Gv, float* Gw, OptHyper h, const int64_t* __restrict__ step,
                                      ShTable NT, float* next_rows, int rdiv, int vbf16, int rbf16) {
  sh_owner_apply_elem<K, MODE, OPT>(blockIdx.x * blockDim.x + threadIdx.x, recv_ids, total, N, C, rstride,
                                    recv_g, T, tv, tw, s0v, s1v, s0w, s1w, ldv, ldw, Gv, Gw, h, step, NT,
                                    next_rows, rdiv, vbf16, rbf16);
}

// ------------------------------------------------------------------------------------ host API
HFM_API int hfm_sh_count_blocks(int nmax) { return (nmax + SH_TILE - 1) / SH_TILE; }

// ukeys/num_u: this rank's unique ids (sorted); nmax: host upper bound of U (= slots per step)
HFM_API int hfm_sh_bucket(const int* ukeys, const int* num_u, int nmax, int N, int C, int* cnt_tmp,
                          int* send_ids, int* upos, int* send_cnt, unsigned* err, hipStream_t st) {
  if (N < 1 || N > SH_MAXN) return (int)hipErrorInvalidValue;
  const int nb = hfm_sh_count_blocks(nmax);
  int nbits = 0;
  while ((1 << nbits) < N) ++nbits;
  hipError_t e = hipMemsetAsync(send_ids, 0xFF, (size_t)N * C * sizeof(int), st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(sh_count_kernel, dim3(nb), dim3(SH_THREADS), 0, st, ukeys, num_u, N, cnt_tmp);
  hipLaunchKernelGGL(sh_scatter_kernel, dim3(nb), dim3(SH_THREADS), 0, st, ukeys, num_u, N, nbits, C,
                     cnt_tmp, nb, send_ids, upos, send_cnt, err);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_sh_route_tiles(int n) { return (n + RT_TILE - 1) / RT_TILE; }

// sorted slot ids -> sid_incl / owner buckets (see sh_route_scatter_kernel); tcnt: [tiles][N + 1]
HFM_API int hfm_sh_route(const int* sorted_keys, int n, int N, int C, int* tcnt, int* sid_incl, int* send_ids,
                         int* upos, int* send_cnt, int* num_u, unsigned* err, hipStream_t st) {
  if (N < 1 || N > SH_MAXN || n <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  const int nt = hfm_sh_route_tiles(n);
  int nbits = 0;
  while ((1 << nbits) < N) ++nbits;
  hipLaunchKernelGGL(sh_route_count_kernel, dim3(nt), dim3(SH_THREADS), 0, st, sorted_keys, n, N, nbits, tcnt);
  hipLaunchKernelGGL(sh_route_scatter_kernel, dim3(nt), dim3(SH_THREADS), 0, st, sorted_keys, n, N, nbits, C,
                     tcnt, nt, sid_incl, send_ids, upos, send_cnt, num_u, err);
  HFM_LAUNCH_CHECK();
}

// G batches' routing (descriptors rb [G], device): count, then scatter + slot rows -- two launches;
// ostride: owner block stride of every batch's send_ids (>= C); F, ld: slot map layout (ld = 0:
// row-major [n], else field-major [F][ld], ld >= n / F)
// slot_rows == 0: no slot -> row maps (the replicated exchange reads its gradient rows by unique
// index, never through them)
HFM_API int hfm_sh_route_run(const ShRouteBatch* rb, int G, int n, int N, int C, int ostride, int F, int ld,
                             int slot_rows, unsigned* err, hipStream_t st) {
  if (!rb || G <= 0 || G > 65535 || N < 1 || N > SH_MAXN || n <= 0 || C <= 0 || ostride < C || F <= 0 ||
      n % F || (ld && ld < n / F))
    return (int)hipErrorInvalidValue;
  const int nt = hfm_sh_route_tiles(n);
  int nbits = 0;
  while ((1 << nbits) < N) ++nbits;
  hipLaunchKernelGGL(sh_route_count_run_kernel, dim3(nt, G), dim3(SH_THREADS), 0, st, rb, n, N, nbits);
  // (the slot -> row maps come out of the scatter itself: 2 launches, was 3)
  hipLaunchKernelGGL(sh_route_scatter_run_kernel, dim3(nt, G), dim3(SH_THREADS), 0, st, rb, n, N, nbits, C, nt, err,
                     ostride, F, ld, slot_rows);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_sh_route_batch_bytes() { return (int)sizeof(ShRouteBatch); }

HFM_API int hfm_sh_slot_rows(const int* perm, const int* sid_incl, const int* upos, int n, int* idx,
                             hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sh_slot_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, st, perm, sid_incl, upos,
                     n, idx);
  HFM_LAUNCH_CHECK();
}

#define HFM_K_DISPATCH(K, CALL) \
  switch (K) {                  \
    case 4: CALL(4); break;     \
    case 8: CALL(8); break;     \
    case 16: CALL(16); break;   \
    case 32: CALL(32); break;   \
    case 64: CALL(64); break;   \
    default: return (int)hipErrorInvalidValue; \
  }

// table = {key, pos, mask} of the request table, or key == null (eval-style fetch: no insert)
HFM_API int hfm_sh_serve(int K, const int* recv_ids, int total, int N, int C, int rstride, const float* tv,
                         const float* tw,
                         long ldv, long ldw, float* rows, const int64_t* step, const ShTable* table,
                         int stamp_off, int vbf16, int rbf16, unsigned char* rflag, hipStream_t st) {
  const long th = (long)total * (K / 4);
  const int grid = (int)((th + 255) / 256);
  if (grid == 0) return 0;
  const ShTable T = table ? *table : ShTable{nullptr, nullptr, 0u, 0};
  if (T.key && (!step || C <= 0 || (T.mask & (T.mask + 1)) != 0 || T.mask + 1 < 2u * (unsigned)total))
    return (int)hipErrorInvalidValue;
  if (rstride > C && (C <= 0 || rstride % C)) return (int)hipErrorInvalidValue;
  if (stamp_off != 1 && stamp_off != 2) return (int)hipErrorInvalidValue;
#define CALL(KK) hipLaunchKernelGGL(sh_serve_kernel<KK>, dim3(grid), dim3(256), 0, st, recv_ids, total, N, \
                                    C, rstride, tv, tw, ldv, ldw, rows, step, T, stamp_off, vbf16, rbf16, \
                                    T.key ? rflag : nullptr)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
  HFM_LAUNCH_CHECK();
}

struct ShApplyArgs {
  const int* recv_ids;
  int total, N, C, mode;
  int rstride;  // request row stride (see sh_rid)
  const float* recv_g;
  ShTable table;
  float *tv, *tw, *s0v, *s1v, *s0w, *s1w;
  long ldv, ldw;
  float *Gv, *Gw;
  OptHyper h;
  const int64_t* step;
  ShTable next;       // lazy mode: the next step's request table when its rows were served ahead
  float* next_rows;   //   (key == null: none) and its served rows, patched by this update
  int rdiv;           // local row = id / rdiv (0: N, the row-sharded owner; 1: a replicated table)
  int vbf16;          // table v rows and v slots are bf16 (lazy mode only)
  int rbf16;          // the served rows (next_rows) are compact bf16 rows (sh_row_words)
  // tf1_dense split form (sh_apply_dense): the l2-only update of every local row NOT requested this
  // step (byte flag rflag, set by the serve / tag kernel), as sweep workgroups of the launch; the
  // requested rows take their full update from the lazy owner apply
  float* rec;         // table records [R][rec_ld] (deepfm.py record layout), or null: no sweep
  unsigned char* rflag;
  long R;
  int rec_ld, sweep_blocks;
};

__host__ __device__ static inline int sh_rdiv(const ShApplyArgs& A) { return A.rdiv > 0 ? A.rdiv : A.N; }

template <int K>
static int sh_apply_k(int opt, const ShApplyArgs& A, hipStream_t st) {
  const long th = (long)A.total * (K / 4);
  const int grid = (int)((th + 255) / 256);
  if (A.mode & 2)  // tags not stamped by this step's serve (eval-style fetch): stamp them here
    hipLaunchKernelGGL(sh_owner_tag_kernel, dim3((A.total + 255) / 256), dim3(256), 0, st, A.recv_ids,
                       A.total, A.N, A.C, A.rstride, A.step, A.table, sh_rdiv(A), (unsigned char*)nullptr);
#define L_(M, O)                                                                                      \
  hipLaunchKernelGGL((sh_owner_apply_kernel<K, M, O>), dim3(grid), dim3(256), 0, st, A.recv_ids, A.total, \
                     A.N, A.C, A.rstride, A.recv_g, A.table, A.tv, A.tw, A.s0v, A.s1v, A.s0w, A.s1w, A.ldv, A.ldw, \
                     A.Gv, A.Gw, A.h, A.step, (M) == 0 ? A.next : ShTable{nullptr, nullptr, 0u, 0}, A.next_rows, \
                     sh_rdiv(A), (M) == 0 ? A.vbf16 : 0, A.rbf16)
  if ((A.mode & 1) == 1) {
    L_(1, 0);
    return 0;
  }
  switch (opt) {
    case OPT_ADAM: L_(0, OPT_ADAM); break;
    case OPT_ADAGRAD: L_(0, OPT_ADAGRAD); break;
    case OPT_MOMENTUM: L_(0, OPT_MOMENTUM); break;
    case OPT_FTRL: L_(0, OPT_FTRL); break;
    case OPT_GD: L_(0, OPT_GD); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef L_
  return 0;
}

// owner side of the backward: tag every received gradient row, then the lead requester of each
// row sums all requesters' rows in rank order and applies the optimizer (mode 0) or scatters
// into the tf1_dense gradient buffer (mode 1)
HFM_API int hfm_sh_owner_apply(int K, int opt, const ShApplyArgs* A, hipStream_t st) {
  if (A->total <= 0) return 0;
  const unsigned m = A->table.mask;
  if (!A->table.key || (m & (m + 1)) != 0 || m + 1 < 2u * (unsigned)A->total) return (int)hipErrorInvalidValue;
  if (A->next.key && (!A->next_rows || (A->next.mask & (A->next.mask + 1)) != 0)) return (int)hipErrorInvalidValue;
  int rc = 0;
#define CALL(KK) rc = sh_apply_k<KK>(opt, *A, st)
  HFM_K_DISPATCH(K, CALL)
#undef CALL
  if (rc) return rc;
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_sh_apply_args_bytes() { return (int)sizeof(ShApplyArgs); }

// The lazy owner update and the dense optimizer (after the dense all-reduce) in ONE launch: the
// two are independent, and the end of the multi-GPU step then has one kernel boundary less.
// Workgroups [0, apply_blocks) run the owner update, the rest sweep the dense parameters
// (dense_opt_elem, bitwise the dense_opt launch); every workgroup read the step counter before
// it arrives on `done`, and the last arrival advances it (and re-arms the counter).
struct ShDenseArgs {
  float* p;
  const float* g;
  float* s0;
  float* s1;
  long n;
  OptHyper h;
  const ShadowSeg* segs;
  int nseg;
  int blocks;       // workgroups of the dense sweep
  unsigned* done;   // [1], zero between launches
  int nsum;         // 0: g is the gradient; R > 0: g holds R rank gradients [R][n], summed in rank order
};

template <int K, int OPT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) sh_apply_dense_kernel(ShApplyArgs A, ShDenseArgs D, int apply_blocks) {
  // block order: the owner apply, the dense sweep, then the tf1 sweep (the dense workgroups first
  // measured 30.2 vs 27.0 us)
  const int b = blockIdx.x;
  if (b < apply_blocks) {
    sh_owner_apply_elem<K, 0, OPT>(b * 256 + threadIdx.x, A.recv_ids, A.total, A.N, A.C, A.rstride,
                                   A.recv_g, A.table, A.tv, A.tw, A.s0v, A.s1v, A.s0w, A.s1w, A.ldv, A.ldw, A.Gv,
                                   A.Gw, A.h, A.step, A.next, A.next_rows, sh_rdiv(A), A.vbf16, A.rbf16);
  } else if (b >= apply_blocks + D.blocks) {   // tf1_dense split form: the l2-only sweep
    const float lr_t = OPT == OPT_ADAM ? adam_lr_t(A.h, *A.step + 1) : A.h.lr;
    tf1_sweep_rows<K, OPT, 1>(A.rec, A.rec_ld, A.R, A.rflag, A.h, lr_t,
                              (long)(b - apply_blocks - D.blocks) * 256 + threadIdx.x, (long)A.sweep_blocks * 256);
  } else {
    const float lr_t = OPT == OPT_ADAM ? adam_lr_t(D.h, *A.step + 1) : D.h.lr;
    for (long i = (long)(b - apply_blocks) * 256 + threadIdx.x; i < D.n; i += (long)D.blocks * 256) {
      if (D.nsum > 0) {  // the all-gathered per-rank dense gradients: the all-reduce, in rank order
        float gi = D.g[i];
        for (int q = 1; q < D.nsum; ++q) gi += D.g[(size_t)q * D.n + i];
        dense_opt_apply<OPT>(D.p, gi, D.s0, D.s1, i, D.h, lr_t, D.segs, D.nseg);
      } else {
        dense_opt_elem<OPT>(D.p, D.g, D.s0, D.s1, i, D.h, lr_t, D.segs, D.nseg);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(D.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(D.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *const_cast<int64_t*>(A.step) += 1;
    }
  }
}

// lazy rows only: mode 0 (tags stamped by this step's serve) or 2 (tagged here first: the
// replicated-table exchange has no serve)
HFM_API int hfm_sh_apply_dense(int K, int opt, const ShApplyArgs* A, const ShDenseArgs* D, hipStream_t st) {
  if ((A->mode & 1) != 0 || !D->done || D->blocks < 1 || !A->step) return (int)hipErrorInvalidValue;
  if (A->total <= 0) return (int)hipErrorInvalidValue;
  const bool sweep = A->rec != nullptr;
  if (sweep && (!A->rflag || A->R <= 0 || A->sweep_blocks < 1 || A->vbf16 || A->next.key ||
                A->rec_ld < K + 4))
    return (int)hipErrorInvalidValue;
  if (A->mode & 2)
    hipLaunchKernelGGL(sh_owner_tag_kernel, dim3((A->total + 255) / 256), dim3(256), 0, st, A->recv_ids,
                       A->total, A->N, A->C, A->rstride, A->step, A->table, sh_rdiv(*A),
                       sweep ? A->rflag : (unsigned char*)nullptr);
  if (A->next.key && (!A->next_rows || (A->next.mask & (A->next.mask + 1)) != 0)) return (int)hipErrorInvalidValue;
  const long th = (long)A->total * (K / 4);
  const int ab = (int)((th + 255) / 256);
  const dim3 g(ab + D->blocks + (sweep ? A->sweep_blocks : 0)), blk(256);
#define L_(KK, O) hipLaunchKernelGGL((sh_apply_dense_kernel<KK, O>), g, blk, 0, st, *A, *D, ab)
#define OPTS(KK)                                         \
  switch (opt) {                                         \
    case OPT_ADAM: L_(KK, OPT_ADAM); break;              \
    case OPT_ADAGRAD: L_(KK, OPT_ADAGRAD); break;        \
    case OPT_MOMENTUM: L_(KK, OPT_MOMENTUM); break;      \
    case OPT_FTRL: L_(KK, OPT_FTRL); break;              \
    case OPT_GD: L_(KK, OPT_GD); break;                  \
    default: return (int)hipErrorInvalidValue;           \
  }
  HFM_K_DISPATCH(K, OPTS)
#undef OPTS
#undef L_
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_sh_dense_args_bytes() { return (int)sizeof(ShDenseArgs); }
