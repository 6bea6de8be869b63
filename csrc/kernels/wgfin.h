// wgfin: the fused tower's weight gradients + split-K combine + bias gradients + head reductions
// + dense optimizer as workgroup work (replaces wgrad_group + finalize[_opt] for the fused tower).
// Run by its own launch (tower.hip wgfin_kernel) or inside the sparse backward's launch
// (sparse_fused.hip sfwg_kernel: the two are independent and both latency-bound).
//
// Output tile (layer, 32x32) work is split over the batch into NS workgroup-splits of 4 waves;
// each wave reduces its own k-chunk on MFMA, the 4 wave tiles are summed in LDS (fixed order),
// and the workgroup's partial goes to its slab with write-through stores.  The workgroup that
// draws the NS-th arrival on the tile's counter (counters only ever grow: arrival % NS == NS - 1,
// nothing to reset) sums the NS slabs in slab order and applies the dense optimizer to its 32x32
// parameters right away, bf16 shadows included (OPT < 0: writes the gradient only -- multi-rank,
// before the all-reduce).  Its slab loads and the parameter / slot loads are issued together, so
// the combine costs one round trip.  Column-tile 0 workgroups also sum their dZ^T rows: the bias
// gradient, combined the same way.  One extra workgroup reduces the tower's per-block head
// partials (deep_out weights, its bias, fm_bias, the loss sum).
//
// Phase timing (wall clock per workgroup, NS = 4, 1 GPU, Criteo-1TB step): k-loop 15-17 us, slab
// publication ~1.6 us, combine + optimizer of the last arriver ~7-9 us before the loads were
// batched, head workgroup ~14 us (in parallel).
#pragma once
#include "common.h"
#include "mma32.h"
#include "sync.h"

constexpr int WGF_MAXC = 512;   // head columns (last deep layer + 2): two per thread of the head workgroup
constexpr int WGF_MAXNS = 8;    // workgroup splits of the batch per tile

struct WgFinJob {
  const bf16* A;   // dZ_i^T [Np_i, ldk]
  const bf16* B;   // X_i^T  [Kp_i, ldk]
  float* slab;     // [NS][Np_i][Kp_i]
  float* bslab;    // [NS][Np_i]
  float* gw;       // gradient of W_i in the flat buffer [Np_i, Kp_i]
  float* gb;       // gradient of b_i [Np_i]
  bf16* w16;       // bf16 shadows of W_i: [Np_i, Kp_i] and [Kp_i, Np_i] (MFMA operands)
  bf16* wt16;
  // fp8 tower (else null): e4m3 W_i [Np_i, Kp_i] with per-output-channel power-of-two scales
  // (sdq = dequantization factor), from the row |W| max of the PREVIOUS step (delayed scaling,
  // one binade of headroom); amax3 [3][Np_i] (float bits) rotates with the step: this step's
  // row maxima are atomicMax-ed into slot (t % 3), slot (t - 1) % 3 is read, (t + 1) % 3 zeroed
  uint8_t* w8;
  float* sdq;
  unsigned* amax3;
  int M, N;        // Np_i, Kp_i
  int tiles_m, tiles_n;
  int tile0;       // first counter of this job
  int wg0;         // first workgroup of this job
};

struct WgFinArgs {
  const WgFinJob* jobs;
  int njobs, ldk, kchunk, ns;      // ldk = batch rows M; kchunk = rows per wave; NS splits
  int tile_wgs;                    // workgroups of the tile work; workgroup tile_wgs = head
  unsigned* tile_ctr;              // [tiles]
  unsigned* done_ctr;              // [1]
  const float* partial;            // [nhead][L + 2] tower head partials
  int nhead, L;
  float* g_wout;                   // [L]
  float* g_bout;                   // [1]
  float* g_fmbias;                 // [1]
  float* loss_sum;                 // [1]
  FinOpt o;
  int opt_on;
};

struct WgfSmem {
  float red[4][32][33];
  float bred[4][32];
  int last;
};

// gradient gv of the flat element dst: store it, then (OPT >= 0) the optimizer on p / slots that
// the caller already loaded (pv, av, cv); returns the new parameter.  Same arithmetic as
// fin_opt_apply / dense_opt (bitwise: the gradient is pinned to a rounded register first).
template <int OPT>
__device__ __forceinline__ float wgf_update(const WgFinArgs& a, float lr_t, float* dst, float gv, float pv,
                                            float av, float cv) {
  *dst = gv;
  if (OPT < 0) return 0.f;
  const long i = dst - a.o.g;
  asm volatile("" : "+v"(gv));
  opt_update<OPT>(pv, gv, av, cv, a.o.h, lr_t);
  a.o.p[i] = pv;
  if (OPT != OPT_GD) a.o.s0[i] = av;
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) a.o.s1[i] = cv;
  return pv;
}

// optimizer inputs of flat element i (zeros when OPT < 0)
template <int OPT>
__device__ __forceinline__ void wgf_load_state(const WgFinArgs& a, const float* dst, float& pv, float& av,
                                               float& cv) {
  pv = av = cv = 0.f;
  if (OPT < 0) return;
  const long i = dst - a.o.g;
  pv = a.o.p[i];
  if (OPT != OPT_GD) av = a.o.s0[i];
  if (OPT == OPT_ADAM || OPT == OPT_FTRL) cv = a.o.s1[i];
}

template <int OPT>
__device__ __forceinline__ void wgf_apply(const WgFinArgs& a, float lr_t, float* dst, float gv) {
  float pv, av, cv;
  wgf_load_state<OPT>(a, dst, pv, av, cv);
  wgf_update<OPT>(a, lr_t, dst, gv, pv, av, cv);
}

// workgroup b of the wgfin work (b < tile_wgs: a tile split; b == tile_wgs: the head reduction);
// PF: k-steps in flight per wave, NSM: largest NS, TQ: combine batch (all size the registers)
template <int OPT, int PF, int NSM, int TQ = 4>
__device__ __forceinline__ void wgfin_body(const WgFinArgs& a, int b, WgfSmem& sm) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float lr_t = OPT == OPT_ADAM ? adam_lr_t(a.o.h, *a.o.step + 1) : a.o.h.lr;
  if (b < a.tile_wgs) {
    int j = 0;
    while (j + 1 < a.njobs && b >= a.jobs[j + 1].wg0) ++j;
    const WgFinJob jb = a.jobs[j];
    const int local = b - jb.wg0;
    const int tile = local / a.ns, wz = local - tile * a.ns;
    const int tm = tile / jb.tiles_n, tn = tile - tm * jb.tiles_n;
    const int row0 = tm * 32, col0 = tn * 32;
    const int k0 = (wz * 4 + wave) * a.kchunk;
    f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;
    float rs[2] = {0.f, 0.f};
    if (tn == 0)
      mma32<PF, true>(jb.A + (size_t)row0 * a.ldk + k0, a.ldk, jb.B + (size_t)col0 * a.ldk + k0, a.ldk,
                      a.kchunk / 32, lane, c00, c01, c10, c11, rs);
    else
      mma32<PF>(jb.A + (size_t)row0 * a.ldk + k0, a.ldk, jb.B + (size_t)col0 * a.ldk + k0, a.ldk,
                a.kchunk / 32, lane, c00, c01, c10, c11);
    const int cr = (lane >> 4) * 4, cc = lane & 15;
    f32x4 acc[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int q = 0; q < 4; ++q) sm.red[wave][ti * 16 + cr + q][tj * 16 + cc] = acc[ti][tj][q];
    if (tn == 0) {  // bias gradient partial: the 4 k-groups of lanes holding rows r, r+16
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        rs[h] += __shfl_xor(rs[h], 16, 64);
        rs[h] += __shfl_xor(rs[h], 32, 64);
      }
      if (lane < 16) {
        sm.bred[wave][lane] = rs[0];
        sm.bred[wave][16 + lane] = rs[1];
      }
    }
    __syncthreads();
    // workgroup partial tile -> slab wz (write-through stores: no release fence needed)
    float* sl = jb.slab + ((size_t)wz * jb.M + row0) * jb.N + col0;
    for (int e = tid; e < 1024; e += 256) {
      const int r = e >> 5, c = e & 31;
      const float v = ((sm.red[0][r][c] + sm.red[1][r][c]) + sm.red[2][r][c]) + sm.red[3][r][c];
      __hip_atomic_store(sl + (size_t)r * jb.N + c, v, HFM_RLX_AGENT);
    }
    if (tn == 0 && tid < 32) {
      const float v = ((sm.bred[0][tid] + sm.bred[1][tid]) + sm.bred[2][tid]) + sm.bred[3][tid];
      __hip_atomic_store(jb.bslab + (size_t)wz * jb.M + row0 + tid, v, HFM_RLX_AGENT);
    }
    hx_drain();
    __syncthreads();
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add(a.tile_ctr + jb.tile0 + tile, 1u, HFM_RLX_AGENT);
      sm.last = (prev % (unsigned)a.ns) == (unsigned)(a.ns - 1);
      if (sm.last) {
        // the tile's last arriver reads the other splits' slabs: ONE agent-scope acquire first
        // (cdna guide §6 G16; the sc1-only form is validated for one workgroup per CU only), its
        // wait, then the barrier releases the reading waves
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (sm.last) {  // the tile's last workgroup: sum the NS slabs in slab order, then the optimizer
      const float* base = jb.slab + (size_t)row0 * jb.N + col0;
      const bool brow = tn == 0 && tid < 32;
      float bv[NSM], bp = 0.f, ba = 0.f, bc = 0.f;
#pragma unroll
      for (int z = 0; z < NSM; ++z)
        bv[z] = (brow && z < a.ns) ? hx_ldf(jb.bslab + (size_t)z * jb.M + row0 + tid) : 0.f;
      if (brow) wgf_load_state<OPT>(a, jb.gb + row0 + tid, bp, ba, bc);
      const bool q8 = OPT >= 0 && jb.w8 != nullptr;
      const unsigned slot = q8 ? (unsigned)((*a.o.step + 1) % 3) : 0u;
      // this thread's 4 elements in batches of TQ, every load of a batch in flight at once:
      // slabs, parameters, optimizer slots (TQ = 4: one round trip; 2: fewer live registers)
#pragma unroll
      for (int q0 = 0; q0 < 4; q0 += TQ) {
        float sv[TQ][NSM], pv[TQ], av[TQ], cv[TQ], am[TQ];
#pragma unroll
        for (int q = 0; q < TQ; ++q) {
          const int e = tid + (q0 + q) * 256, r = e >> 5, c = e & 31;
#pragma unroll
          for (int z = 0; z < NSM; ++z)
            sv[q][z] = z < a.ns ? hx_ldf(base + ((size_t)z * jb.M + r) * jb.N + c) : 0.f;
          wgf_load_state<OPT>(a, jb.gw + (size_t)(row0 + r) * jb.N + col0 + c, pv[q], av[q], cv[q]);
          am[q] = q8 ? __uint_as_float(jb.amax3[((slot + 2) % 3) * jb.M + row0 + r]) : 0.f;
        }
#pragma unroll
        for (int q = 0; q < TQ; ++q) {
          const int e = tid + (q0 + q) * 256, r = e >> 5, c = e & 31;
          float v = 0.f;
#pragma unroll
          for (int z = 0; z < NSM; ++z)
            if (z < a.ns) v += sv[q][z];
          const float np = wgf_update<OPT>(a, lr_t, jb.gw + (size_t)(row0 + r) * jb.N + col0 + c, v, pv[q],
                                           av[q], cv[q]);
          if (OPT >= 0) {
            jb.w16[(size_t)(row0 + r) * jb.N + col0 + c] = f2bf(np);
            jb.wt16[(size_t)(col0 + c) * jb.M + row0 + r] = f2bf(np);
          }
          if (q8) {  // row r's 32 columns sit in 32 consecutive lanes
            const float qs = 0.5f * fp8_pow2_scale(am[q]);
            jb.w8[(size_t)(row0 + r) * jb.N + col0 + c] = (uint8_t)(pack4_fp8(np * qs, 0.f, 0.f, 0.f) & 0xFFu);
            float m = fabsf(np);
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
            if (c == 0) {
              jb.sdq[row0 + r] = 1.f / qs;
              atomicMax(jb.amax3 + slot * jb.M + row0 + r, __float_as_uint(m));
            }
          }
        }
      }
      if (q8 && tn == 0 && tid < 32) jb.amax3[((slot + 1) % 3) * jb.M + row0 + tid] = 0u;
      if (brow) {
        float v = 0.f;
#pragma unroll
        for (int z = 0; z < NSM; ++z)
          if (z < a.ns) v += bv[z];
        wgf_update<OPT>(a, lr_t, jb.gb + row0 + tid, v, bp, ba, bc);
      }
    }
  } else if (b == a.tile_wgs) {
    // head partials [nhead][L + 2]: columns 0..L-1 -> deep_out weights, L -> deep_out bias and
    // fm_bias (both d/dy of the logit), L + 1 -> the loss sum.  Row chunks go through LDS with
    // coalesced loads (all in flight); thread t keeps columns t and t + 256 (a last layer of 256
    // has 258 columns), each summed in row order (deterministic).
    float* buf = &sm.red[0][0][0];
    const int C = a.L + 2;
    const int rows = (4 * 32 * 33) / C;
    float acc[2] = {0.f, 0.f};
    for (int r0 = 0; r0 < a.nhead; r0 += rows) {
      const int nr = min(rows, a.nhead - r0);
      __syncthreads();
      for (int e = tid; e < nr * C; e += 256) buf[e] = a.partial[(size_t)r0 * C + e];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = tid + 256 * k;
        if (c < C)
          for (int r = 0; r < nr; ++r) acc[k] += buf[r * C + c];
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + 256 * k;
      const float v = acc[k];
      if (c < a.L) {
        wgf_apply<OPT>(a, lr_t, a.g_wout + c, v);
      } else if (c == a.L) {
        wgf_apply<OPT>(a, lr_t, a.g_bout, v);
        wgf_apply<OPT>(a, lr_t, a.g_fmbias, v);
      } else if (c == a.L + 1) {
        *a.loss_sum = v;
      }
    }
  }
}
