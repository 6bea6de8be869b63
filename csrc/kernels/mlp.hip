// K6 mlp_fwd / K6-bwd mlp_bwd / K7 head_loss.
//
// Every deep-tower GEMM is expressed as an "NT" product  C[M,N] = A[M,Kd] . B[N,Kd]^T  with
// BOTH operands contiguous along the reduction dimension, because every producer in the step
// writes its output twice — row-major and transposed (fm.hip writes E and E^T, the forward
// epilogue writes H and H^T, the backward epilogues write dZ and dZ^T, the dense optimizer
// keeps W and W^T in bf16).  The gfx950 MFMA fragments for v_mfma_f32_16x16x32_bf16
// (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j=0..7) are then single 16-B global loads
// straight into VGPRs — no LDS staging and no LDS transposes:
//   forward  H_i   = relu(X_i W_i^T + b_i) (.) dropout      A = X_i  [M,K_i]  B = W_i   [N_i,K_i]
//   dgrad    dZ_{i-1} = (dZ_i W_i) (.) mask(H_{i-1})/keep    A = dZ_i [M,N_i]  B = W_i^T [K_i,N_i]
//   wgrad    dW_i  = dZ_i^T X_i  (split over the batch)      A = dZ_i^T [N_i,M] B = X_i^T [K_i,M]
// Tiles: one wave owns a 32x32 output block (2x2 MFMA 16x16x32 tiles, 4 f32x4 accumulators);
// a workgroup is WM x WN waves.  Dropout masks are regenerated from a counter hash
// (utils/rng.py) in the forward epilogue; the backward recovers the mask from H>0, so no mask
// tensor is ever stored.  The whole deep tower is ~1 MFLOP/sample: these kernels are sized for
// occupancy and HBM traffic, not for MFMA peak.
#include "common.h"

enum EpiMode {
  EPI_F32 = 0,        // C f32 [M,N] (split-K: slab blockIdx.z at C + z*M*N)
  EPI_FWD = 1,        // +bias, relu, dropout -> H bf16 [M,N] and H^T bf16 [N,M]
  EPI_DGRAD = 2,      // mask by Hprev>0, *scale -> dZ bf16 [M,N] and dZ^T [N,M]
  EPI_FWD_EVAL = 3,   // +bias, relu (no dropout), H only
  EPI_RELU_F32 = 4,   // +bias, relu -> f32 [M,N] (batch-norm input: BN divides by the batch
                      // std, which would amplify bf16 rounding of R by mean/std)
};

struct EpiArgs {
  const float* bias;       // [N]
  const bf16* hprev;       // EPI_DGRAD: activation whose >0 pattern masks the gradient [M,N]
  float scale;             // EPI_DGRAD: 1/keep of that activation's dropout
  uint32_t seed, layer, keep_thr;
  int drop;                // apply dropout
  const int64_t* step;     // device step counter (dropout salt)
  void* out;               // f32 C or bf16 H/dZ
  bf16* out_t;             // transposed copy (nullable)
};

// One 16x16 accumulator tile's epilogue: lane (rowb.., col) holds rows rowb + j, j = 0..3 (MFMA C/D
// map), shared by every NT GEMM kernel below.
template <int EPI>
__device__ __forceinline__ void epi_store(const EpiArgs& ep, const f32x4 acc, int rowb, int col, int M,
                                          int N, uint32_t salt) {
  if (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(ep.out) + (size_t)blockIdx.z * M * N;
#pragma unroll
    for (int j = 0; j < 4; ++j) C[(size_t)(rowb + j) * N + col] = acc[j];
  } else if (EPI == EPI_RELU_F32) {
    float* C = reinterpret_cast<float*>(ep.out);
    const float bc = ep.bias[col];
#pragma unroll
    for (int j = 0; j < 4; ++j) C[(size_t)(rowb + j) * N + col] = fmaxf(acc[j] + bc, 0.f);
  } else {
    bf16x4 tv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = rowb + j;
      float v = acc[j];
      if (EPI == EPI_FWD || EPI == EPI_FWD_EVAL) {
        v = fmaxf(v + ep.bias[col], 0.f);
        if (EPI == EPI_FWD && ep.drop)
          v = dropout_keep((uint32_t)(row * N + col), salt, ep.keep_thr) ? v * ep.scale : 0.f;
      } else {  // EPI_DGRAD (hprev == nullptr: plain bf16 store, e.g. dX0 of layer 1)
        v = (!ep.hprev || bf2f(ep.hprev[(size_t)row * N + col]) > 0.f) ? v * ep.scale : 0.f;
      }
      const bf16 hv = f2bf(v);
      reinterpret_cast<bf16*>(ep.out)[(size_t)row * N + col] = hv;
      tv[j] = hv;
    }
    if (ep.out_t) *reinterpret_cast<bf16x4*>(ep.out_t + (size_t)col * M + rowb) = tv;
  }
}

template <int WM, int WN, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) gemm_nt_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int row0 = blockIdx.x * (WM * 32) + wm * 32;
  const int col0 = blockIdx.y * (WN * 32) + wn * 32;
  const int k0 = blockIdx.z * kchunk;
  const int r = lane & 15, kq = (lane >> 4) * 8;

  const bf16* a0 = A + (size_t)(row0 + r) * lda + k0 + kq;
  const bf16* a1 = a0 + (size_t)16 * lda;
  const bf16* b0 = Bm + (size_t)(col0 + r) * ldb + k0 + kq;
  const bf16* b1 = b0 + (size_t)16 * ldb;

  f32x4 c00 = {0, 0, 0, 0}, c01 = c00, c10 = c00, c11 = c00;

  // Register ring of PF k-steps: the fragments of step k+PF are requested while step k is
  // multiplied, so PF x 4 KB of loads per wave are in flight.  These GEMMs are short in
  // MFMA work (4 MFMAs per 4 fragment loads) and latency-bound without it: one wave per
  // SIMD, 10 k-steps, each waiting a full memory round trip (measured 14 us -> see profiles/).
  constexpr int PF = 4;
  const int nsteps = kchunk / 32;
  bf16x8 ra0[PF], ra1[PF], rb0[PF], rb1[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    if (j < nsteps) {
      ra0[j] = *reinterpret_cast<const bf16x8*>(a0 + j * 32);
      ra1[j] = *reinterpret_cast<const bf16x8*>(a1 + j * 32);
      rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + j * 32);
      rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + j * 32);
    }
  }
  for (int kb = 0; kb < nsteps; kb += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int ks = kb + j;
      if (ks < nsteps) {
        c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra0[j], rb0[j], c00, 0, 0, 0);
        c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra0[j], rb1[j], c01, 0, 0, 0);
        c10 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra1[j], rb0[j], c10, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra1[j], rb1[j], c11, 0, 0, 0);
        const int kn = (ks + PF) * 32;
        if (ks + PF < nsteps) {
          ra0[j] = *reinterpret_cast<const bf16x8*>(a0 + kn);
          ra1[j] = *reinterpret_cast<const bf16x8*>(a1 + kn);
          rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + kn);
          rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + kn);
        }
      }
    }
  }

  // C/D map: col = lane&15, row = (lane>>4)*4 + j
  const int cr = (lane >> 4) * 4, cc = lane & 15;
  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  const f32x4 accs[2][2] = {{c00, c01}, {c10, c11}};
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
      epi_store<EPI>(ep, accs[ti][tj], row0 + ti * 16 + cr, col0 + tj * 16 + cc, M, N, salt);
}

template <int WM, int WN, int EPI>
static int launch_gemm(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                       int splitk, const EpiArgs& ep, hipStream_t st) {
  if (M % (WM * 32) || N % (WN * 32) || Kd % (32 * splitk)) return (int)hipErrorInvalidValue;
  dim3 grid(M / (WM * 32), N / (WN * 32), splitk);
  hipLaunchKernelGGL((gemm_nt_kernel<WM, WN, EPI>), grid, dim3(WM * WN * 64), 0, st, A, lda, B, ldb,
                     M, N, Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ wide-layer GEMM (tile 8)
// The per-layer path of towers the fused kernel cannot hold (the reference's GPU recipe,
// deep_layers 4096,4096,4096, DOC p.37; batch norm, HVD:204-210): GEMMs of 2 * 16384 * 4096 *
// 4096 = 0.55 TFLOP each, where the register-fed 32x32 tiles above re-read every operand from
// L2 per wave.  Here a 256-thread workgroup (2 x 2 waves) owns a 128 x 128 output tile; the
// k-loop stages 64-deep A and B panels HBM -> LDS with 16-B LDS-DMA loads
// (global_load_lds_dwordx4, no VGPR round trip) into two buffers, so panel t+1 streams in while
// the MFMAs consume panel t.  Each wave computes 64 x 64 = 4 x 4 MFMA 16x16x32 tiles (16 f32x4
// accumulators) from bf16x8 fragments read with ds_read_b128.
//   LDS image of a panel: [128 rows][64 bf16] = 128-B rows, the 16-B chunk c of row r stored
//   at slot c ^ ((r >> 1) & 7).  A 16-lane ds_read group reads 16 consecutive rows at one chunk:
//   rows of equal parity share a 256-B bank row only at distinct slots -> conflict-free.  The
//   DMA writes lane-linear (wave base + 16 * lane), so the swizzle is applied to the per-lane
//   GLOBAL source address (lane l of an 8-row piece fetches chunk (l & 7) ^ swz(row)).
//   Tiles are numbered XCD-aware: consecutive tile ids (same 128-row A panel, neighbouring B
//   panels) run on the same XCD and share its L2.
constexpr int GL_BM = 128, GL_BN = 128, GL_BK = 64, GL_THREADS = 256;
constexpr int GL_PANEL = GL_BM * GL_BK * 2;       // bytes of one A (or B) panel
static_assert(GL_BM == GL_BN, "square tile: A and B panels share the staging code");

__device__ __forceinline__ int gl_slot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// stage one 128 x 64 panel (rows row0.., k from k0) into `lds`: 16 DMA pieces of 8 rows, 4 per wave
__device__ __forceinline__ void gl_stage(char* lds, const bf16* __restrict__ g, int ld, int row0, int k0,
                                         int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int r = piece * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const bf16* src = g + (size_t)(row0 + r) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + piece * 1024), 16, 0, 0);
  }
}

template <int EPI>
__global__ void __launch_bounds__(GL_THREADS, 2) gemm_lds_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  // ONE __shared__ array (a second one can make hipcc drain the DMA queue before every ds_read)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * GL_PANEL];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile id (bijective for any tile count): the blocks the hardware sends to one XCD
  // (bid % 8) take a contiguous range of tile ids
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int tid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tiles_n = N / GL_BN;
  const int m0 = (tid / tiles_n) * GL_BM, n0 = (tid % tiles_n) * GL_BN;
  const int kb = blockIdx.z * kchunk;
  const int nt = kchunk / GL_BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gl_stage(smem, A, lda, m0, kb, wave, lane);
  gl_stage(smem + GL_PANEL, Bm, ldb, n0, kb, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nt; ++t) {
    char* cur = smem + (t & 1) * 2 * GL_PANEL;
    if (t + 1 < nt) {                     // the next panels stream in behind this step's MFMAs
      char* nxt = smem + ((t + 1) & 1) * 2 * GL_PANEL;
      gl_stage(nxt, A, lda, m0, kb + (t + 1) * GL_BK, wave, lane);
      gl_stage(nxt + GL_PANEL, Bm, ldb, n0, kb + (t + 1) * GL_BK, wave, lane);
    }
    const char* pa = cur;
    const char* pb = cur + GL_PANEL;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + fq;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = *reinterpret_cast<const bf16x8*>(pa + gl_slot(wm * 64 + i * 16 + fr, c));
        b[i] = *reinterpret_cast<const bf16x8*>(pb + gl_slot(wn * 64 + i * 16 + fr, c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    // the next panels have landed (this wave's DMA) and every wave is done reading `cur`
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  const int cr = fq * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      epi_store<EPI>(ep, acc[i][j], m0 + wm * 64 + i * 16 + cr, n0 + wn * 64 + j * 16 + fr, M, N, salt);
}

// ------------------------------------------------------------------ ping-pong GEMM (tile 9)
// 256 x 256 workgroup tile, 512 threads = 8 waves in two groups of 4 (group g owns output rows
// g*128.., wave c of a group owns columns c*64..: a 128 x 64 block per wave, 8 x 4 MFMA 16x16x32
// tiles = 32 f32x4 accumulators).  Each SIMD hosts one wave of each group, and the groups run one
// barrier apart ("ping-pong"): between two consecutive s_barriers one group issues the LDS
// fragment reads (and LDS-DMA staging) of its next phase while the other group's 16 MFMAs run, so
// the matrix pipe of every SIMD alternates between its two waves instead of idling through each
// wave's reads.  A 64-deep K-tile is 4 phases, one 64 x 32 output quadrant each, in the snake
// order (A0,B0) (A0,B1) (A1,B1) (A1,B0): a phase re-reads only the operand half that changes.
//   slot s (the interval between two barriers): group 0 loads phase s/2 when s is even and
//   computes it when s is odd; group 1 is one slot later.  K-tile t occupies slots 8t .. 8t+8.
//   Staging of K-tile t+1 into buffer (t+1)&1 (last read by K-tile t-1, whose reads every wave
//   retired by slot 8t): group 1 in its load slots 8t+1, 8t+3, group 0 in 8t+2, 8t+4 (4 pieces of
//   1 KB per slot per wave); each wave waits for its own DMA (vmcnt(0)) in its phase-3 load slot
//   (slots 8t+6 / 8t+7), so the barrier before slot 8t+8 publishes all of K-tile t+1 to every
//   wave -- one counted wait per K-tile, DMA in flight across 2-5 barriers.
// LDS: 2 buffers x (A 256 x 64 + B 256 x 64) bf16 = 128 KB, the swizzled image of tile 8.
constexpr int PP_BM = 256, PP_BK = 64, PP_THREADS = 512;
constexpr int PP_PANEL = PP_BM * PP_BK * 2;            // 32 KB: one operand's K-tile
constexpr int PP_BUF = 2 * PP_PANEL;                   // A + B of one K-tile

// 4 DMA pieces (8 rows x 128 B each) of a 256-row panel: pieces [first, first + 4)
__device__ __forceinline__ void pp_stage4(char* lds, const bf16* __restrict__ g, int ld, int row0, int k0,
                                          int first, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = first + i;
    const int r = piece * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const bf16* src = g + (size_t)(row0 + r) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + piece * 1024), 16, 0, 0);
  }
}

// pieces [P0, P1) of a wave's 8 staging pieces of one K-tile: 0..3 = A pieces 4w.., 4..7 = B pieces 4w..
// `off[p]`: the lane's element offset of piece p in its operand at k = 0 (hoisted out of the loop:
// a piece then costs one address add instead of the row / swizzle arithmetic)
template <int P0, int P1>
__device__ __forceinline__ void pp_stage_pieces(char* buf, const bf16* __restrict__ A, const bf16* __restrict__ Bm,
                                                const int* off, int k0, int wave) {
#pragma unroll
  for (int p = P0; p < P1; ++p) {
    const bool isb = p >= 4;
    const int piece = wave * 4 + (p & 3);
    const bf16* src = (isb ? Bm : A) + off[p] + k0;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + (isb ? PP_PANEL : 0) + piece * 1024),
                                     16, 0, 0);
  }
}

// SPREAD 0: 4 + 4 pieces in two load slots per group (group 1: phases 0, 1; group 0: 1, 2), each
//           wave's vmcnt(0) in its phase-3 load slot.
// SPREAD 1: 3 + 3 + 2 pieces over three load slots (group 1: phases 0-2; group 0: 1-3); group 1
//           waits in its phase-3 load slot, group 0 at the end of its phase-3 compute slot (its
//           last pieces leave in that phase's load slot; the barrier after the wait publishes
//           them before either group reads the K-tile).
template <int EPI, int SPREAD>
__global__ void __launch_bounds__(PP_THREADS, 1) gemm_pp_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_BUF];   // (the only __shared__ object)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = wave >> 2, wc = wave & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int tid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (bid >> 3);
  const int tiles_n = N / PP_BM;
  const int m0 = (tid / tiles_n) * PP_BM, n0 = (tid % tiles_n) * PP_BM;
  const int kb = blockIdx.z * kchunk;
  const int nt = kchunk / PP_BK;
  const int fr = lane & 15, fq = lane >> 4;
  // fragment byte offsets in a panel: row r = base + 16 i + fr has swizzle (r >> 1) & 7 = (fr >> 1) & 7
  // (the row bases are multiples of 16), so a read is a lane base + a compile-time offset
  const int swz = (fr >> 1) & 7;
  const int la[2] = {(grp * 128 + fr) * 128 + ((fq ^ swz) << 4), (grp * 128 + fr) * 128 + (((4 + fq) ^ swz) << 4)};
  const int lb[2] = {(wc * 64 + fr) * 128 + ((fq ^ swz) << 4), (wc * 64 + fr) * 128 + (((4 + fq) ^ swz) << 4)};
  int soff[8];                            // (SPREAD 1) per-piece source offsets at k = 0
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r = (wave * 4 + (p & 3)) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    soff[p] = p < 4 ? (m0 + r) * lda + c * 8 : (n0 + r) * ldb + c * 8;
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tile 0 into buffer 0 (pieces 4w..4w+3 of A and of B per wave)
  pp_stage4(smem, A, lda, m0, kb, wave * 4, lane);
  pp_stage4(smem + PP_PANEL, Bm, ldb, n0, kb, wave * 4, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (grp == 1) {                         // the stagger: group 1 runs one slot behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }

  bf16x8 fa[4][2], fb[2][2];
  for (int t = 0; t < nt; ++t) {
    const char* pa = smem + (t & 1) * PP_BUF;
    const char* pb = pa + PP_PANEL;
    char* nxt = smem + ((t + 1) & 1) * PP_BUF;
    const bool more = t + 1 < nt;
    const int kn = kb + (t + 1) * PP_BK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qa = (q == 0 || q == 1) ? 0 : 1;     // snake: (0,0) (0,1) (1,1) (1,0)
      const int qb = (q == 0 || q == 3) ? 0 : 1;
      // ---- load slot: this phase's fragments (+ staging of the next K-tile)
      if (q == 3 && (SPREAD == 0 || grp == 1))
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // my DMA of K-tile t+1 landed
      if (q == 0 || q == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fa[i][ks] = *reinterpret_cast<const bf16x8*>(pa + la[ks] + (qa * 64 + i * 16) * 128);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fb[j][ks] = *reinterpret_cast<const bf16x8*>(pb + lb[ks] + (qb * 32 + j * 16) * 128);
      if (SPREAD == 0) {
        // group 1 stages in its phase-0/1 load slots, group 0 in its phase-1/2 slots
        if (more && ((grp == 1 && q == 0) || (grp == 0 && q == 1)))
          pp_stage4(nxt, A, lda, m0, kn, wave * 4, lane);
        if (more && ((grp == 1 && q == 1) || (grp == 0 && q == 2)))
          pp_stage4(nxt + PP_PANEL, Bm, ldb, n0, kn, wave * 4, lane);
      } else if (more) {
        const int sl = q - (grp == 0 ? 1 : 0);     // this group's staging slot 0..2
        if (sl == 0) pp_stage_pieces<0, 3>(nxt, A, Bm, soff, kn, wave);
        if (sl == 1) pp_stage_pieces<3, 6>(nxt, A, Bm, soff, kn, wave);
        if (sl == 2) pp_stage_pieces<6, 8>(nxt, A, Bm, soff, kn, wave);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- compute slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qa * 4 + i][qb * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (SPREAD == 1 && q == 3 && grp == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // (every wave passes the same number of barriers)

#ifdef HFM_PP_NOEPI   // (diagnostic build: epilogue replaced by one store per lane -- timing only)
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  if (sum == 1.2345e-30f) reinterpret_cast<float*>(ep.out)[threadIdx.x] = sum;
  return;
#endif
  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  __syncthreads();                      // (every wave past its last K-tile read: the images reuse it)
  epi_tile_lds<EPI, 8, 4>(ep, acc, smem + wave * 16384, lane, m0 + grp * 128, n0 + wc * 64, M, N, salt);
}

// ------------------------------------------------------------------ LDS-staged wave epilogue
// A wave's MI x NJ accumulator tiles (rows row0 + 16 i + 4 fq + k, cols col0 + 16 j + fr) leave
// through a wave-private 16 KB LDS image, so every global access is a 16-byte row chunk: the output
// rows (bf16 H / dZ, or the f32 C slab), and the dgrad mask's hprev rows.  The per-element
// epilogue (epi_store) wrote 2- or 4-byte scattered stores and read hprev 2 bytes at a time: with
// it the 256x256 tiles spent 19-41 % of a 16384x4096x4096 GEMM there (timing build without it:
// profiles/r6_gemm_epilogue_ablation.log).  Same values, bit for bit: bias / relu / dropout in
// registers as before; the dgrad mask is applied to the bf16-rounded value (rounding and a mask to
// +0 commute).  out_t keeps its 8-byte column stores (masked values re-read from the image).
// Image: rows of NJ * 16 elements, 16-byte chunk c of row r at chunk c ^ (r mod chunks-per-row).
// Caller: every wave of the workgroup is past its last LDS read of the main loop.
template <int EPI, int MI, int NJ>
__device__ __forceinline__ void epi_tile_lds(const EpiArgs& ep, const f32x4 (&acc)[MI][NJ], char* img, int lane,
                                             int row0, int col0, int M, int N, uint32_t salt) {
  constexpr bool F32 = EPI == EPI_F32 || EPI == EPI_RELU_F32;
  constexpr int ES = F32 ? 4 : 2;
  constexpr int RB = NJ * 16 * ES;           // image row bytes
  constexpr int CPR = RB / 16;               // 16-byte chunks per row
  constexpr int ROWS = 16384 / RB;           // rows per pass
  constexpr int MIP = ROWS / 16;             // m-tiles per pass
  static_assert(MI % MIP == 0 && (CPR & (CPR - 1)) == 0, "image geometry");
  const int fr = lane & 15, fq = lane >> 4;
  const bool mask = EPI == EPI_DGRAD && ep.hprev != nullptr;
  auto wsync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto eoff = [](int r, int cb) { return r * RB + ((((cb >> 4) ^ (r & (CPR - 1)))) << 4) + (cb & 15); };
#pragma unroll
  for (int p = 0; p < MI / MIP; ++p) {
    // 1. registers -> image (and out_t straight from the registers when no mask applies)
#pragma unroll
    for (int ii = 0; ii < MIP; ++ii) {
      const int i = p * MIP + ii;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = j * 16 + fr, col = col0 + c;
        bf16x4 tv;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ri = ii * 16 + fq * 4 + k, row = row0 + i * 16 + fq * 4 + k;
          float v = acc[i][j][k];
          if (EPI == EPI_FWD || EPI == EPI_FWD_EVAL) {
            v = fmaxf(v + ep.bias[col], 0.f);
            if (EPI == EPI_FWD && ep.drop)
              v = dropout_keep((uint32_t)(row * N + col), salt, ep.keep_thr) ? v * ep.scale : 0.f;
          } else if (EPI == EPI_DGRAD) {
            v = v * ep.scale;
          } else if (EPI == EPI_RELU_F32) {
            v = fmaxf(v + ep.bias[col], 0.f);
          }
          if (F32) {
            *reinterpret_cast<float*>(img + eoff(ri, c * 4)) = v;
          } else {
            const bf16 hv = f2bf(v);
            *reinterpret_cast<bf16*>(img + eoff(ri, c * 2)) = hv;
            tv[k] = hv;
          }
        }
        if (!F32 && !mask && ep.out_t)
          *reinterpret_cast<bf16x4*>(ep.out_t + (size_t)col * M + row0 + i * 16 + fq * 4) = tv;
      }
    }
    wsync();
    // 2. image rows -> global rows, 16 bytes per lane (dgrad: hprev rows masked in, written back)
    const int rbase = row0 + p * ROWS;
#pragma unroll 4
    for (int e = lane; e < ROWS * CPR; e += 64) {
      const int r = e / CPR, q = e % CPR;
      char* ip = img + r * RB + ((q ^ (r & (CPR - 1))) << 4);
      uint4 v = *reinterpret_cast<const uint4*>(ip);
      const size_t g = (size_t)(rbase + r) * N + col0 + q * (16 / ES);
      if (F32) {
        *reinterpret_cast<uint4*>(reinterpret_cast<float*>(ep.out) + (size_t)blockIdx.z * M * N + g) = v;
      } else {
        if (mask) {
          const uint4 h = *reinterpret_cast<const uint4*>(ep.hprev + g);
          uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
          const uint32_t* hw = reinterpret_cast<const uint32_t*>(&h);
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const bool lo = __uint_as_float(hw[w] << 16) > 0.f, hi = __uint_as_float(hw[w] & 0xFFFF0000u) > 0.f;
            vw[w] &= (lo ? 0x0000FFFFu : 0u) | (hi ? 0xFFFF0000u : 0u);
          }
          if (ep.out_t) *reinterpret_cast<uint4*>(ip) = v;
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(ep.out) + g) = v;
      }
    }
    if (!F32 && mask && ep.out_t) {    // out_t of the masked values: the lane's own 4-row columns
      wsync();
#pragma unroll
      for (int ii = 0; ii < MIP; ++ii)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = j * 16 + fr;
          bf16x4 tv;
#pragma unroll
          for (int k = 0; k < 4; ++k) tv[k] = *reinterpret_cast<const bf16*>(img + eoff(ii * 16 + fq * 4 + k, c * 2));
          *reinterpret_cast<bf16x4*>(ep.out_t + (size_t)(col0 + c) * M + rbase + ii * 16 + fq * 4) = tv;
        }
    }
    wsync();                           // (the next pass overwrites the image)
  }
}

// ------------------------------------------------------------------ register-blocked GEMM (tile 11)
// 256 x 256 workgroup tile, 4 waves (one per SIMD), each owning a 128 x 128 block: 8 x 8 MFMA
// 16x16x32 tiles = 64 f32x4 accumulators (256 registers, the accumulation file).  Per 64-deep
// K-tile a wave reads 2 x (8 + 8) fragments for 128 MFMAs -- a quarter of an LDS read per MFMA,
// half the ping-pong tile's (profiles/r6_gemm_pmc_raw.md: its LDS-issue stalls and barrier waits
// held MFMA busy at 39 %).  Fragments of the second 32-deep half are read while the first half's
// 64 MFMAs run; the next K-tile streams in by LDS-DMA (16 pieces per wave) into the other buffer,
// one vmcnt(0) + barrier per K-tile.  LDS: 2 x (A 256 x 64 + B 256 x 64) bf16 = 128 KB.
constexpr int RB_THREADS = 256;

template <int EPI>
__global__ void __launch_bounds__(RB_THREADS) __attribute__((amdgpu_waves_per_eu(1, 1))) gemm_rb_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_BUF];   // (the only __shared__ object)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wcn = wave & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int tid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (bid >> 3);
  const int tiles_n = N / PP_BM;
  const int m0 = (tid / tiles_n) * PP_BM, n0 = (tid % tiles_n) * PP_BM;
  const int kb = blockIdx.z * kchunk;
  const int nt = kchunk / PP_BK;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K-tile staging: 32 A pieces + 32 B pieces of 1 KB, 8 + 8 per wave (pieces 0-7: A, 8-15: B);
  // per-lane source offsets at k = 0 hoisted
  int soff[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int r = (wave * 8 + (p & 7)) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    soff[p] = p < 8 ? (m0 + r) * lda + c * 8 : (n0 + r) * ldb + c * 8;
  }
  auto piece = [&](char* buf, int k0, int p) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)((p < 8 ? A : Bm) + soff[p] + k0),
        (__attribute__((address_space(3))) void*)(buf + (p < 8 ? 0 : PP_PANEL) + (wave * 8 + (p & 7)) * 1024),
        16, 0, 0);
  };
  // fragment byte offsets (rows base + 16 i + fr: swizzle (fr >> 1) & 7), k-halves h = 0, 1
  const int swz = (fr >> 1) & 7;
  const int la0 = (wr * 128 + fr) * 128 + ((fq ^ swz) << 4), la1 = (wr * 128 + fr) * 128 + (((4 + fq) ^ swz) << 4);
  const int lb0 = (wcn * 128 + fr) * 128 + ((fq ^ swz) << 4), lb1 = (wcn * 128 + fr) * 128 + (((4 + fq) ^ swz) << 4);
#pragma unroll
  for (int p = 0; p < 16; ++p) piece(smem, kb, p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16x8 fa[8], fb[8], ga[8], gb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fb[i] = *reinterpret_cast<const bf16x8*>(smem + PP_PANEL + lb0 + i * 2048);
    fa[i] = *reinterpret_cast<const bf16x8*>(smem + la0 + i * 2048);
  }
  // Issue order pinned per K-tile (sched_barrier around every non-MFMA op: one wave per SIMD, so
  // any stall of the in-order stream idles the matrix core):
  //   half 0: 64 MFMAs; a staging DMA of the next K-tile after each of the first 16, a fragment
  //           read of half 1 after each of the next 16
  //   half 1: 48 MFMAs; vmcnt(0) lgkmcnt(0) + barrier; the last 16 MFMAs each followed by a
  //           fragment read of the next K-tile's half 0 (from the buffer that just landed)
  for (int t = 0; t < nt; ++t) {
    const char* pa = smem + (t & 1) * PP_BUF;
    char* nb = smem + ((t + 1) & 1) * PP_BUF;
    const bool more = t + 1 < nt;
    const int kn = kb + (more ? t + 1 : t) * PP_BK;   // the last K-tile re-stages itself (idle buffer)
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int i = n >> 3, j = n & 7;
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (n < 16) {
        piece(nb, kn, n);
        __builtin_amdgcn_sched_barrier(0);
      } else if (n < 32) {
        const int q = n - 16;
        if (q < 8) gb[q] = *reinterpret_cast<const bf16x8*>(pa + PP_PANEL + lb1 + q * 2048);
        else ga[q - 8] = *reinterpret_cast<const bf16x8*>(pa + la1 + (q - 8) * 2048);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int n = 0; n < 48; ++n) {
      acc[n >> 3][n & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[n >> 3], gb[n & 7], acc[n >> 3][n & 7], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 48; n < 64; ++n) {
      acc[n >> 3][n & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[n >> 3], gb[n & 7], acc[n >> 3][n & 7], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
        const int q = n - 48;
        if (q < 8) fb[q] = *reinterpret_cast<const bf16x8*>(nb + PP_PANEL + lb0 + q * 2048);
        else fa[q - 8] = *reinterpret_cast<const bf16x8*>(nb + la0 + (q - 8) * 2048);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  const int cr = fq * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      epi_store<EPI>(ep, acc[i][j], m0 + wr * 128 + i * 16 + cr, n0 + wcn * 128 + j * 16 + fr, M, N, salt);
}

// ------------------------------------------------------------------ K-half ring GEMM (tile 12)
// 256 x 256 workgroup tile, 8 waves as two staggered groups (G = wave >> 2 owns rows G*128..+128,
// wc = wave & 3 columns wc*64..+64: acc[8][4] per wave), like tile 9/10 -- but the K loop runs over
// 32-deep K-HALVES held in a ring of 4 LDS buffers (A [256][32] + B [256][32] bf16, 32 KB each:
// 128 KB), so the LDS-DMA of K-half h + 3 is issued while h is consumed and stays in flight
// across ~8 barriers, retired by a COUNTED vmcnt(8) (never 0 in the steady state).  Tile 9/10's
// 64-deep K-tiles in two buffers left the DMA in flight for about one phase before its vmcnt(0).
// Per K-half and wave: 2 phases of 16 MFMAs (rows 4s..4s+3 of the wave's 8 m-tiles x its 4
// n-tiles); B fragments read in phase 0, A fragments of the phase's rows in each phase.
// Slot schedule (G1 one slot behind G0: each SIMD alternates a G0 and a G1 wave between loading
// and MFMAs): slot 4h + 2s = G0 load / G1 compute of phase (h, s), 4h + 2s + 1 the reverse.
//   staging of K-half h + 3 into buffer (h - 1) % 4: G0 all 4 DMAs in its load slot of (h, 1)
//   (slot 4h + 2), G1 two in each of its load slots of (h, 0) / (h, 1) (slots 4h + 1, 4h + 3):
//   every read of K-half h - 1 was retired by its reader's lgkmcnt(0) before the barrier that
//   ends slot 4h.
//   retirement of K-half h + 1 before slot 4h + 4 (its first read): G0 at the end of its compute
//   slot 4h + 3, G1 in its load slot 4h + 3 after issuing its DMAs -- 8 newer DMAs (K-halves
//   h + 2, h + 3) may stay in flight; vmcnt(0) where fewer were issued (the last K-halves).
// Image of a K-half operand: rows of 64 B, lane-linear DMA pieces of 16 rows; 16-B chunk c of row r
// stored at slot c ^ ((r >> 2) & 3) (16 rows x one chunk = 16 distinct bank groups).
constexpr int P8_KH = 32;                       // K-half depth
constexpr int P8_OP = PP_BM * P8_KH * 2;        // 16 KB: one operand's K-half
constexpr int P8_BUF = 2 * P8_OP;               // A + B: 32 KB, 4 in the ring

template <int EPI>
__global__ void __launch_bounds__(PP_THREADS, 1) gemm_p8_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[4 * P8_BUF];   // (the only __shared__ object)
  // (wave-uniform in an SGPR: the group branches below are scalar)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int grp = wave >> 2, wc = wave & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int tid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (bid >> 3);
  const int tiles_n = N / PP_BM;
  const int m0 = (tid / tiles_n) * PP_BM, n0 = (tid % tiles_n) * PP_BM;
  const int kb = blockIdx.z * kchunk;
  const int nkh = kchunk / P8_KH;
  const int fr = lane & 15, fq = lane >> 4;
  // this wave's 4 staging pieces per K-half: A pieces 2w, 2w + 1 and B pieces 2w, 2w + 1
  int soff[4], doff[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int piece = wave * 2 + (p & 1);
    const int r = piece * 16 + (lane >> 2);
    const int c = (lane & 3) ^ ((r >> 2) & 3);
    soff[p] = p < 2 ? (m0 + r) * lda + c * 8 : (n0 + r) * ldb + c * 8;
    doff[p] = (p < 2 ? 0 : P8_OP) + piece * 1024;
  }
  auto stage = [&](int h, int p) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)((p < 2 ? A : Bm) + soff[p] + kb + h * P8_KH),
        (__attribute__((address_space(3))) void*)(smem + (h & 3) * P8_BUF + doff[p]), 16, 0, 0);
  };
  // fragment byte offsets: row base + fr (bases multiples of 16: swizzle (fr >> 2) & 3), chunk fq
  const int cs = (fq ^ ((fr >> 2) & 3)) << 4;
  const int la = (grp * 128 + fr) * 64 + cs;
  const int lb = P8_OP + (wc * 64 + fr) * 64 + cs;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-halves 0, 1, 2 in flight, 0 and 1 retired (the 4 DMAs of 2 may remain)
#pragma unroll
  for (int h = 0; h < 3; ++h)
#pragma unroll
    for (int p = 0; p < 4; ++p) stage(h, p);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (grp == 1) {                         // the stagger: group 1 runs one slot behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  // fragments one phase ahead: fa[phase parity], fb[K-half parity]; phase (0, 0)'s now
  bf16x8 fa[2][4], fb[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = *reinterpret_cast<const bf16x8*>(smem + lb + j * 1024);
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[0][i] = *reinterpret_cast<const bf16x8*>(smem + la + i * 1024);

  // phase (h, s) with h parity HP (fragment sets static after unrolling by two K-halves)
  auto phase = [&](int h, auto HPc, auto Sc) {
    constexpr int HP = decltype(HPc)::value, S = decltype(Sc)::value;
    const bool st3 = h + 3 < nkh;
    // ---- load slot: staging of K-half h + 3, the retirement of h + 2 (group 1)
    if (st3) {
      if (grp == 0 && S == 1) {
#pragma unroll
        for (int p = 0; p < 4; ++p) stage(h + 3, p);
      } else if (grp == 1) {
        stage(h + 3, 2 * S);
        stage(h + 3, 2 * S + 1);
      }
    }
    if (grp == 1 && S == 1) {
      if (st3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- compute slot: this phase's fragments were read one slot ago
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    // next phase: (h, 1) -> A rows 4-7 of K-half h; (h + 1, 0) -> B and A rows 0-3 of K-half h + 1
    const bool nxt = S == 0 || h + 1 < nkh;
    const char* nbuf = smem + ((S == 0 ? h : h + 1) & 3) * P8_BUF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[S * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[S][i], fb[HP][j], acc[S * 4 + i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (nxt) {
          if (S == 0 && j == 1) fa[1][i] = *reinterpret_cast<const bf16x8*>(nbuf + la + (4 + i) * 1024);
          if (S == 1 && j == 1) fb[HP ^ 1][i] = *reinterpret_cast<const bf16x8*>(nbuf + lb + i * 1024);
          if (S == 1 && j == 3) fa[0][i] = *reinterpret_cast<const bf16x8*>(nbuf + la + i * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (grp == 0 && S == 1) {              // retire K-half h + 2 (h + 3's DMAs may stay in flight)
      if (st3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int h = 0; h < nkh; h += 2) {
    phase(h, I0{}, I0{});
    phase(h, I0{}, I1{});
    phase(h + 1, I1{}, I0{});
    phase(h + 1, I1{}, I1{});
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // (every wave passes the same number of barriers)

  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  __syncthreads();                      // (every wave past its last K-tile read: the images reuse it)
  epi_tile_lds<EPI, 8, 4>(ep, acc, smem + wave * 16384, lane, m0 + grp * 128, n0 + wc * 64, M, N, salt);
}

template <int EPI>
static int launch_gemm_p8(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                          int splitk, const EpiArgs& ep, hipStream_t st) {
  // (an even number of K-halves per split, at least 4: the loop runs K-half pairs, the prologue
  // stages three)
  if (M % PP_BM || N % PP_BM || splitk < 1 || Kd % (2 * P8_KH * splitk) || Kd / splitk < 4 * P8_KH || lda % 8 ||
      ldb % 8 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  dim3 grid((M / PP_BM) * (N / PP_BM), 1, splitk);
  hipLaunchKernelGGL((gemm_p8_kernel<EPI>), grid, dim3(PP_THREADS), 0, st, A, lda, B, ldb, M, N,
                     Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ register-blocked K-half ring (tile 13)
// The shape of hipBLASLt's kernel on these GEMMs (profiles/r6_gemm_pmc_raw.md: 4 waves per 256 x 256
// workgroup, one wave per SIMD, half the LDS reads per MFMA of the 8-wave tiles): each wave owns a
// 128 x 128 block (acc[8][8], 256 accumulation registers), fed from tile 12's ring of four 32-deep
// K-half buffers.  Per K-half and wave: 64 MFMAs on fragments read during the PREVIOUS K-half
// (two register sets), the 8 staging DMAs of K-half h + 3 issued after the first 8 MFMAs, the 16
// fragment reads of K-half h + 1 spread over the rest; one lgkmcnt(0) + counted vmcnt(8) (K-half
// h + 2 retired, h + 3 in flight) + barrier per K-half.  Order pinned by sched_barrier.
//   WAR: buffer (h + 3) & 3 = (h - 1) & 3 was last read during K-half h - 2, retired by the
//   lgkmcnt(0) before the barrier that ends h - 2.  RAW: K-half h + 1 (read during h) was retired
//   by every wave's vmcnt before the barrier that ends h - 1.
template <int EPI>
__global__ void __launch_bounds__(RB_THREADS) __attribute__((amdgpu_waves_per_eu(1, 1))) gemm_r8_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bm, int ldb, int M, int N,
    int kchunk, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) char smem[4 * P8_BUF];   // (the only __shared__ object)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wr = wave >> 1, wcn = wave & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int tid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (bid >> 3);
  const int tiles_n = N / PP_BM;
  const int m0 = (tid / tiles_n) * PP_BM, n0 = (tid % tiles_n) * PP_BM;
  const int kb = blockIdx.z * kchunk;
  const int nkh = kchunk / P8_KH;
  const int fr = lane & 15, fq = lane >> 4;
  // this wave's 8 pieces per K-half: A pieces 4w..4w+3 (p 0-3), B pieces 4w..4w+3 (p 4-7)
  int soff[8], doff[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int piece = wave * 4 + (p & 3);
    const int r = piece * 16 + (lane >> 2);
    const int c = (lane & 3) ^ ((r >> 2) & 3);
    soff[p] = p < 4 ? (m0 + r) * lda + c * 8 : (n0 + r) * ldb + c * 8;
    doff[p] = (p < 4 ? 0 : P8_OP) + piece * 1024;
  }
  auto stage = [&](int h, int p) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)((p < 4 ? A : Bm) + soff[p] + kb + h * P8_KH),
        (__attribute__((address_space(3))) void*)(smem + (h & 3) * P8_BUF + doff[p]), 16, 0, 0);
  };
  const int cs = (fq ^ ((fr >> 2) & 3)) << 4;
  const int la = (wr * 128 + fr) * 64 + cs;
  const int lb = P8_OP + (wcn * 128 + fr) * 64 + cs;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-halves 0, 1, 2 in flight; 0 retired and its fragments read
#pragma unroll
  for (int h = 0; h < 3; ++h)
#pragma unroll
    for (int p = 0; p < 8; ++p) stage(h, p);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 fa[8], fb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fb[i] = *reinterpret_cast<const bf16x8*>(smem + lb + i * 1024);
    fa[i] = *reinterpret_cast<const bf16x8*>(smem + la + i * 1024);
  }
  // (K-half 1 retired before the first K-half reads it)
  asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // one register set, snake order: even K-halves run rows outer (fa[i] is free after row i and is
  // reloaded at once; fb[j] after MFMA (7, j)), odd K-halves columns outer (the mirror) -- the
  // next K-half's first MFMAs find their fragments read 7+ MFMAs earlier.  Staging past the last
  // K-half re-stages the last one into the idle buffer (no branch; drained after the loop).
  // fragment register freed by MFMA n of a K-half (snake order P), reloaded from the next K-half
  auto reload = [&](int n, auto Pc, const char* nb) {
    constexpr int P = decltype(Pc)::value;
    const int o = n >> 3, q = n & 7;
    const int i = P == 0 ? o : q, j = P == 0 ? q : o;
    if (P == 0) {
      if (q == 7) fa[i] = *reinterpret_cast<const bf16x8*>(nb + la + i * 1024);
      if (o == 7) fb[j] = *reinterpret_cast<const bf16x8*>(nb + lb + j * 1024);
    } else {
      if (q == 7) fb[j] = *reinterpret_cast<const bf16x8*>(nb + lb + j * 1024);
      if (o == 7) fa[i] = *reinterpret_cast<const bf16x8*>(nb + la + i * 1024);
    }
  };
  auto khalf = [&](int h, auto Pc) {
    constexpr int P = decltype(Pc)::value;     // 0: rows outer, 1: columns outer
    const int hs = h + 3 < nkh ? h + 3 : nkh - 1;
    const char* nb = smem + ((h + 1) & 3) * P8_BUF;
#pragma unroll
    for (int n = 0; n < 64; ++n) {
      const int o = n >> 3, q = n & 7;          // outer / inner index
      const int i = P == 0 ? o : q, j = P == 0 ? q : o;
      // (inline asm pins the accumulator in the AGPR file: with the builtin the register allocator
      // kept part of acc in VGPRs and copied it into AGPRs around every MFMA -- 500 v_accvgpr
      // moves + nops per K-tile; independent accumulators, so no MFMA hazard for the asm to hide)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[j]));
      __builtin_amdgcn_sched_barrier(0);
#ifndef HFM_R8_NODMA
      if (n >= 4 && n < 12) stage(hs, n - 4);
#endif
#ifndef HFM_R8_NOLDS
      // the fragment freed by the PREVIOUS MFMA (one MFMA between an MFMA and the overwrite of a
      // register it reads); freed: rows outer -> fa[i] at the row's end, fb[j] in the last row
      if (n > 0) reload(n - 1, Pc, nb);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
#ifndef HFM_R8_NOLDS
    reload(63, Pc, nb);
#endif
    __builtin_amdgcn_sched_barrier(0);
#ifndef HFM_R8_NOBAR
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // K-half h + 2 retired (h + 3 in flight)
    __builtin_amdgcn_s_barrier();
#endif
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int h = 0; h < nkh; h += 2) {
    khalf(h, I0{});
    khalf(h + 1, I1{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // (no DMA may land after the workgroup ends)
  // the last MFMAs' results are read by the epilogue's compiler code: the asm MFMAs are not padded
  // by hipcc (an 8-pass XDL result needs 12 wait states before another reader)
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");

  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  const int cr = fq * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      epi_store<EPI>(ep, acc[i][j], m0 + wr * 128 + i * 16 + cr, n0 + wcn * 128 + j * 16 + fr, M, N, salt);
}

template <int EPI>
static int launch_gemm_r8(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                          int splitk, const EpiArgs& ep, hipStream_t st) {
  // (an even number of K-halves per split, at least 4)
  if (M % PP_BM || N % PP_BM || splitk < 1 || Kd % (2 * P8_KH * splitk) || Kd / splitk < 4 * P8_KH || lda % 8 ||
      ldb % 8 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  dim3 grid((M / PP_BM) * (N / PP_BM), 1, splitk);
  hipLaunchKernelGGL((gemm_r8_kernel<EPI>), grid, dim3(RB_THREADS), 0, st, A, lda, B, ldb, M, N,
                     Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

template <int EPI>
static int launch_gemm_rb(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                          int splitk, const EpiArgs& ep, hipStream_t st) {
  if (M % PP_BM || N % PP_BM || splitk < 1 || Kd % (PP_BK * splitk) || lda % 8 || ldb % 8 ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  dim3 grid((M / PP_BM) * (N / PP_BM), 1, splitk);
  hipLaunchKernelGGL((gemm_rb_kernel<EPI>), grid, dim3(RB_THREADS), 0, st, A, lda, B, ldb, M, N,
                     Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

template <int EPI, int SPREAD>
static int launch_gemm_pp(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                          int splitk, const EpiArgs& ep, hipStream_t st) {
  if (M % PP_BM || N % PP_BM || splitk < 1 || Kd % (PP_BK * splitk) || lda % 8 || ldb % 8 ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  dim3 grid((M / PP_BM) * (N / PP_BM), 1, splitk);
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, SPREAD>), grid, dim3(PP_THREADS), 0, st, A, lda, B, ldb, M, N,
                     Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

template <int EPI>
static int launch_gemm_lds(const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                           int splitk, const EpiArgs& ep, hipStream_t st) {
  if (M % GL_BM || N % GL_BN || splitk < 1 || Kd % (GL_BK * splitk) || lda % 8 || ldb % 8 ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return (int)hipErrorInvalidValue;
  dim3 grid((M / GL_BM) * (N / GL_BN), 1, splitk);
  hipLaunchKernelGGL((gemm_lds_kernel<EPI>), grid, dim3(GL_THREADS), 0, st, A, lda, B, ldb, M, N,
                     Kd / splitk, ep);
  HFM_LAUNCH_CHECK();
}

// tile: 0 = 64x64 (2x2 waves), 1 = 128x32 (4x1), 2 = 32x128 (1x4), 3 = 32x32 (1x1), 4 = 32x64 (1x2),
//       5 = 32x160 (1x5), 6 = 32x320 (1x10), 7 = 32x256 (1x8), 8 = 128x128 LDS-staged (wide layers),
//       9 = 256x256 ping-pong (wide layers, 8 waves), 10 = same, staging spread, 11 = 256x256
//       register-blocked (4 waves), 12 = 256x256 K-half ring (8 waves, counted DMA waits),
//       13 = 256x256 register-blocked on the K-half ring (4 waves)
template <int EPI>
static int gemm_tile(int tile, const bf16* A, int lda, const bf16* B, int ldb, int M, int N, int Kd,
                     int splitk, const EpiArgs& ep, hipStream_t st) {
  switch (tile) {
    case 0: return launch_gemm<2, 2, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 1: return launch_gemm<4, 1, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 2: return launch_gemm<1, 4, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 3: return launch_gemm<1, 1, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 4: return launch_gemm<1, 2, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 5: return launch_gemm<1, 5, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 6: return launch_gemm<1, 10, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 7: return launch_gemm<1, 8, EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 8: return launch_gemm_lds<EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 9: return launch_gemm_pp<EPI, 0>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 10: return launch_gemm_pp<EPI, 1>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 11: return launch_gemm_rb<EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 12: return launch_gemm_p8<EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    case 13: return launch_gemm_r8<EPI>(A, lda, B, ldb, M, N, Kd, splitk, ep, st);
    default: return (int)hipErrorInvalidValue;
  }
}

HFM_API int hfm_gemm_nt(int epi, int tile, const void* A, int lda, const void* B, int ldb, int M,
                        int N, int Kd, int splitk, const EpiArgs* ep, hipStream_t st) {
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)B;
  switch (epi) {
    case EPI_F32: return gemm_tile<EPI_F32>(tile, a, lda, b, ldb, M, N, Kd, splitk, *ep, st);
    case EPI_FWD: return gemm_tile<EPI_FWD>(tile, a, lda, b, ldb, M, N, Kd, 1, *ep, st);
    case EPI_DGRAD: return gemm_tile<EPI_DGRAD>(tile, a, lda, b, ldb, M, N, Kd, 1, *ep, st);
    case EPI_FWD_EVAL: return gemm_tile<EPI_FWD_EVAL>(tile, a, lda, b, ldb, M, N, Kd, 1, *ep, st);
    case EPI_RELU_F32: return gemm_tile<EPI_RELU_F32>(tile, a, lda, b, ldb, M, N, Kd, 1, *ep, st);
    default: return (int)hipErrorInvalidValue;
  }
}

HFM_API int hfm_epi_args_bytes() { return (int)sizeof(EpiArgs); }

// ------------------------------------------------------------------ stand-alone epilogue pass
// The forward / dgrad epilogue over an fp32 product C [M, N] that a library GEMM (hipBLASLt via
// torch.mm, bf16 operands, fp32 out) wrote: the same per-element values as epi_store /
// epi_tile_lds (bias, relu, counter-hash dropout; dgrad scale, bf16 rounding, hprev>0 mask), the
// row-major bf16 output in 16-byte stores, the transposed copy through a padded LDS tile.  One
// 256-thread workgroup per 64 x 64 tile; M, N multiples of 64 (checked by the host entry).
template <int EPI>
__global__ void __launch_bounds__(256) epi_pass_kernel(const float* __restrict__ C, int M, int N, EpiArgs ep) {
  __shared__ bf16 t[64][64 + 8];
  const int tid = threadIdx.x;
  const int row0 = blockIdx.y * 64, col0 = blockIdx.x * 64;
  uint32_t salt = 0;
  if (EPI == EPI_FWD && ep.drop) salt = dropout_salt(ep.seed, (uint32_t)(*ep.step), ep.layer);
  const bool mask = EPI == EPI_DGRAD && ep.hprev != nullptr;
  bf16* out = reinterpret_cast<bf16*>(ep.out);
  // the thread's 8 bias values (the same columns in both row pieces) in two 16-byte loads
  f32x4 bv[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  if (EPI == EPI_FWD || EPI == EPI_FWD_EVAL) {
    bv[0] = *reinterpret_cast<const f32x4*>(ep.bias + col0 + (tid & 7) * 8);
    bv[1] = *reinterpret_cast<const f32x4*>(ep.bias + col0 + (tid & 7) * 8 + 4);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = (tid >> 3) + 32 * p, c = (tid & 7) * 8;
    const int row = row0 + r, col = col0 + c;
    const size_t g = (size_t)row * N + col;
    const float4 a0 = *reinterpret_cast<const float4*>(C + g);
    const float4 a1 = *reinterpret_cast<const float4*>(C + g + 4);
    const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    bf16x8 h;
    if (mask) h = *reinterpret_cast<const bf16x8*>(ep.hprev + g);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = a[k];
      if (EPI == EPI_FWD || EPI == EPI_FWD_EVAL) {
        v = fmaxf(v + bv[k >> 2][k & 3], 0.f);
        if (EPI == EPI_FWD && ep.drop)
          v = dropout_keep((uint32_t)(row * N + col + k), salt, ep.keep_thr) ? v * ep.scale : 0.f;
      } else {
        v = v * ep.scale;
        if (mask && !((float)h[k] > 0.f)) v = 0.f;
      }
      o[k] = f2bf(v);
    }
    *reinterpret_cast<bf16x8*>(out + g) = o;
    *reinterpret_cast<bf16x8*>(&t[r][c]) = o;
  }
  if (!ep.out_t) return;
  __syncthreads();
  // transposed: thread -> column cc of the tile, 16 consecutive rows (32 contiguous bytes of out_t)
  const int cc = tid >> 2, rr = (tid & 3) * 16;
  bf16x8 o0, o1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    o0[k] = t[rr + k][cc];
    o1[k] = t[rr + 8 + k][cc];
  }
  bf16* dt = ep.out_t + (size_t)(col0 + cc) * M + row0 + rr;
  *reinterpret_cast<bf16x8*>(dt) = o0;
  *reinterpret_cast<bf16x8*>(dt + 8) = o1;
}

HFM_API int hfm_epi_pass(int epi, const float* C, int M, int N, const EpiArgs* ep, hipStream_t st) {
  if (M <= 0 || N <= 0 || (M & 63) || (N & 63) || !ep->out) return (int)hipErrorInvalidValue;
  const dim3 grid(N / 64, M / 64);
  switch (epi) {
    case EPI_FWD: epi_pass_kernel<EPI_FWD><<<grid, 256, 0, st>>>(C, M, N, *ep); break;
    case EPI_FWD_EVAL: epi_pass_kernel<EPI_FWD_EVAL><<<grid, 256, 0, st>>>(C, M, N, *ep); break;
    case EPI_DGRAD: epi_pass_kernel<EPI_DGRAD><<<grid, 256, 0, st>>>(C, M, N, *ep); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ K7 head
// Per sample: y_d = h_L . w_out + b_out;  y = y_fm + y_d;  p = sigmoid(y);
//   loss_b = BCE(y, label) (or (p-label)^2);  dlogit = dL/dy * gscale  (gscale = 1/global batch)
//   dZ_L = dlogit * w_out (.) (h_L > 0) / keep_L     (bf16, + transpose)
// Block partials (deterministic LDS tree): [ sum dlogit*h_L (L) | sum dlogit | sum loss ].
struct HeadArgs {
  const bf16* h;        // [M, L] last hidden activation (post dropout)
  const float* w_out;   // [L] (inside the flat param buffer)
  const float* b_out;   // [1]
  const float* y_fm;    // [M]
  const float* labels;  // [M] (nullable in predict mode)
  int M, L, nvalid;     // nvalid: rows < nvalid contribute to loss/grad (padding rows excluded)
  int square_loss;
  int train;            // 0: predict/eval (probabilities + loss only)
  float gscale;         // 1 / global batch
  float scale_l;        // 1/keep of the last hidden layer's dropout
  float* prob;          // [M]
  float* logit;         // [M] (nullable)
  float* dlogit;        // [M]
  bf16* dz;             // [M, L]
  bf16* dz_t;           // [L, M]
  float* partial;       // [gridDim.x, L + 2]
  float* dh;            // batch-norm towers: raw dL/dh_L = dlogit * w_out, f32 [M, L] (the BN
                        // backward applies dropout/ReLU itself); dz/dz_t are then unused
};

// 4 lanes per sample (each owns L/4 hidden columns): 64 samples per 256-thread workgroup, so a
// 16K batch is 256 workgroups (one per CU) instead of 64.
template <int L>
__global__ void __launch_bounds__(256) head_kernel(HeadArgs a) {
  constexpr int Q = L / 4;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x * 64 + (tid >> 2), q = tid & 3;
  float hv[Q];
  float dl = 0.f, lossb = 0.f;
  const bool inb = b < a.M;
  const bool valid = b < a.nvalid;
  float yd = 0.f;
  if (inb) {
    const bf16* hr = a.h + (size_t)b * L + q * Q;
#pragma unroll
    for (int j = 0; j < Q; j += 8) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(hr + j);
#pragma unroll
      for (int t = 0; t < 8; ++t) hv[j + t] = bf2f(v[t]);
    }
#pragma unroll
    for (int j = 0; j < Q; ++j) yd += hv[j] * a.w_out[q * Q + j];
  } else {
#pragma unroll
    for (int j = 0; j < Q; ++j) hv[j] = 0.f;
  }
  yd += __shfl_xor(yd, 1, 64);
  yd += __shfl_xor(yd, 2, 64);
  if (inb) {
    const float y = a.y_fm[b] + yd + a.b_out[0];
    const float p = 1.f / (1.f + __expf(-y));
    if (q == 0) {
      a.prob[b] = p;
      if (a.logit) a.logit[b] = y;
    }
    if (a.labels && valid) {
      const float lab = a.labels[b];
      if (a.square_loss) {
        lossb = (p - lab) * (p - lab);
        dl = 2.f * (p - lab) * p * (1.f - p) * a.gscale;
      } else {
        lossb = fmaxf(y, 0.f) - y * lab + log1pf(__expf(-fabsf(y)));
        dl = (p - lab) * a.gscale;
      }
    }
    if (a.train && a.dh) {
      if (q == 0) a.dlogit[b] = dl;
      float* dhr = a.dh + (size_t)b * L + q * Q;
#pragma unroll
      for (int j = 0; j < Q; ++j) dhr[j] = dl * a.w_out[q * Q + j];
    } else if (a.train) {
      if (q == 0) a.dlogit[b] = dl;
      bf16* dzr = a.dz + (size_t)b * L + q * Q;
#pragma unroll
      for (int j = 0; j < Q; j += 8) {
        bf16x8 pk;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int col = q * Q + j + t;
          const float g = hv[j + t] > 0.f ? dl * a.w_out[col] * a.scale_l : 0.f;
          pk[t] = f2bf(g);
          a.dz_t[(size_t)col * a.M + b] = pk[t];
        }
        *reinterpret_cast<bf16x8*>(dzr + j) = pk;
      }
    }
  }
  // block partials [sum dl*h (L) | sum dl | sum loss]: butterflies over the 16 lanes of a wave
  // that share q, then the 4 waves in order through LDS (deterministic).
  __shared__ float wsum[4][L + 2];
#pragma unroll
  for (int j = 0; j < Q; ++j) {
    float v = a.train ? dl * hv[j] : 0.f;
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 4) wsum[wv][lane * Q + j] = v;   // lane == q here
  }
  float v0 = (q == 0) ? dl : 0.f, v1 = (q == 0) ? lossb : 0.f;
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) {
    v0 += __shfl_xor(v0, o, 64);
    v1 += __shfl_xor(v1, o, 64);
  }
  if (lane == 0) {
    wsum[wv][L] = v0;
    wsum[wv][L + 1] = v1;
  }
  __syncthreads();
  float* part = a.partial + (size_t)blockIdx.x * (L + 2);
  for (int c = tid; c < L + 2; c += blockDim.x)
    part[c] = ((wsum[0][c] + wsum[1][c]) + wsum[2][c]) + wsum[3][c];
}

// Wide last layers (L > 256, multiple of 64: the reference's 4096-wide GPU tower, DOC p.37), 64
// samples per 256-thread workgroup like head_kernel (same partial rows and finalize jobs):
//   pass 1: each wave takes 16 samples: y_d by a lane-strided dot + butterfly, then p / loss /
//           dlogit; the 64 dlogits go to LDS;
//   pass 2: each lane owns columns (wave w: c = 64 w + lane + 256 k) and walks the 64 samples:
//           dZ row-major stores (coalesced across lanes), the transposed copy as 16-B stores of 8
//           consecutive samples, and the column's partial sum dl * h in sample order.
__global__ void __launch_bounds__(256) head_wide_kernel(HeadArgs a) {
  __shared__ float hw_dl[64], hw_loss[64];
  const int L = a.L;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int bb = blockIdx.x * 64;
  for (int s = 0; s < 16; ++s) {
    const int b = bb + wv * 16 + s;
    float yd = 0.f;
    if (b < a.M) {
      const bf16* hr = a.h + (size_t)b * L;
      for (int c = lane; c < L; c += 64) yd += bf2f(hr[c]) * a.w_out[c];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) yd += __shfl_xor(yd, o, 64);
    float dl = 0.f, lossb = 0.f;
    if (b < a.M) {
      const float y = a.y_fm[b] + yd + a.b_out[0];
      const float p = 1.f / (1.f + __expf(-y));
      if (lane == 0) {
        a.prob[b] = p;
        if (a.logit) a.logit[b] = y;
      }
      if (a.labels && b < a.nvalid) {
        const float lab = a.labels[b];
        if (a.square_loss) {
          lossb = (p - lab) * (p - lab);
          dl = 2.f * (p - lab) * p * (1.f - p) * a.gscale;
        } else {
          lossb = fmaxf(y, 0.f) - y * lab + log1pf(__expf(-fabsf(y)));
          dl = (p - lab) * a.gscale;
        }
      }
      if (a.train && lane == 0) a.dlogit[b] = dl;
    }
    if (lane == 0) {
      hw_dl[wv * 16 + s] = dl;
      hw_loss[wv * 16 + s] = lossb;
    }
  }
  __syncthreads();
  float* part = a.partial + (size_t)blockIdx.x * (L + 2);
  const bool full = bb + 64 <= a.M && (a.M % 8) == 0;
  for (int c = wv * 64 + lane; c < L; c += 256) {
    const float w = a.w_out[c];
    float cs = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      bf16x8 col;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s = g * 8 + j, b = bb + s;
        const float dl = hw_dl[s];
        const float h = b < a.M ? bf2f(a.h[(size_t)b * L + c]) : 0.f;
        cs += dl * h;
        float v = 0.f;
        if (a.train && b < a.M) {
          if (a.dh) a.dh[(size_t)b * L + c] = dl * w;
          else {
            v = h > 0.f ? dl * w * a.scale_l : 0.f;
            a.dz[(size_t)b * L + c] = f2bf(v);
          }
        }
        col[j] = f2bf(v);
      }
      if (a.train && !a.dh) {
        if (full) {
          *reinterpret_cast<bf16x8*>(a.dz_t + (size_t)c * a.M + bb + g * 8) = col;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (bb + g * 8 + j < a.M) a.dz_t[(size_t)c * a.M + bb + g * 8 + j] = col[j];
        }
      }
    }
    part[c] = a.train ? cs : 0.f;
  }
  if (threadIdx.x == 0) {
    float d = 0.f, l = 0.f;
    for (int s = 0; s < 64; ++s) {
      d += hw_dl[s];
      l += hw_loss[s];
    }
    part[L] = d;
    part[L + 1] = l;
  }
}

// Wide head (L % 256 == 0, L > 256) in two launches with 16-byte accesses throughout; the
// one-launch head_wide_kernel read H one bf16 per lane per row in a 256-workgroup grid and took
// ~0.9 ms of a 6.5 ms step at L = 4096 (profiles/r6tw_kernels.md).
// dot: 16 waves per 64-row block, 4 rows each with all their chunks in flight: y, p, loss, dlogit, and
//      the block's dlogit / loss sums (partial columns L, L + 1, rows in order).
// bwd: workgroup = 64 rows x 256 columns; thread = 8 rows x 8 columns (rows 8 rg.., chunk cc):
//      dz / dh rows as 16-byte chunks, dz_t as 8-row 16-byte column chunks, and the block's
//      column sums of dlogit * h (rows in order per thread, the 8 row groups in order).
__global__ void __launch_bounds__(1024) head_wide_dot_kernel(HeadArgs a) {
  __shared__ float hw_dl[64], hw_loss[64];
  const int L = a.L;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int bb = blockIdx.x * 64;
  const int nch = L / 8;                      // 16-byte chunks per row
  {                                     // 16 waves x 4 rows: every row's chunks in flight at once
    const int s0 = 0;
    float yd[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ch = lane; ch < nch; ch += 64) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(a.w_out + ch * 8);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(a.w_out + ch * 8 + 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int b = bb + wv * 4 + s0 + u;
        if (b < a.M) {
          const bf16x8 h = *reinterpret_cast<const bf16x8*>(a.h + (size_t)b * L + ch * 8);
          float d = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) d += bf2f(h[k]) * w0[k];
#pragma unroll
          for (int k = 0; k < 4; ++k) d += bf2f(h[4 + k]) * w1[k];
          yd[u] += d;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) yd[u] += __shfl_xor(yd[u], o, 64);
      const int s = s0 + u, b = bb + wv * 4 + s;
      float dl = 0.f, lossb = 0.f;
      if (b < a.M) {
        const float y = a.y_fm[b] + yd[u] + a.b_out[0];
        const float p = 1.f / (1.f + __expf(-y));
        if (lane == 0) {
          a.prob[b] = p;
          if (a.logit) a.logit[b] = y;
        }
        if (a.labels && b < a.nvalid) {
          const float lab = a.labels[b];
          if (a.square_loss) {
            lossb = (p - lab) * (p - lab);
            dl = 2.f * (p - lab) * p * (1.f - p) * a.gscale;
          } else {
            lossb = fmaxf(y, 0.f) - y * lab + log1pf(__expf(-fabsf(y)));
            dl = (p - lab) * a.gscale;
          }
        }
        if (a.train && lane == 0) a.dlogit[b] = dl;
      }
      if (lane == 0) {
        hw_dl[wv * 4 + s] = dl;
        hw_loss[wv * 4 + s] = lossb;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float d = 0.f, l = 0.f;
    for (int s = 0; s < 64; ++s) {
      d += hw_dl[s];
      l += hw_loss[s];
    }
    float* part = a.partial + (size_t)blockIdx.x * (L + 2);
    part[L] = d;
    part[L + 1] = l;
  }
}

__global__ void __launch_bounds__(256) head_wide_bwd_kernel(HeadArgs a) {
  __shared__ float red[8][257];
  const int L = a.L, tid = threadIdx.x;
  const int cc = tid & 31, rg = tid >> 5;
  const int bb = blockIdx.x * 64, c0 = blockIdx.y * 256 + cc * 8;
  float* part = a.partial + (size_t)blockIdx.x * (L + 2) + blockIdx.y * 256;
  if (!a.train) {                       // (predict / eval: no gradients, zero partial columns)
    part[tid] = 0.f;
    return;
  }
  float w[8];
  {
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(a.w_out + c0);
    const f32x4 w1 = *reinterpret_cast<const f32x4*>(a.w_out + c0 + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] = w0[k];
      w[4 + k] = w1[k];
    }
  }
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  bf16 zt[8][8];                        // [column][row] for the dz_t chunks
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int b = bb + rg * 8 + r;
    const bool in = b < a.M;
    const float dl = in ? a.dlogit[b] : 0.f;
    bf16x8 h;
    if (in) h = *reinterpret_cast<const bf16x8*>(a.h + (size_t)b * L + c0);
    bf16x8 z;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float hv = in ? bf2f(h[k]) : 0.f;
      cs[k] += dl * hv;
      const float v = hv > 0.f ? dl * w[k] * a.scale_l : 0.f;
      z[k] = f2bf(v);
      zt[k][r] = z[k];
    }
    if (in) {
      if (a.dh) {
        float* dh = a.dh + (size_t)b * L + c0;
        *reinterpret_cast<f32x4*>(dh) = f32x4{dl * w[0], dl * w[1], dl * w[2], dl * w[3]};
        *reinterpret_cast<f32x4*>(dh + 4) = f32x4{dl * w[4], dl * w[5], dl * w[6], dl * w[7]};
      } else {
        *reinterpret_cast<bf16x8*>(a.dz + (size_t)b * L + c0) = z;
      }
    }
  }
  if (!a.dh) {
    const int r0 = bb + rg * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bf16x8 col;
#pragma unroll
      for (int r = 0; r < 8; ++r) col[r] = zt[k][r];
      if ((a.M & 7) == 0 && r0 + 8 <= a.M) {
        *reinterpret_cast<bf16x8*>(a.dz_t + (size_t)(c0 + k) * a.M + r0) = col;
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (r0 + r < a.M) a.dz_t[(size_t)(c0 + k) * a.M + r0 + r] = col[r];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rg][cc * 8 + k] = cs[k];
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int g = 0; g < 8; ++g) t += red[g][tid];
  part[tid] = t;
}

HFM_API int hfm_head(const HeadArgs* a, hipStream_t st) {
  const int grid = (a->M + 63) / 64;
  if (a->L > 256) {
    if (a->L % 256 == 0) {
      hipLaunchKernelGGL(head_wide_dot_kernel, dim3(grid), dim3(1024), 0, st, *a);
      hipLaunchKernelGGL(head_wide_bwd_kernel, dim3(grid, a->L / 256), dim3(256), 0, st, *a);
      HFM_LAUNCH_CHECK();
    }
    if (a->L % 64) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(head_wide_kernel, dim3(grid), dim3(256), 0, st, *a);
    HFM_LAUNCH_CHECK();
  }
  switch (a->L) {
#define HL(LL) case LL: hipLaunchKernelGGL(head_kernel<LL>, dim3(grid), dim3(256), 0, st, *a); break;
    HL(32) HL(64) HL(96) HL(128) HL(160) HL(192) HL(224) HL(256)
#undef HL
    default: return (int)hipErrorInvalidValue;
  }
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_head_args_bytes() { return (int)sizeof(HeadArgs); }

// ------------------------------------------------------------------ gradient finalize
// Sums split-K wgrad slabs and head partials into the flat dense-gradient buffer (one job
// table, one launch), and computes bias gradients as row sums of the transposed dZ^T.
struct SlabJob {
  float* dst;
  const float* src;
  long n;          // elements
  int nslab;
  long stride;     // elements between slabs
  long src_ld;     // source row stride (elements; == n if contiguous)
  int cols;        // dst/src columns per row (to map linear index -> src offset with src_ld)
  float scale;
  int lanes;       // finalize_kernel: slab-lanes per output (2 or 8); 256/lanes outputs per block
  int chunk0;      // finalize_kernel: first block of this job
};

// blockIdx.y = job.  A workgroup owns 32 consecutive output elements; its 8 slab-lanes per
// element each sum a strided subset of the slabs, then the 8 partials are added in a fixed
// order through LDS (deterministic).  Parallel over both outputs and slabs, so a job with 41K
// outputs x 32 slabs (layer-1 wgrad) and one with 32 outputs x 256 slabs (head partials) are
// both short.
__global__ void __launch_bounds__(256) slab_reduce_kernel(const SlabJob* __restrict__ jobs, int njobs) {
  __shared__ float red[8][33];
  const SlabJob& jr = jobs[blockIdx.y];
  const int n = (int)jr.n, nslab = jr.nslab, stride = (int)jr.stride, cols = jr.cols, ld = (int)jr.src_ld;
  const float* src = jr.src;
  const int e = threadIdx.x & 31, zl = threadIdx.x >> 5;
  for (int i0 = blockIdx.x * 32; i0 < n; i0 += gridDim.x * 32) {
    const int i = i0 + e;
    float s = 0.f;
    if (i < n) {
      const int r = i / cols, c = i - r * cols;
      const float* sp = src + r * ld + c;
      for (int z = zl; z < nslab; z += 8) s += sp[z * stride];
    }
    red[zl][e] = s;
    __syncthreads();
    if (zl == 0 && i < n) {
      float t = ((red[0][e] + red[1][e]) + (red[2][e] + red[3][e])) +
                ((red[4][e] + red[5][e]) + (red[6][e] + red[7][e]));
      jr.dst[i] = t * jr.scale;
    }
    __syncthreads();
  }
}

// One launch for the whole gradient finalize: blocks [0, nslab_blocks) reduce split-K slabs and
// head partials (job j owns blocks [chunk0_j, chunk0_j + ceil(n_j / (256 / lanes_j)))), the
// remaining blocks compute bias gradients as row sums of dZ^T (one block per row).  Every
// reduction has a fixed order (deterministic).
struct RowSumJob;
template <int OPT = -1>
__device__ void rowsum_block(const RowSumJob* jobs, int njobs, int b, const FinOpt* o = nullptr,
                             float lr_t = 0.f);

// OPT >= 0 (single GPU, dense optimizer fused): the thread that writes an element's final
// gradient also applies the optimizer to it (fin_opt_apply), and the last block to finish
// advances the step counter -- the separate dense_opt launch and its kernel boundary go away.
template <int OPT>
__device__ __forceinline__ void finalize_block(const SlabJob* __restrict__ sj, int nsj,
                                               int nslab_blocks, const RowSumJob* rj, int nrj,
                                               const FinOpt& o, float lr_t) {
  const int b = blockIdx.x;
  if (b >= nslab_blocks) {
    rowsum_block<OPT>(rj, nrj, b - nslab_blocks, &o, lr_t);
    return;
  }
  int j = 0;
  while (j + 1 < nsj && b >= sj[j + 1].chunk0) ++j;
  const SlabJob& jr = sj[j];
  const int lanes = jr.lanes, per = 256 / lanes;
  const int e = threadIdx.x % per, zl = threadIdx.x / per;
  const int i = (b - jr.chunk0) * per + e;
  const int n = (int)jr.n, nslab = jr.nslab, stride = (int)jr.stride;
  float s = 0.f;
  if (i < n) {
    const int r = i / jr.cols, c = i - r * jr.cols;
    const float* sp = jr.src + (size_t)r * jr.src_ld + c;
#pragma unroll 8
    for (int z = zl; z < nslab; z += lanes) s += sp[(size_t)z * stride];
  }
  if (lanes == 1) {
    if (i < n) {
      jr.dst[i] = s * jr.scale;
      if (OPT >= 0) fin_opt_apply<OPT>(o, lr_t, jr.dst + i, s * jr.scale);
    }
    return;
  }
  // lanes > 1: per in {32, 128}; combine the lanes in order through LDS
  __shared__ float red2[256];
  red2[threadIdx.x] = s;
  __syncthreads();
  if (zl == 0 && i < n) {
    float t = 0.f;
    for (int l = 0; l < lanes; ++l) t += red2[l * per + e];
    jr.dst[i] = t * jr.scale;
    if (OPT >= 0) fin_opt_apply<OPT>(o, lr_t, jr.dst + i, t * jr.scale);
  }
}

__global__ void __launch_bounds__(256) finalize_kernel(const SlabJob* __restrict__ sj, int nsj,
                                                       int nslab_blocks, const RowSumJob* rj,
                                                       int nrj) {
  finalize_block<-1>(sj, nsj, nslab_blocks, rj, nrj, FinOpt{}, 0.f);
}

template <int OPT>
__global__ void __launch_bounds__(256) finalize_opt_kernel(const SlabJob* __restrict__ sj, int nsj,
                                                           int nslab_blocks, const RowSumJob* rj,
                                                           int nrj, FinOpt o) {
  const float lr_t = OPT == OPT_ADAM ? adam_lr_t(o.h, *o.step + 1) : o.h.lr;
  finalize_block<OPT>(sj, nsj, nslab_blocks, rj, nrj, o, lr_t);
  __syncthreads();
  if (threadIdx.x == 0) {  // every block has read *step (lr_t) before it arrives here
    const unsigned prev = atomicAdd(o.done_ctr, 1u);
    if (prev == gridDim.x - 1) {
      *o.step += 1;
      *o.done_ctr = 0u;
    }
  }
}

HFM_API int hfm_finalize(const void* slab_jobs, int nsj, int nslab_blocks, const void* row_jobs,
                         int nrj, int total_rows, hipStream_t st) {
  const int grid = nslab_blocks + total_rows;
  if (grid <= 0) return 0;
  hipLaunchKernelGGL(finalize_kernel, dim3(grid), dim3(256), 0, st, (const SlabJob*)slab_jobs, nsj,
                     nslab_blocks, (const RowSumJob*)row_jobs, nrj);
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_finalize_opt(int opt, const void* slab_jobs, int nsj, int nslab_blocks,
                             const void* row_jobs, int nrj, int total_rows, float* p, float* g,
                             float* s0, float* s1, long n, const OptHyper* h, int64_t* step,
                             const void* segs, int nseg, unsigned* done_ctr, hipStream_t st) {
  const int grid = nslab_blocks + total_rows;
  if (grid <= 0 || !done_ctr) return (int)hipErrorInvalidValue;
  const FinOpt o{p, g, s0, s1, n, *h, step, (const ShadowSeg*)segs, nseg, done_ctr};
  switch (opt) {
#define CASE(O)                                                                                 \
  case O:                                                                                       \
    hipLaunchKernelGGL(finalize_opt_kernel<O>, dim3(grid), dim3(256), 0, st,                    \
                       (const SlabJob*)slab_jobs, nsj, nslab_blocks, (const RowSumJob*)row_jobs, \
                       nrj, o);                                                                 \
    break;
    CASE(OPT_ADAM) CASE(OPT_ADAGRAD) CASE(OPT_MOMENTUM) CASE(OPT_FTRL) CASE(OPT_GD)
#undef CASE
    default: return (int)hipErrorInvalidValue;
  }
  HFM_LAUNCH_CHECK();
}

HFM_API int hfm_slab_reduce(const void* jobs, int njobs, int max_n, hipStream_t st) {
  int gx = (max_n + 31) / 32;
  if (gx > 2048) gx = 2048;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(gx, njobs), dim3(256), 0, st, (const SlabJob*)jobs, njobs);
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_slab_job_bytes() { return (int)sizeof(SlabJob); }

struct RowSumJob {
  float* dst;       // [rows]
  const bf16* src;  // [rows, ld]
  int rows, n;      // sum the first n entries of each row
  long ld;
};

template <int OPT>
__device__ void rowsum_block(const RowSumJob* jobs, int njobs, int b, const FinOpt* o, float lr_t) {
  __shared__ float red[256];
  // b enumerates (job, row) pairs
  int rem = b, ji = 0;
  while (ji < njobs && rem >= jobs[ji].rows) { rem -= jobs[ji].rows; ++ji; }
  if (ji >= njobs) return;
  const RowSumJob j = jobs[ji];
  const bf16* s = j.src + (size_t)rem * j.ld;
  float acc = 0.f;
#pragma unroll 8
  for (int i = threadIdx.x * 8; i < j.n; i += 256 * 8) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(s + i);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc += bf2f(v[t]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    j.dst[rem] = red[0];
    if (OPT >= 0) fin_opt_apply<OPT>(*o, lr_t, j.dst + rem, red[0]);
  }
}

__global__ void __launch_bounds__(256) rowsum_kernel(const RowSumJob* __restrict__ jobs, int njobs) {
  rowsum_block(jobs, njobs, blockIdx.x);
}

HFM_API int hfm_rowsum(const void* jobs, int njobs, int total_rows, hipStream_t st) {
  if (total_rows <= 0) return 0;
  hipLaunchKernelGGL(rowsum_kernel, dim3(total_rows), dim3(256), 0, st, (const RowSumJob*)jobs, njobs);
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_rowsum_job_bytes() { return (int)sizeof(RowSumJob); }
