// One wave's 32x32 MFMA output tile with K-contiguous A and B operands (shared by the fused
// tower, the grouped weight gradients and the wgfin / sparse+wgfin launches).
#pragma once
#include "common.h"

// One wave: c[2][2] += A[32 x 32*nk] . B[32 x 32*nk]^T, both K-contiguous (row strides lda/ldb
// in elements).  Register ring of PF k-steps so PF fragment sets are in flight.
template <int PF, bool ROWSUM = false>
__device__ __forceinline__ void mma32(const bf16* __restrict__ A, int lda, const bf16* __restrict__ B,
                                      int ldb, int nk, int lane, f32x4& c00, f32x4& c01, f32x4& c10,
                                      f32x4& c11, float* rs = nullptr) {
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const bf16* a0 = A + r * lda + kq;
  const bf16* a1 = a0 + 16 * lda;
  const bf16* b0 = B + r * ldb + kq;
  const bf16* b1 = b0 + 16 * ldb;
  bf16x8 ra0[PF], ra1[PF], rb0[PF], rb1[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    if (j < nk) {
      ra0[j] = *reinterpret_cast<const bf16x8*>(a0 + j * 32);
      ra1[j] = *reinterpret_cast<const bf16x8*>(a1 + j * 32);
      rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + j * 32);
      rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + j * 32);
    }
  }
  for (int kb = 0; kb < nk; kb += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int ks = kb + j;
      if (ks < nk) {
        c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra0[j], rb0[j], c00, 0, 0, 0);
        c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra0[j], rb1[j], c01, 0, 0, 0);
        c10 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra1[j], rb0[j], c10, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra1[j], rb1[j], c11, 0, 0, 0);
        if (ROWSUM) {  // A row sums on the side (bias gradients): lane's 8 elements of rows r, r+16
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            rs[0] += bf2f(ra0[j][t]);
            rs[1] += bf2f(ra1[j][t]);
          }
        }
        const int kn = (ks + PF) * 32;
        if (ks + PF < nk) {
          ra0[j] = *reinterpret_cast<const bf16x8*>(a0 + kn);
          ra1[j] = *reinterpret_cast<const bf16x8*>(a1 + kn);
          rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + kn);
          rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + kn);
        }
      }
    }
  }
}

// ---- primed B fragments (the fused tower's bf16 GEMMs): the B operand of a wave's NEXT 32x32
// tile (weights, L2-resident) is loaded one phase ahead -- while the phase before it (the FM
// gather, the previous layer's epilogue, its barrier and transposed store) runs -- so the tile's
// MFMAs start on registers instead of an L2 round trip per PF k-steps.  NP k-steps are primed;
// a longer reduction streams the rest through the same NP registers (ring).
template <int NP>
__device__ __forceinline__ void bfrag_prime(bf16x8 (&rb0)[NP], bf16x8 (&rb1)[NP], const bf16* __restrict__ B,
                                            int ldb, int nk, int lane) {
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const bf16* b0 = B + r * ldb + kq;
  const bf16* b1 = b0 + 16 * ldb;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    if (j < nk) {
      rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + j * 32);
      rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + j * 32);
    }
  }
}

// c[2][2] += A[32 x 32nk] (LDS, row stride lda) . B[32 x 32nk]^T with B's first NP k-steps in
// (rb0, rb1) from bfrag_prime; k-steps past NP are loaded NP ahead into the freed registers.
template <int NP>
__device__ __forceinline__ void mma32_primed(const bf16* A, int lda, const bf16* __restrict__ B, int ldb,
                                             int nk, int lane, bf16x8 (&rb0)[NP], bf16x8 (&rb1)[NP],
                                             f32x4& c00, f32x4& c01, f32x4& c10, f32x4& c11) {
  const int r = lane & 15, kq = (lane >> 4) * 8;
  const bf16* a0 = A + r * lda + kq;
  const bf16* a1 = a0 + 16 * lda;
  const bf16* b0 = B + r * ldb + kq;
  const bf16* b1 = b0 + 16 * ldb;
  for (int kb = 0; kb < nk; kb += NP) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int ks = kb + j;
      if (ks < nk) {
        const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(a0 + ks * 32);
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(a1 + ks * 32);
        c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, rb0[j], c00, 0, 0, 0);
        c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, rb1[j], c01, 0, 0, 0);
        c10 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, rb0[j], c10, 0, 0, 0);
        c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, rb1[j], c11, 0, 0, 0);
        if (ks + NP < nk) {
          rb0[j] = *reinterpret_cast<const bf16x8*>(b0 + (ks + NP) * 32);
          rb1[j] = *reinterpret_cast<const bf16x8*>(b1 + (ks + NP) * 32);
        }
      }
    }
  }
}
