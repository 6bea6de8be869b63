// tf1_dense split form: the l2-only optimizer update of every table row OUTSIDE the step's batch
// (optim.hip tf1_sweep_kernel on its own graph branch, or sparse_fused.hip sfwg_kernel's sweep
// workgroups).  Rows of the batch carry a byte flag (set from the sorted slot keys before the
// step): the sweep skips them -- the sparse kernel gives them the full update -- and clears it.
#pragma once
#include "common.h"

// record: [ v (K) | w, w_slot0, w_slot1, pad | v_slot0 (K) | v_slot1 (K) | pad ]
template <int K, int OPT>
struct Tf1Rec {
  static constexpr int NS = OPT == OPT_GD ? 0 : ((OPT == OPT_ADAM || OPT == OPT_FTRL) ? 2 : 1);
  static constexpr int USED = K + 4 + NS * K;   // deepfm.py table_record_floats
  static constexpr int FLOATS = USED <= 16 ? (USED + 15) / 16 * 16 : (USED + 31) / 32 * 32;
};

// rows first, first + stride, ... < R; U rows per thread per pass (loads of all U issued first)
template <int K, int OPT, int U>
__device__ __forceinline__ void tf1_sweep_rows(float* __restrict__ rec, int ld, long R,
                                               unsigned char* __restrict__ flags, const OptHyper& h,
                                               float lr_t, long first, long stride) {
  constexpr int NS = Tf1Rec<K, OPT>::NS;
  constexpr int REC = Tf1Rec<K, OPT>::FLOATS;
  constexpr int Q = K / 4;
  for (long base = first; base < R; base += stride * U) {
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long row = base + u * stride;
      act[u] = false;
      if (row < R) {
        if (flags[row]) flags[row] = 0;      // this step's batch row: the sparse kernel's
        else act[u] = true;
      }
    }
    f32x4 p[U][Q], a[U][Q], c[U][Q], wq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!act[u]) continue;
      const float* r = rec + (size_t)(base + u * stride) * ld;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        p[u][q] = *reinterpret_cast<const f32x4*>(r + 4 * q);
        if (NS >= 1) a[u][q] = *reinterpret_cast<const f32x4*>(r + K + 4 + 4 * q);
        if (NS >= 2) c[u][q] = *reinterpret_cast<const f32x4*>(r + 2 * K + 4 + 4 * q);
      }
      wq[u] = *reinterpret_cast<const f32x4*>(r + K);   // {w, w_slot0, w_slot1, pad}
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!act[u]) continue;
      float* r = rec + (size_t)(base + u * stride) * ld;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        f32x4 pp = p[u][q], aa = {0, 0, 0, 0}, cc = {0, 0, 0, 0};
        if (NS >= 1) aa = a[u][q];
        if (NS >= 2) cc = c[u][q];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float gj = l2_grad(0.f, h.l2, pp[j]);
          float pj = pp[j], aj = aa[j], cj = cc[j];
          opt_update<OPT>(pj, gj, aj, cj, h, lr_t);
          pp[j] = pj; aa[j] = aj; cc[j] = cj;
        }
        *reinterpret_cast<f32x4*>(r + 4 * q) = pp;
        if (NS >= 1) *reinterpret_cast<f32x4*>(r + K + 4 + 4 * q) = aa;
        if (NS >= 2) *reinterpret_cast<f32x4*>(r + 2 * K + 4 + 4 * q) = cc;
      }
      f32x4 w = wq[u];
      float pw = w[0], aw = w[1], cw = w[2];
      float gw = l2_grad(0.f, h.l2, pw);
      opt_update<OPT>(pw, gw, aw, cw, h, lr_t);
      w[0] = pw;
      if (NS >= 1) w[1] = aw;
      if (NS >= 2) w[2] = cw;
      *reinterpret_cast<f32x4*>(r + K) = w;
      // the record's tail pad (always zero) is written too: whole 128-B lines leave L2 fully
      // dirty, so their write-back needs no read-modify-write
#pragma unroll
      for (int q = (K + 4 + NS * K) / 4; q < REC / 4; ++q)
        *reinterpret_cast<f32x4*>(r + 4 * q) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// the sweep workgroups of sfwg_kernel (nblk = 0: none)
struct SweepArgs {
  float* rec;
  unsigned char* flags;
  int64_t* sw_step;   // the branch sweep's counter: set to the advanced step by the last arriver
  long R;
  int ld;
  int nblk;
};
