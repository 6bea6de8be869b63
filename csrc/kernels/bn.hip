// K6b batch norm in the deep tower: the reference's
// ``batch_norm_layer`` (1-ps-cpu/DeepFM-dist-ps-for-multipleCPU-multiInstance.py:288-292,
// tf.contrib.layers.batch_norm, center+scale, eps 1e-3, updates_collections=None) applied
// AFTER the ReLU and BEFORE dropout (PS:213-218), batch statistics per rank (no sync-BN, as
// with Horovod).
//
// Per BN layer the step is
//   fwd:  R = relu(X W^T + b)                 (gemm_nt EPI_RELU_F32, f32 R)
//         part[tile] = (sum R, sum R^2)        bn_partial<0>   (deterministic per-64-row tiles)
//         mean, var, scale, shift, moving      bn_finalize<0>  (double reduction, fixed order)
//         H = (R*scale + shift)*keep/keep_p    bn_apply<0>     (-> H and H^T, LDS transpose)
//   bwd:  dY = dH (.) keep/keep_p              (dH fp32 from gemm EPI_F32 or the head)
//         part[tile] = (sum dY, sum dY*xhat)   bn_partial<1>
//         dbeta, dgamma, c1, c2                bn_finalize<2>  (grads land in the flat buffer)
//         dZ = (R>0) gamma*rstd*(dY - c1 - xhat*c2)   bn_apply<1>  (-> dZ and dZ^T)
// Dropout masks are regenerated from the counter hash with the same flat index as the GEMM
// epilogue (row * Npad + col).  Padding rows (>= nvalid) are excluded from every statistic
// and get a zero gradient.
#include "common.h"

struct BnArgs {
  int M, N, nvalid;
  const float* r;         // [M,N] relu output (pre-BN), f32
  const float* dh;        // [M,N] gradient w.r.t. the layer output (post BN + dropout)
  const float* gamma;     // [N]
  const float* beta;      // [N]
  float* mm;              // moving mean [N]
  float* mv;              // moving variance [N]
  float* save;            // [6,N]: mean, rstd, scale, shift, c1, c2
  float* part;            // [M/64, 2N]
  float* dgamma;          // [N] (flat gradient buffer)
  float* dbeta;           // [N]
  float eps, decay;
  uint32_t seed, layer, keep_thr;
  int drop;
  float inv_keep;
  const int64_t* step;
  bf16* out;              // fwd: H [M,N]   bwd: dZ [M,N]
  bf16* out_t;            // fwd: H^T       bwd: dZ^T   (nullable)
};

__device__ __forceinline__ float drop_factor(const BnArgs& a, uint32_t salt, int row, int col) {
  if (!a.drop) return 1.f;
  return dropout_keep((uint32_t)(row * a.N + col), salt, a.keep_thr) ? a.inv_keep : 0.f;
}

// grid (M/64, N/(32 CPT)), 256 threads: 32 column groups of CPT adjacent columns x 8 row-groups
// of 8 rows.  CPT = 4 (N % 128 == 0): 16-byte loads of r / dh; every column's sums take the same
// order for either CPT (8 rows in sequence per row-group, then the fixed 8-way tree), so both
// variants write bitwise the same partials.
template <int BWD, int CPT>
__global__ void __launch_bounds__(256) bn_partial_kernel(BnArgs a) {
  typedef float vecT __attribute__((ext_vector_type(CPT)));
  __shared__ float red[2][8][32 * CPT];
  const int c = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int col = blockIdx.y * 32 * CPT + c * CPT;
  const int r0 = blockIdx.x * 64 + rg * 8;
  const float* sv = a.save;
  float mean[CPT], rstd[CPT];
  uint32_t salt = 0;
#pragma unroll
  for (int q = 0; q < CPT; ++q) mean[q] = rstd[q] = 0.f;
  if (BWD) {
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      mean[q] = sv[col + q];
      rstd[q] = sv[a.N + col + q];
    }
    if (a.drop) salt = dropout_salt(a.seed, (uint32_t)(*a.step), a.layer);
  }
  float s0[CPT], s1[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) s0[q] = s1[q] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = r0 + j;
    if (row < a.nvalid) {
      const size_t o = (size_t)row * a.N + col;
      vecT x, d;
      if (CPT == 1) {
        x[0] = a.r[o];
        if (BWD) d[0] = a.dh[o];
      } else {
        x = *reinterpret_cast<const vecT*>(a.r + o);
        if (BWD) d = *reinterpret_cast<const vecT*>(a.dh + o);
      }
#pragma unroll
      for (int q = 0; q < CPT; ++q) {
        if (BWD) {
          const float dy = d[q] * drop_factor(a, salt, row, col + q);
          s0[q] += dy;
          s1[q] += dy * (x[q] - mean[q]) * rstd[q];
        } else {
          s0[q] += x[q];
          s1[q] += x[q] * x[q];
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    red[0][rg][c * CPT + q] = s0[q];
    red[1][rg][c * CPT + q] = s1[q];
  }
  __syncthreads();
  // 2 x 32 CPT output columns: thread -> (sum kind, column)
  for (int e = threadIdx.x; e < 2 * 32 * CPT; e += 256) {
    const int k = e / (32 * CPT), cc = e % (32 * CPT);
    const float* v = &red[k][0][cc];
    constexpr int S = 32 * CPT;
    const float t = ((v[0] + v[S]) + (v[2 * S] + v[3 * S])) + ((v[4 * S] + v[5 * S]) + (v[6 * S] + v[7 * S]));
    a.part[(size_t)blockIdx.x * 2 * a.N + k * a.N + blockIdx.y * 32 * CPT + cc] = t;
  }
}

// MODE 0: train forward (batch stats + moving-average update), 1: eval (moving stats),
// 2: backward (dbeta/dgamma + c1/c2).  grid N/32, 256 threads: 32 columns x 8 row-lanes.
template <int MODE>
__global__ void __launch_bounds__(256) bn_finalize_kernel(BnArgs a, int nrow) {
  __shared__ double red[2][8][32];
  const int c = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + c;
  const int N = a.N;
  double s0 = 0.0, s1 = 0.0;
  if (MODE != 1) {
    for (int r = rl; r < nrow; r += 8) {
      s0 += (double)a.part[(size_t)r * 2 * N + col];
      s1 += (double)a.part[(size_t)r * 2 * N + N + col];
    }
  }
  red[0][rl][c] = s0;
  red[1][rl][c] = s1;
  __syncthreads();
  if (rl != 0) return;
  s0 = ((red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c])) +
       ((red[0][4][c] + red[0][5][c]) + (red[0][6][c] + red[0][7][c]));
  s1 = ((red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c])) +
       ((red[1][4][c] + red[1][5][c]) + (red[1][6][c] + red[1][7][c]));
  float* sv = a.save;
  const double n = (double)a.nvalid;
  if (MODE == 2) {
    a.dbeta[col] = (float)s0;
    a.dgamma[col] = (float)s1;
    sv[4 * N + col] = (float)(s0 / n);
    sv[5 * N + col] = (float)(s1 / n);
    return;
  }
  float mean, var;
  if (MODE == 0) {
    const double m = s0 / n;
    double v = s1 / n - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    const float d = a.decay;
    const float unb = (float)(v * (n / (n > 1.0 ? n - 1.0 : 1.0)));   // fused BN reports Bessel var
    a.mm[col] = a.mm[col] * d + mean * (1.f - d);
    a.mv[col] = a.mv[col] * d + unb * (1.f - d);
  } else {
    mean = a.mm[col];
    var = a.mv[col];
  }
  const float rstd = 1.f / sqrtf(var + a.eps);
  const float scale = a.gamma[col] * rstd;
  sv[col] = mean;
  sv[N + col] = rstd;
  sv[2 * N + col] = scale;
  sv[3 * N + col] = a.beta[col] - mean * scale;
}

// grid (M/64, N/32), 256 threads; tile 64 rows x 32 cols, 8 contiguous columns per thread,
// transposed copy through LDS (each thread then writes 8 consecutive rows of one column).
template <int BWD>
__global__ void __launch_bounds__(256) bn_apply_kernel(BnArgs a) {
  __shared__ bf16 tile[32][64 + 8];
  const int t = threadIdx.x;
  const int lr = t >> 2, cq = (t & 3) * 8;
  const int row = blockIdx.x * 64 + lr;
  const int cb = blockIdx.y * 32 + cq;
  const int N = a.N;
  const float* sv = a.save;
  uint32_t salt = 0;
  if (a.drop) salt = dropout_salt(a.seed, (uint32_t)(*a.step), a.layer);
  const size_t o = (size_t)row * N + cb;
  const f32x4 xr0 = *reinterpret_cast<const f32x4*>(a.r + o);
  const f32x4 xr1 = *reinterpret_cast<const f32x4*>(a.r + o + 4);
  f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0;      // dL/dh in 16-byte loads, issued with r's
  if (BWD) {
    d0 = *reinterpret_cast<const f32x4*>(a.dh + o);
    d1 = *reinterpret_cast<const f32x4*>(a.dh + o + 4);
  }
  bf16x8 ov;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = cb + j;
    const float x = j < 4 ? xr0[j] : xr1[j - 4];
    float v;
    if (BWD) {
      if (row < a.nvalid && x > 0.f) {
        const float dy = (j < 4 ? d0[j] : d1[j - 4]) * drop_factor(a, salt, row, col);
        const float xhat = (x - sv[col]) * sv[N + col];
        v = sv[2 * N + col] * (dy - sv[4 * N + col] - xhat * sv[5 * N + col]);
      } else {
        v = 0.f;
      }
    } else {
      v = (x * sv[2 * N + col] + sv[3 * N + col]) * drop_factor(a, salt, row, col);
    }
    ov[j] = f2bf(v);
    tile[cq + j][lr] = ov[j];
  }
  *reinterpret_cast<bf16x8*>(a.out + o) = ov;
  if (!a.out_t) return;
  __syncthreads();
  const int tc = t >> 3, tr = (t & 7) * 8;
  bf16x8 w;
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = tile[tc][tr + j];
  *reinterpret_cast<bf16x8*>(a.out_t + (size_t)(blockIdx.y * 32 + tc) * a.M + blockIdx.x * 64 + tr) = w;
}

// The same per-element values as bn_apply_kernel over 64 x 64 tiles (N % 64 == 0): two 8-column
// row pieces per thread, every load (r, dh, the per-column statistics) in 16-byte vectors, the
// transposed copy through a padded LDS tile with 32 contiguous bytes of out_t per thread.
template <int BWD>
__global__ void __launch_bounds__(256) bn_apply64_kernel(BnArgs a) {
  __shared__ bf16 tile[64][64 + 8];
  const int t = threadIdx.x;
  const int row0 = blockIdx.x * 64, col0 = blockIdx.y * 64;
  const int N = a.N;
  const float* sv = a.save;
  uint32_t salt = 0;
  if (a.drop) salt = dropout_salt(a.seed, (uint32_t)(*a.step), a.layer);
  const int c = (t & 7) * 8, cb = col0 + c;
  // per-column statistics of the thread's 8 columns (the same for both row pieces)
  f32x4 s2[2], s3[2], s0[2], s1[2], s4[2], s5[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    s2[h] = *reinterpret_cast<const f32x4*>(sv + 2 * N + cb + 4 * h);
    if (BWD) {
      s0[h] = *reinterpret_cast<const f32x4*>(sv + cb + 4 * h);
      s1[h] = *reinterpret_cast<const f32x4*>(sv + N + cb + 4 * h);
      s4[h] = *reinterpret_cast<const f32x4*>(sv + 4 * N + cb + 4 * h);
      s5[h] = *reinterpret_cast<const f32x4*>(sv + 5 * N + cb + 4 * h);
    } else {
      s3[h] = *reinterpret_cast<const f32x4*>(sv + 3 * N + cb + 4 * h);
    }
  }
  f32x4 xr[2][2], dr[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const size_t o = (size_t)(row0 + (t >> 3) + 32 * p) * N + cb;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      xr[p][h] = *reinterpret_cast<const f32x4*>(a.r + o + 4 * h);
      if (BWD) dr[p][h] = *reinterpret_cast<const f32x4*>(a.dh + o + 4 * h);
    }
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int lr = (t >> 3) + 32 * p, row = row0 + lr;
    bf16x8 ov;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = cb + j, h = j >> 2, q = j & 3;
      const float x = xr[p][h][q];
      float v;
      if (BWD) {
        if (row < a.nvalid && x > 0.f) {
          const float dy = dr[p][h][q] * drop_factor(a, salt, row, col);
          const float xhat = (x - s0[h][q]) * s1[h][q];
          v = s2[h][q] * (dy - s4[h][q] - xhat * s5[h][q]);
        } else {
          v = 0.f;
        }
      } else {
        v = (x * s2[h][q] + s3[h][q]) * drop_factor(a, salt, row, col);
      }
      ov[j] = f2bf(v);
    }
    *reinterpret_cast<bf16x8*>(a.out + (size_t)row * N + cb) = ov;
    *reinterpret_cast<bf16x8*>(&tile[lr][c]) = ov;
  }
  if (!a.out_t) return;
  __syncthreads();
  const int cc = t >> 2, rr = (t & 3) * 16;
  bf16x8 w0, w1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w0[k] = tile[rr + k][cc];
    w1[k] = tile[rr + 8 + k][cc];
  }
  bf16* dt = a.out_t + (size_t)(col0 + cc) * a.M + row0 + rr;
  *reinterpret_cast<bf16x8*>(dt) = w0;
  *reinterpret_cast<bf16x8*>(dt + 8) = w1;
}

static bool bn_shape_ok(const BnArgs& a) { return a.M % 64 == 0 && a.N % 32 == 0 && a.M > 0 && a.N > 0; }

// phase: 0 fwd partial, 1 fwd finalize (train), 2 eval finalize, 3 fwd apply,
//        4 bwd partial, 5 bwd finalize, 6 bwd apply
HFM_API int hfm_bn(int phase, const BnArgs* ap, hipStream_t st) {
  const BnArgs a = *ap;
  if (!bn_shape_ok(a)) return (int)hipErrorInvalidValue;
  const dim3 tiles(a.M / 64, a.N / 32);
  const int nrow = a.M / 64;
  switch (phase) {
    case 0:
      if (a.N % 128 == 0) hipLaunchKernelGGL((bn_partial_kernel<0, 4>), dim3(a.M / 64, a.N / 128), dim3(256), 0, st, a);
      else hipLaunchKernelGGL((bn_partial_kernel<0, 1>), tiles, dim3(256), 0, st, a);
      break;
    case 1: hipLaunchKernelGGL(bn_finalize_kernel<0>, dim3(a.N / 32), dim3(256), 0, st, a, nrow); break;
    case 2: hipLaunchKernelGGL(bn_finalize_kernel<1>, dim3(a.N / 32), dim3(256), 0, st, a, nrow); break;
    case 3:
      if (a.N % 64 == 0) hipLaunchKernelGGL(bn_apply64_kernel<0>, dim3(a.M / 64, a.N / 64), dim3(256), 0, st, a);
      else hipLaunchKernelGGL(bn_apply_kernel<0>, tiles, dim3(256), 0, st, a);
      break;
    case 4:
      if (a.N % 128 == 0) hipLaunchKernelGGL((bn_partial_kernel<1, 4>), dim3(a.M / 64, a.N / 128), dim3(256), 0, st, a);
      else hipLaunchKernelGGL((bn_partial_kernel<1, 1>), tiles, dim3(256), 0, st, a);
      break;
    case 5: hipLaunchKernelGGL(bn_finalize_kernel<2>, dim3(a.N / 32), dim3(256), 0, st, a, nrow); break;
    case 6:
      if (a.N % 64 == 0) hipLaunchKernelGGL(bn_apply64_kernel<1>, dim3(a.M / 64, a.N / 64), dim3(256), 0, st, a);
      else hipLaunchKernelGGL(bn_apply_kernel<1>, tiles, dim3(256), 0, st, a);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  HFM_LAUNCH_CHECK();
}
HFM_API int hfm_bn_args_bytes() { return (int)sizeof(BnArgs); }
