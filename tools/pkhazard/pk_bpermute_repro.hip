// Minimal reproducer: a packed-FP32 VALU result (v_pk_add_f32, 2 lanes-halves per VGPR pair) read
// by the very next ds_bpermute_b32 (the lowering of __shfl_xor) on gfx950.
//
// Each lane holds 8 float pairs built with float2 arithmetic (the compiler emits v_pk_add_f32 for
// them when packed-FP32 ops are enabled), then reduces them over groups of 8 lanes with the xor
// butterfly 1, 2, 4 -- the tower kernel's FM-gather reduction pattern.  Every lane of a group must
// end with the same, exactly representable sum (small integers), so any mismatch is a stale read.
// Mode 1 replaces the shuffles with a DPP butterfly (quad_perm xor1 / xor2, row_half_mirror): no
// DS instruction reads the packed result.
//
// build: hipcc --offload-arch=gfx950 -O3 [-Xclang -target-feature -Xclang -packed-fp32-ops] \
//        pk_bpermute_repro.hip -o pkrepro ; run: ./pkrepro <mode 0|1> <iterations>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ float xor_dpp(float v, int ctrl) {
  int x = __float_as_int(v);
  int r;
  switch (ctrl) {
    case 1: r = __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false); break;   // quad_perm 1,0,3,2
    case 2: r = __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false); break;   // quad_perm 2,3,0,1
    default: r = __builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false); break; // row_half_mirror
  }
  return __int_as_float(r);
}

template <int MODE>
__global__ void __launch_bounds__(256) repro(const float* __restrict__ in, unsigned* __restrict__ bad, int iters) {
  const int tid = threadIdx.x;
  const int g = blockIdx.x * 256 + tid;
  unsigned nbad = 0;
  for (int it = 0; it < iters; ++it) {
    float2 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float2 a = {in[(g * 8 + 2 * j + it) & 4095], in[(g * 8 + 2 * j + 1 + it) & 4095]};
      const float2 b = {in[(g * 8 + 2 * j + 7 * it) & 4095], in[(g * 8 + 2 * j + 3 + it) & 4095]};
      s[j] = make_float2(a.x + b.x, a.y + b.y);   // -> v_pk_add_f32 with packed ops on
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (MODE == 0) {
          s[j].x += __shfl_xor(s[j].x, o, 64);
          s[j].y += __shfl_xor(s[j].y, o, 64);
        } else {
          s[j].x += xor_dpp(s[j].x, o);
          s[j].y += xor_dpp(s[j].y, o);
        }
      }
    }
    // every lane of the 8-lane group must hold the group's sum: compare with lane 0 of the group
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x0 = __shfl(s[j].x, tid & ~7, 64), y0 = __shfl(s[j].y, tid & ~7, 64);
      nbad += (s[j].x != x0) + (s[j].y != y0);
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0, iters = argc > 2 ? atoi(argv[2]) : 2000;
  float h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (float)(i % 97);
  float* d;
  unsigned* bad;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&bad, 4);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 4);
  const int blocks = 256 * 2;   // two workgroups per CU (the condition the tower kernel ran in)
  if (mode == 0) hipLaunchKernelGGL(repro<0>, dim3(blocks), dim3(256), 0, 0, d, bad, iters);
  else hipLaunchKernelGGL(repro<1>, dim3(blocks), dim3(256), 0, 0, d, bad, iters);
  unsigned nb = 0;
  hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
  const double total = (double)blocks * 256 * iters * 8;
  printf("mode %d (%s): %u mismatching lanes of %.0f (%.3g)\n", mode, mode ? "DPP" : "ds_bpermute", nb, total,
         nb / total);
  hipFree(d);
  hipFree(bad);
  return 0;
}
