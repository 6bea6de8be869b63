// Reproducer 2: the gather-fused tower's FM prologue alone (tower.hip tower_gather, the code that
// lost run-to-run determinism with packed-FP32 VALU ops on): 512 workgroups of 32 samples with the
// tower's LDS footprint (two per CU), launched repeatedly on identical inputs; every launch's FM
// logits must be bitwise equal to the first one's.
// build: hipcc --offload-arch=gfx950 -O3 -I../../csrc/kernels [-Xclang -target-feature -Xclang
//        -packed-fp32-ops] gather_repro.hip -o gather_repro ; run: ./gather_repro <launches>
#include "../../csrc/kernels/tower.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int KE>
__global__ void __launch_bounds__(256) gather_only(TowerArgs a, float* out) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  bf16* lds = reinterpret_cast<bf16*>(lds_raw);
  __shared__ float s_yfm[TW_ROWS];
  __shared__ float s_dq0[TW_ROWS];
  const int row0 = blockIdx.x * TW_ROWS;
  tower_gather<false, KE>(a, row0, lds, a.K0p + 8, nullptr, 0, s_yfm, s_dq0);
  __syncthreads();
  if (threadIdx.x < TW_ROWS) out[row0 + threadIdx.x] = s_yfm[threadIdx.x];
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 50;
  const int B = 16384, F = 39, K = 8, LD = 32, K0p = 320;
  const long V = 1 << 20;
  std::vector<float> tab((size_t)V * LD), vals((size_t)B * F);
  std::vector<int> ids((size_t)B * F);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s; };
  for (auto& x : tab) x = ((int)(rnd() >> 9) % 2001 - 1000) * 1e-5f;
  for (int b = 0; b < B; ++b)
    for (int f = 0; f < F; ++f) {
      ids[(size_t)b * F + f] = (int)(rnd() % (V / F)) + f * (int)(V / F);
      vals[(size_t)b * F + f] = f < 13 ? ((rnd() >> 8) % 1000) * 1e-3f : 1.f;
    }
  float *dtab, *dvals, *dout, *dbias;
  int* dids;
  (void)hipMalloc(&dtab, tab.size() * 4);
  (void)hipMalloc(&dvals, vals.size() * 4);
  (void)hipMalloc(&dids, ids.size() * 4);
  (void)hipMalloc(&dout, (size_t)launches * B * 4);
  (void)hipMalloc(&dbias, 4);
  (void)hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dvals, vals.data(), vals.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemset(dbias, 0, 4);
  TowerArgs a{};
  a.idx = dids;
  a.vals = dvals;
  a.tv = dtab;
  a.tw = dtab + K;
  a.ldv = a.ldw = LD;
  a.F = F;
  a.K0p = K0p;
  a.fm_bias = dbias;
  const int lds = 100 * 1024;       // the tower's footprint class: two workgroups per CU
  (void)hipFuncSetAttribute((const void*)gather_only<8>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  for (int l = 0; l < launches; ++l)
    hipLaunchKernelGGL(gather_only<8>, dim3(B / TW_ROWS), dim3(256), lds, 0, a, dout + (size_t)l * B);
  std::vector<float> out((size_t)launches * B);
  (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  long bad = 0, bad_launches = 0;
  for (int l = 1; l < launches; ++l) {
    long nb = 0;
    for (int b = 0; b < B; ++b) nb += out[(size_t)l * B + b] != out[b];
    bad += nb;
    bad_launches += nb != 0;
  }
  printf("launches %d: %ld samples differ from launch 0 in %ld launches\n", launches, bad, bad_launches);
  return 0;
}
