// Standalone timing of the run-level sort body (csrc/kernels/fsort_run.h) on one 16K-row field:
// row-major vs field-major ids, and pass-capped builds (-DFS2_DBG_PASSES=n) to split the time
// between the id loads and the LSD passes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels fs2_bench.hip -o fs2b && ./fs2b
#include <cstdio>
#include <vector>
#include <algorithm>
#include "fsort_run.h"

__global__ void __launch_bounds__(FS2_THREADS) k_sort(const FsJob* jobs, int nitems) {
  extern __shared__ __align__(16) unsigned char lds[];
  fs2_sort_item(jobs[0], blockIdx.x % nitems, lds);
}

int main() {
  const int B = 16384, F = 39, bits = 28;
  std::vector<int> ids((size_t)B * F), fr(4 * F);
  unsigned x = 12345;
  for (auto& v : ids) { x = x * 1664525u + 1013904223u; v = (int)(x >> 4) & ((1 << bits) - 1); }
  for (int f = 0; f < F; ++f) { fr[4 * f] = 0; fr[4 * f + 1] = 1 << bits; fr[4 * f + 2] = bits; fr[4 * f + 3] = 0; }
  std::vector<int> idsT((size_t)B * F);
  for (int b = 0; b < B; ++b) for (int f = 0; f < F; ++f) idsT[(size_t)f * B + b] = ids[(size_t)b * F + f];
  int *d_ids, *d_idsT, *d_fr, *d_work, *d_keys, *d_perm; unsigned* d_err; FsJob* d_job;
  hipMalloc(&d_ids, ids.size() * 4); hipMalloc(&d_idsT, ids.size() * 4); hipMalloc(&d_fr, fr.size() * 4);
  hipMalloc(&d_keys, ids.size() * 4); hipMalloc(&d_perm, ids.size() * 4); hipMalloc(&d_err, 4);
  hipMalloc(&d_job, sizeof(FsJob));
  std::vector<int> work(2 * F); for (int f = 0; f < F; ++f) { work[2 * f] = f; work[2 * f + 1] = 0; }
  hipMalloc(&d_work, work.size() * 4);
  hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_idsT, idsT.data(), ids.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_fr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_work, work.data(), work.size() * 4, hipMemcpyHostToDevice);
  hipMemset(d_err, 0, 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int fm = 0; fm < 2; ++fm) {
    for (int nwg : {1, 39, 256, 512}) {
      FsJob J{}; J.ids = fm ? d_idsT : d_ids; J.ld = fm ? B : 0; J.B = B; J.F = F; J.fr = d_fr; J.work = d_work;
      J.nwork = F; J.keys = d_keys; J.perm = d_perm; J.err = d_err;
      hipMemcpy(d_job, &J, sizeof(J), hipMemcpyHostToDevice);
      const int R = 20;
      hipLaunchKernelGGL(k_sort, dim3(nwg), dim3(FS2_THREADS), FS2_LDS, 0, d_job, F);
      hipEventRecord(a);
      for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_sort, dim3(nwg), dim3(FS2_THREADS), FS2_LDS, 0, d_job, F);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("fs2 sort %s ids, %3d workgroups: %8.2f us/launch\n", fm ? "field-major" : "row-major  ", nwg,
             ms * 1000 / R);
    }
  }
  // correctness of field 0 (row-major run)
  FsJob J{}; J.ids = d_ids; J.ld = 0; J.B = B; J.F = F; J.fr = d_fr; J.work = d_work; J.nwork = F;
  J.keys = d_keys; J.perm = d_perm; J.err = d_err;
  hipMemcpy(d_job, &J, sizeof(J), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_sort, dim3(F), dim3(FS2_THREADS), FS2_LDS, 0, d_job, F);
  std::vector<int> keys(B), perm(B);
  hipMemcpy(keys.data(), d_keys, B * 4, hipMemcpyDeviceToHost);
  hipMemcpy(perm.data(), d_perm, B * 4, hipMemcpyDeviceToHost);
  std::vector<std::pair<int, int>> ref(B);
  for (int b = 0; b < B; ++b) ref[b] = {ids[(size_t)b * F], b * F};
  std::stable_sort(ref.begin(), ref.end(), [](auto& p, auto& q) { return p.first < q.first; });
  long bad = 0;
  for (int i = 0; i < B; ++i) bad += (keys[i] != ref[i].first) || (perm[i] != ref[i].second);
  printf("field 0 mismatches: %ld (passes %d)\n", bad, (bits + 7) / 8);
  return 0;
}
