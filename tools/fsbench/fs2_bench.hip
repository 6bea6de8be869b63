// Standalone timing of the run-level sort body (csrc/kernels/fsort_run.h): the counter-rank form
// (fs2_sort_item, 4-bit digits) against the ballot form (fs2_sort_item_ballot, 8-bit digits) over
// field widths, batch sizes and id layouts, each checked against std::stable_sort.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../csrc/kernels fs2_bench.hip -o fs2b && ./fs2b
// (-DFS2_DBG_PASSES=n caps the LSD passes to split the time between the id loads and the passes)
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstdlib>
#include "fsort_run.h"

template <int FORM>
__global__ void __launch_bounds__(FS2_THREADS) k_sort(const FsJob* jobs, int nitems) {
  extern __shared__ __align__(16) unsigned char lds[];
  if (FORM) fs2_sort_item(jobs[0], blockIdx.x % nitems, lds);
  else fs2_sort_item_ballot(jobs[0], blockIdx.x % nitems, lds);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const int F = 39;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  long total_bad = 0;
  const bool quick = getenv("FS2_QUICK") != nullptr;
  for (int B : {16384, 1024, 6000, 3000, 1500, 12000, 6001}) {
    if (!quick && B != 16384 && B != 1024) continue;
    for (int bits : {6, 13, 22, 28}) {
      std::vector<int> ids((size_t)B * F), fr(4 * F);
      unsigned x = 12345u + bits;
      for (auto& v : ids) { x = x * 1664525u + 1013904223u; v = (int)(x >> 4) & ((1 << bits) - 1); }
      for (int f = 0; f < F; ++f) { fr[4 * f] = 0; fr[4 * f + 1] = 1 << bits; fr[4 * f + 2] = bits; fr[4 * f + 3] = 0; }
      std::vector<int> idsT((size_t)B * F);
      for (int r = 0; r < B; ++r) for (int f = 0; f < F; ++f) idsT[(size_t)f * B + r] = ids[(size_t)r * F + f];
      int *d_ids, *d_idsT, *d_fr, *d_work, *d_keys, *d_perm; unsigned* d_err; FsJob* d_job;
      CK(hipMalloc(&d_ids, ids.size() * 4)); CK(hipMalloc(&d_idsT, ids.size() * 4)); CK(hipMalloc(&d_fr, fr.size() * 4));
      CK(hipMalloc(&d_keys, ids.size() * 4)); CK(hipMalloc(&d_perm, ids.size() * 4)); CK(hipMalloc(&d_err, 4));
      CK(hipMalloc(&d_job, sizeof(FsJob)));
      std::vector<int> work(2 * F); for (int f = 0; f < F; ++f) { work[2 * f] = f; work[2 * f + 1] = 0; }
      CK(hipMalloc(&d_work, work.size() * 4));
      CK(hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_idsT, idsT.data(), ids.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_fr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_work, work.data(), work.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemset(d_err, 0, 4));
      // reference: stable sort of every field
      std::vector<int> rk((size_t)B * F), rp((size_t)B * F);
      for (int f = 0; f < F; ++f) {
        std::vector<std::pair<int, int>> ref(B);
        for (int r = 0; r < B; ++r) ref[r] = {ids[(size_t)r * F + f], r * F + f};
        std::stable_sort(ref.begin(), ref.end(), [](auto& p, auto& q) { return p.first < q.first; });
        for (int i = 0; i < B; ++i) { rk[(size_t)f * B + i] = ref[i].first; rp[(size_t)f * B + i] = ref[i].second; }
      }
      for (int fm = 0; fm < 2; ++fm) {
        for (int form = 0; form < 2; ++form) {
          FsJob J{}; J.ids = fm ? d_idsT : d_ids; J.ld = fm ? B : 0; J.B = B; J.F = F; J.fr = d_fr; J.work = d_work;
          J.nwork = F; J.keys = d_keys; J.perm = d_perm; J.err = d_err;
          CK(hipMemcpy(d_job, &J, sizeof(J), hipMemcpyHostToDevice));
          CK(hipMemset(d_keys, 0xff, ids.size() * 4));
          auto launch = [&](int nwg) {
            if (form) hipLaunchKernelGGL(k_sort<1>, dim3(nwg), dim3(FS2_THREADS), FS2_LDS, 0, d_job, F);
            else hipLaunchKernelGGL(k_sort<0>, dim3(nwg), dim3(FS2_THREADS), FS2_LDS_BALLOT, 0, d_job, F);
          };
          launch(F);
          CK(hipDeviceSynchronize());
          std::vector<int> keys((size_t)B * F), perm((size_t)B * F);
          CK(hipMemcpy(keys.data(), d_keys, keys.size() * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(perm.data(), d_perm, perm.size() * 4, hipMemcpyDeviceToHost));
          long bad = 0;
          long first = -1;
          for (size_t i = 0; i < keys.size(); ++i) {
            const bool b1 = (keys[i] != rk[i]) || (perm[i] != rp[i]);
            if (b1 && first < 0) first = (long)i;
            bad += b1;
          }
          total_bad += bad;
          if (bad) printf("  first mismatch at %ld (field %ld, pos %ld): key %d/%d perm %d/%d\n", first, first / B, first % B,
                          keys[first], rk[first], perm[first], rp[first]);
          for (int nwg : {39, 256, 780}) {
            if (quick && nwg != 256) continue;
            const int R = 20;
            launch(nwg);
            CK(hipEventRecord(a));
            for (int r = 0; r < R; ++r) launch(nwg);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("B %5d bits %2d %s %s %3d wg: %8.2f us/launch  mismatches %ld\n", B, bits,
                   fm ? "field-major" : "row-major  ", form ? "counter" : "ballot ", nwg, ms * 1000 / R, bad);
          }
        }
      }
      hipFree(d_ids); hipFree(d_idsT); hipFree(d_fr); hipFree(d_work); hipFree(d_keys); hipFree(d_perm);
      hipFree(d_err); hipFree(d_job);
    }
  }
  printf("total mismatches %ld\n", total_bad);
  return total_bad ? 2 : 0;
}
