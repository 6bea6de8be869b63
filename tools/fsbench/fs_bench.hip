// Standalone timing harness for the per-field LDS sort (csrc/kernels/field_sort.hip) and its
// variants: decomposes the kernel time into loads / ranking / scan / scatter.
// build: hipcc --offload-arch=gfx950 -O3 -I csrc/kernels tools/fsbench/fs_bench.hip -o /tmp/fs_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>
#include "../../csrc/kernels/field_sort.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 16384;
  const int F = 39;
  // Criteo-1TB-shape field cardinalities (13 integer fields: 1 id each)
  const long cat[26] = {227605432, 39060, 17295, 7424, 20265, 3, 7122, 1543, 63, 130229467, 3067956,
                        405282, 10, 2209, 11938, 155, 4, 976, 14, 292775614, 40790948, 187188510,
                        590152, 12973, 108, 36};
  std::vector<int> fr(4 * F), work;
  const int max_pb = argc > 2 ? atoi(argv[2]) : 4;
  long lo = 0;
  for (int f = 0; f < F; ++f) {
    long card = f < 13 ? 1 : cat[f - 13];
    int bits = 0;
    while ((1L << bits) < card) ++bits;
    const int pb = bits < max_pb ? bits : max_pb;
    fr[4 * f] = (int)lo; fr[4 * f + 1] = (int)(lo + card); fr[4 * f + 2] = bits; fr[4 * f + 3] = pb;
    for (int c = 0; c * FS_MAXB < B; ++c)
      for (int p = 0; p < (1 << pb); ++p) { work.push_back(f); work.push_back(p); work.push_back(c); }
    lo += card;
  }
  std::mt19937_64 rng(1);
  std::vector<int> ids((size_t)B * F);
  for (int b = 0; b < B; ++b)
    for (int f = 0; f < F; ++f) {
      long card = fr[4 * f + 1] - fr[4 * f];
      double u = std::uniform_real_distribution<double>(0, 1)(rng);
      long r = (long)std::floor(std::exp(u * std::log1p((double)card))) - 1;
      r = std::min(std::max(r, 0L), card - 1);
      ids[(size_t)b * F + f] = fr[4 * f] + (int)((r * 2654435761L) % card);
    }
  int *d_ids, *d_fr, *d_sk, *d_pm, *d_work, *d_idsT; unsigned* d_err;
  const int nwork = (int)work.size() / 3;
  int *d_rk, *d_rp;
  CK(hipMalloc(&d_rk, (size_t)B * F * 4)); CK(hipMalloc(&d_rp, (size_t)B * F * 4));
  CK(hipMalloc(&d_work, work.size() * 4)); CK(hipMalloc(&d_idsT, ids.size() * 4));
  CK(hipMemcpy(d_work, work.data(), work.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_ids, ids.size() * 4)); CK(hipMalloc(&d_fr, fr.size() * 4));
  CK(hipMalloc(&d_sk, ids.size() * 4)); CK(hipMalloc(&d_pm, ids.size() * 4)); CK(hipMalloc(&d_err, 4));
  CK(hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_fr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_err, 0, 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = 0; it < 5; ++it) hfm_field_sort(d_ids, B, F, d_fr, d_work, nwork, d_idsT, d_rk, d_rp, d_sk, d_pm, d_err, st);
  CK(hipStreamSynchronize(st));
  const int R = 50;
  CK(hipEventRecord(e0, st));
  for (int it = 0; it < R; ++it) hfm_field_sort(d_ids, B, F, d_fr, d_work, nwork, d_idsT, d_rk, d_rp, d_sk, d_pm, d_err, st);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  // check
  std::vector<int> sk(ids.size()), pm(ids.size());
  CK(hipMemcpy(sk.data(), d_sk, sk.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(pm.data(), d_pm, pm.size() * 4, hipMemcpyDeviceToHost));
  std::vector<std::pair<int,int>> ref(ids.size());
  for (size_t i = 0; i < ids.size(); ++i) ref[i] = {ids[i], (int)i};
  std::stable_sort(ref.begin(), ref.end(), [](auto& a, auto& b) { return a.first < b.first; });
  long bad = 0;
  for (size_t i = 0; i < ids.size(); ++i) bad += (ref[i].first != sk[i]) || (ref[i].second != pm[i]);
  unsigned err; CK(hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost));
  printf("field_sort B=%d nwork=%d: %.2f us/launch  mismatches=%ld err=%u\n", B, nwork, ms * 1000 / R, bad, err);
  return 0;
}
