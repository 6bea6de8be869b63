// Host micro-benchmark of the TFRecord path: CRC32C and Example decode per record, one thread
// (built against csrc/io/hfm_io.cpp; scripts/experiments/r5_nice.sh runs it on the GPU box).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <string>
#include <cstdint>
extern "C" {
uint32_t hfmio_crc32c(const uint8_t* p, size_t n);
int hfmio_decode_example(const uint8_t* p, size_t len, int F, float* label, int64_t* ids, float* vals);
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  std::vector<uint8_t> buf;
  fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
  buf.resize(n); fread(buf.data(), 1, n, f); fclose(f);
  std::vector<std::pair<size_t,size_t>> recs;
  size_t off = 0;
  while (off + 12 <= (size_t)n) { uint64_t len; memcpy(&len, &buf[off], 8); recs.push_back({off + 12, len}); off += 12 + len + 4; }
  printf("records %zu, mean len %.1f\n", recs.size(), (double)(n) / recs.size());
  float lab, vals[39]; int64_t ids[39];
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    uint32_t acc = 0;
    for (auto& r : recs) acc ^= hfmio_crc32c(&buf[r.first], r.second);
    auto t1 = std::chrono::steady_clock::now();
    long ok = 0;
    for (auto& r : recs) ok += hfmio_decode_example(&buf[r.first], r.second, 39, &lab, ids, vals) == 0;
    auto t2 = std::chrono::steady_clock::now();
    auto ns = [&](auto a, auto b) { return std::chrono::duration<double, std::nano>(b - a).count() / recs.size(); };
    printf("crc %.1f ns/rec, decode %.1f ns/rec (ok %ld, %u)\n", ns(t0, t1), ns(t1, t2), ok, acc & 1);
  }
}
