// Single-thread cost of the TFRecord input stages (csrc/io/hfm_io.cpp) on one file: block read +
// CRC, Example decode, and both; ns per record.  Build: g++ -O3 -std=c++17 -msse4.2 -pthread
// tools/io_microbench.cpp -o /tmp/io_microbench ; run: /tmp/io_microbench <file.tfrecords> [F]
#include "../csrc/io/hfm_io.cpp"
#include <chrono>
int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int F = argc > 2 ? atoi(argv[2]) : 39;
  using Clk = std::chrono::steady_clock;
  std::vector<float> vals(F), lab(1);
  std::vector<int64_t> ids(F);
  for (int mode = 0; mode < 3; ++mode) {
    BlockReader r(argv[1]);
    const uint8_t* rp;
    uint64_t len;
    size_t pend = 0;
    long n = 0;
    const auto t0 = Clk::now();
    while (next_tfrecord_view(r, rp, len, mode != 1, pend) == 1) {
      if (mode >= 1 && !decode_example(rp, len, F, lab.data(), ids.data(), vals.data())) return 1;
      ++n;
    }
    const double s = std::chrono::duration<double>(Clk::now() - t0).count();
    printf("%s: %ld records, %.1f ns/record\n",
           mode == 0 ? "read+crc" : mode == 1 ? "read+decode (no crc)" : "read+crc+decode", n, s * 1e9 / n);
  }
  return 0;
}
