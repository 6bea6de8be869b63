// Host self-test of the native IO library, built with sanitizers:
//   g++ -fsanitize=address,undefined  -> heap/stack overflows, UB in the decoders
//   g++ -fsanitize=thread             -> races in the threaded loader (worker pool + queue)
// tests/test_sanitizers.py compiles hfm_io.cpp + this driver both ways and runs them.
//
// Checks: write/read round trip through the multi-threaded loader (order-deterministic across
// runs, every record exactly once, record-level sharding partitions the data), CRC corruption is
// detected, libsvm -> TFRecord conversion, and the Example decoder survives truncated and
// random inputs without out-of-bounds accesses.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

extern "C" {
const char* hfmio_last_error();
uint32_t hfmio_crc32c(const uint8_t* p, size_t n);
int hfmio_decode_example(const uint8_t* p, size_t len, int F, float* label, int64_t* ids, float* vals);
void* hfmio_loader_create(const char** paths, int npaths, int format, int F, int batch,
                          int drop_remainder, int num_threads, int shard_n, int shard_i,
                          int verify_crc, int queue_depth, int64_t id_limit, int narrow32);
int hfmio_loader_next(void* h, float* labels, int64_t* ids, float* vals);
void hfmio_loader_destroy(void* h);
void hfmio_loader_set_copy_threads(void* h, int n);
int hfmio_loader_start_ring(void* h, int n, float** labels, int32_t** ids, float** vals, int compact);
int hfmio_loader_ring_take(void* h, int* slot, uint64_t* mask);
void hfmio_loader_ring_give(void* h, int slot);
void* hfmio_loader_create_raw(const char** paths, int npaths, int F, int batch, int drop_remainder,
                              int num_threads, int shard_n, int shard_i, int verify_crc, int queue_depth);
int hfmio_loader_start_ring_raw(void* h, int n, uint8_t** rawb, size_t cap, uint32_t** offs);
int hfmio_write_examples(const char* path, const float* labels, const int64_t* ids,
                         const float* vals, long n, int F, int append);
long hfmio_libsvm_to_tfrecord(const char* src, const char* dst, int F);
long hfmio_count_records(const char* path, int format, int verify);
}

#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #c,     \
              hfmio_last_error());                                                 \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static const int F = 39;

struct Sum {
  double lab = 0, val = 0;
  uint64_t ids = 0, order = 0;
  long rows = 0;
};

static Sum read_all(const std::vector<std::string>& files, int threads, int shard_n, int shard_i,
                    int narrow32 = 0) {
  std::vector<const char*> p;
  for (auto& f : files) p.push_back(f.c_str());
  void* h = hfmio_loader_create(p.data(), (int)p.size(), 0, F, 64, 0, threads, shard_n, shard_i, 1, 8, 0,
                                narrow32);
  CHECK(h != nullptr);
  std::vector<float> lab(64), vals(64 * F);
  std::vector<int64_t> ids(64 * F);
  Sum s;
  for (;;) {
    const int r = hfmio_loader_next(h, lab.data(), ids.data(), vals.data());
    CHECK(r >= 0);
    if (r == 0) break;
    for (int i = 0; i < r; ++i) {
      s.lab += lab[i];
      for (int f = 0; f < F; ++f) {
        s.ids += (uint64_t)ids[i * F + f];
        s.val += vals[i * F + f];
      }
      s.order = s.order * 1000003ull + (uint64_t)ids[i * F];   // order-sensitive hash
      ++s.rows;
    }
  }
  hfmio_loader_destroy(h);
  return s;
}

// the assembly ring (assembler thread + copy pool + taker, compact values): every record once, in
// the order next() gives, the constant-1.0 fields never shipped; then destroyed mid-stream while
// the assembler waits for a slot (TSan: the ring hand-offs and the shutdown)
static Sum read_ring(const std::vector<std::string>& files, int threads, int copy_threads) {
  std::vector<const char*> p;
  for (auto& f : files) p.push_back(f.c_str());
  const int n = 3, Bt = 64;
  Sum s;
  for (int pass = 0; pass < 2; ++pass) {
    void* h = hfmio_loader_create(p.data(), (int)p.size(), 0, F, Bt, 0, threads, 1, 0, 1, 8, 0, 1);
    CHECK(h != nullptr);
    hfmio_loader_set_copy_threads(h, copy_threads);
    std::vector<std::vector<float>> lab(n, std::vector<float>(Bt)), vals(n, std::vector<float>(Bt * F));
    std::vector<std::vector<int32_t>> ids(n, std::vector<int32_t>(Bt * F));
    float* lp[n];
    float* vp[n];
    int32_t* ip[n];
    for (int i = 0; i < n; ++i) lp[i] = lab[i].data(), vp[i] = vals[i].data(), ip[i] = ids[i].data();
    CHECK(hfmio_loader_start_ring(h, n, lp, ip, vp, 1) == 0);
    for (int taken = 0;; ++taken) {
      int slot = -1;
      uint64_t mask = 0;
      const int r = hfmio_loader_ring_take(h, &slot, &mask);
      CHECK(r >= 0);
      if (r == 0 || (pass == 1 && taken == n - 1)) break;   // pass 1: every slot held, assembler waiting
      CHECK(slot >= 0 && slot < n && (mask >> 13) == 0);  // fields 13.. are all 1.0: not shipped
      const int nc = __builtin_popcountll(mask);
      if (pass == 0) {
        for (int i = 0; i < r; ++i) {
          s.lab += lab[slot][i];
          for (int f = 0; f < F; ++f) {
            s.ids += (uint64_t)ids[slot][i * F + f];
            float v = 1.0f;
            if ((mask >> f) & 1) v = vals[slot][i * nc + __builtin_popcountll(mask & ((1ull << f) - 1))];
            s.val += v;
          }
          s.order = s.order * 1000003ull + (uint64_t)ids[slot][i * F];
          ++s.rows;
        }
        hfmio_loader_ring_give(h, slot);
      }
    }
    hfmio_loader_destroy(h);
  }
  return s;
}

// the raw-record ring (mapped files, framing + CRC by the workers, assembly by the copy pool):
// every record's Example bytes once, in the decoding loader's order (host-decoded here), then
// destroyed mid-stream with every slot held (TSan: hand-offs, chunk recycling, unmapping)
static Sum read_ring_raw(const std::vector<std::string>& files, int threads, int copy_threads) {
  std::vector<const char*> p;
  for (auto& f : files) p.push_back(f.c_str());
  const int n = 3, Bt = 64;
  const size_t cap = (size_t)Bt * 2048;
  Sum s;
  for (int pass = 0; pass < 2; ++pass) {
    void* h = hfmio_loader_create_raw(p.data(), (int)p.size(), F, Bt, 0, threads, 1, 0, 1, 8);
    CHECK(h != nullptr);
    hfmio_loader_set_copy_threads(h, copy_threads);
    std::vector<std::vector<uint8_t>> raw(n, std::vector<uint8_t>(cap));
    std::vector<std::vector<uint32_t>> offs(n, std::vector<uint32_t>(Bt + 1));
    uint8_t* rp[n];
    uint32_t* op[n];
    for (int i = 0; i < n; ++i) rp[i] = raw[i].data(), op[i] = offs[i].data();
    CHECK(hfmio_loader_start_ring_raw(h, n, rp, cap, op) == 0);
    std::vector<float> lab(1), vals(F);
    std::vector<int64_t> ids(F);
    for (int taken = 0;; ++taken) {
      int slot = -1;
      uint64_t bytes = 0;
      const int r = hfmio_loader_ring_take(h, &slot, &bytes);
      CHECK(r >= 0);
      if (r == 0 || (pass == 1 && taken == n - 1)) break;
      CHECK(slot >= 0 && slot < n && offs[slot][r] == bytes && bytes <= cap);
      if (pass == 0) {
        for (int i = 0; i < r; ++i) {
          const uint32_t o0 = offs[slot][i], o1 = offs[slot][i + 1];
          CHECK(o0 < o1 && o1 <= bytes);
          CHECK(hfmio_decode_example(raw[slot].data() + o0, o1 - o0, F, lab.data(), ids.data(), vals.data()) == 0);
          s.lab += lab[0];
          for (int f = 0; f < F; ++f) {
            s.ids += (uint64_t)ids[f];
            s.val += vals[f];
          }
          s.order = s.order * 1000003ull + (uint64_t)ids[0];
          ++s.rows;
        }
      }
      hfmio_loader_ring_give(h, slot);
    }
    hfmio_loader_destroy(h);
  }
  return s;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const long n_per = 1500;
  const int nfiles = 3;
  std::vector<std::string> files;
  Sum want;
  for (int fi = 0; fi < nfiles; ++fi) {
    std::vector<float> lab(n_per), vals(n_per * F);
    std::vector<int64_t> ids(n_per * F);
    for (long i = 0; i < n_per; ++i) {
      lab[i] = (float)((i + fi) % 2);
      want.lab += lab[i];
      for (int f = 0; f < F; ++f) {
        ids[i * F + f] = (int64_t)((fi * 1000003L + i * 131L + f * 7919L) % 117581L);
        vals[i * F + f] = f < 13 ? (float)((i % 17) * 0.25) : 1.0f;
        want.ids += (uint64_t)ids[i * F + f];
        want.val += vals[i * F + f];
      }
    }
    files.push_back(dir + "/tr_selftest_" + std::to_string(fi) + ".tfrecords");
    CHECK(hfmio_write_examples(files.back().c_str(), lab.data(), ids.data(), vals.data(), n_per, F, 0) == 0);
    CHECK(hfmio_count_records(files.back().c_str(), 0, 1) == n_per);
  }
  want.rows = n_per * nfiles;

  // 1) full read, 4 worker threads: every record once; deterministic order across runs
  const Sum a = read_all(files, 4, 1, 0), b = read_all(files, 4, 1, 0);
  CHECK(a.rows == want.rows && a.ids == want.ids && a.lab == want.lab && a.val == want.val);
  CHECK(a.order == b.order);
  // ids narrowed to int32 while decoding (the device path) read back identically
  const Sum n32 = read_all(files, 4, 1, 0, 1);
  CHECK(n32.rows == a.rows && n32.ids == a.ids && n32.order == a.order && n32.val == a.val);
  // the assembly ring reads the same stream, in the same order, through compact values
  const Sum rg = read_ring(files, 4, 3);
  CHECK(rg.rows == a.rows && rg.ids == a.ids && rg.order == a.order && rg.val == a.val && rg.lab == a.lab);
  // the raw-record ring (GPU-decode wire) ships the same records in the same order
  const Sum rr = read_ring_raw(files, 4, 3);
  CHECK(rr.rows == a.rows && rr.ids == a.ids && rr.order == a.order && rr.val == a.val && rr.lab == a.lab);
  // 2) record-level sharding partitions the data
  const Sum s0 = read_all(files, 3, 2, 0), s1 = read_all(files, 3, 2, 1);
  CHECK(s0.rows + s1.rows == want.rows && s0.ids + s1.ids == want.ids);

  // 3) CRC corruption is detected
  {
    FILE* f = fopen(files[0].c_str(), "rb");
    CHECK(f);
    std::vector<uint8_t> bytes;
    int c;
    while ((c = fgetc(f)) != EOF) bytes.push_back((uint8_t)c);
    fclose(f);
    bytes[bytes.size() / 2] ^= 0x5A;
    const std::string bad = dir + "/tr_selftest_bad.tfrecords";
    f = fopen(bad.c_str(), "wb");
    fwrite(bytes.data(), 1, bytes.size(), f);
    fclose(f);
    CHECK(hfmio_count_records(bad.c_str(), 0, 1) < 0);
    remove(bad.c_str());
  }

  // 4) libsvm -> TFRecord
  {
    const std::string src = dir + "/selftest.libsvm", dst = dir + "/selftest_conv.tfrecords";
    FILE* f = fopen(src.c_str(), "w");
    for (int i = 0; i < 100; ++i) {
      fprintf(f, "%d", i % 2);
      for (int k = 0; k < F; ++k) fprintf(f, " %d:%g", k * 10 + i % 10, k < 13 ? 0.5 : 1.0);
      fprintf(f, "\n");
    }
    fclose(f);
    CHECK(hfmio_libsvm_to_tfrecord(src.c_str(), dst.c_str(), F) == 100);
    CHECK(hfmio_count_records(dst.c_str(), 0, 1) == 100);
    CHECK(hfmio_count_records(src.c_str(), 1, 0) == 100);
    remove(src.c_str());
    remove(dst.c_str());
  }

  // 5) decoder robustness: truncations and random bytes (ASan flags any out-of-bounds read)
  {
    std::vector<float> lab(1), vals(F);
    std::vector<int64_t> ids(F);
    // a valid record to truncate
    FILE* f = fopen(files[1].c_str(), "rb");
    uint8_t hdr[12];
    CHECK(fread(hdr, 1, 12, f) == 12);
    uint64_t len;
    memcpy(&len, hdr, 8);
    std::vector<uint8_t> rec(len);
    CHECK(fread(rec.data(), 1, len, f) == len);
    fclose(f);
    CHECK(hfmio_decode_example(rec.data(), rec.size(), F, lab.data(), ids.data(), vals.data()) == 0);
    for (size_t cut = 0; cut < rec.size(); ++cut) {
      std::vector<uint8_t> t(rec.begin(), rec.begin() + cut);   // exact-size heap buffer
      (void)hfmio_decode_example(t.data(), t.size(), F, lab.data(), ids.data(), vals.data());
    }
    uint32_t x = 12345;
    for (int it = 0; it < 20000; ++it) {
      std::vector<uint8_t> t(1 + it % 200);
      for (auto& v : t) {
        x = x * 1664525u + 1013904223u;
        v = (uint8_t)(x >> 24);
      }
      (void)hfmio_decode_example(t.data(), t.size(), F, lab.data(), ids.data(), vals.data());
    }
    // CRC of a known vector (RFC 3720 test: 32 bytes of zeros -> 0x8A9136AA)
    std::vector<uint8_t> z(32, 0);
    CHECK(hfmio_crc32c(z.data(), z.size()) == 0x8A9136AAu);
  }
  for (auto& fl : files) remove(fl.c_str());
  printf("io_selftest ok\n");
  return 0;
}
