// hipfm host I/O runtime.
//
// Replaces the TensorFlow C++ input stack the reference relies on:
//   TFRecordDataset (record framing + CRC)           PS:108, HVD:93          -> TfRecordReader
//   tf.parse_example with FixedLenFeature schema     PS:79-92, HVD:76-89     -> decode_example
//   PipeModeDataset (SageMaker FIFO stream)           PS:111, HVD:105         -> same reader on a FIFO
//   shard / batch(drop_remainder) / prefetch          PS:113-128, HVD:95-128  -> Loader
// plus the libsvm text format (CONV:15-23, DOC p.42) and a fast TFRecord writer.
//
// Loader: W worker threads own files w, w+W, ... (file-level parallelism, each rank reads only
// its own files — SURVEY Q1), decode records straight into SoA chunks (label f32, ids i64[F],
// values f32[F]) and hand them over through bounded per-worker queues.  The consumer takes
// chunks round-robin over the workers (a deterministic interleave, like tf.data's
// interleave(deterministic=True)), so the batch sequence is reproducible for any thread
// timing.  Record-level sharding (dataset.shard(n, i), the reference's semantics) uses one
// sequential worker and keeps records with index % n == i.
//
// C ABI, bound with ctypes from hipfm/data/native_io.py.
#include <errno.h>
#include <fcntl.h>
#include <nmmintrin.h>
#include <stdint.h>
#include <unistd.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <functional>
#include <vector>

#define HFMIO_API extern "C" __attribute__((visibility("default")))

// ------------------------------------------------------------------------------ errors
static thread_local std::string g_err;
static void set_err(const std::string& s) { g_err = s; }
HFMIO_API const char* hfmio_last_error() { return g_err.c_str(); }

// ------------------------------------------------------------------------------ CRC32C
static uint32_t crc_table[256];
static bool crc_init = [] {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc_table[i] = c;
  }
  return true;
}();

static bool have_sse42() {
  static int v = -1;
  if (v < 0) v = __builtin_cpu_supports("sse4.2") ? 1 : 0;
  return v == 1;
}

__attribute__((target("sse4.2"))) static uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = crc ^ 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}

static uint32_t crc32c_sw(const uint8_t* p, size_t n, uint32_t crc) {
  uint32_t c = crc ^ 0xFFFFFFFFu;
  while (n--) c = crc_table[(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

HFMIO_API uint32_t hfmio_crc32c(const uint8_t* p, size_t n) {
  return have_sse42() ? crc32c_hw(p, n, 0) : crc32c_sw(p, n, 0);
}
HFMIO_API uint32_t hfmio_crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  return have_sse42() ? crc32c_hw(p, n, crc) : crc32c_sw(p, n, crc);
}
static inline uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }
HFMIO_API uint32_t hfmio_masked_crc32c(const uint8_t* p, size_t n) { return masked(hfmio_crc32c(p, n)); }

// ------------------------------------------------------------------------------ readers
class ByteReader {  // buffered sequential reader: files and FIFOs alike (no seeks)
 public:
  explicit ByteReader(const std::string& path) : path_(path) {
    f_ = fopen(path.c_str(), "rb");
    if (f_) setvbuf(f_, nullptr, _IOFBF, 1 << 22);
  }
  ~ByteReader() {
    if (f_) fclose(f_);
  }
  bool ok() const { return f_ != nullptr; }
  size_t read(void* dst, size_t n) { return fread(dst, 1, n, f_); }
  // line read for libsvm; returns false at EOF
  bool getline(std::string& out) {
    out.clear();
    int c;
    while ((c = fgetc(f_)) != EOF) {
      if (c == '\n') return true;
      out.push_back((char)c);
    }
    return !out.empty();
  }
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  FILE* f_ = nullptr;
};

// Block reader for the TFRecord framing: read(2) of 8 MB blocks, records parsed in place (the
// stdio path cost two locked fread calls and a copy per ~300-B record: 175-190 ns of the
// ~480 ns a record took on one thread, /tmp microbenchmark of a 1M-record Kaggle-shape file).
// Works on FIFOs (short reads are retried until the requested bytes or EOF).
class BlockReader {
 public:
  explicit BlockReader(const std::string& path) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ >= 0) posix_fadvise(fd_, 0, 0, POSIX_FADV_SEQUENTIAL);
    blk_.resize(8u << 20);
  }
  ~BlockReader() {
    if (fd_ >= 0) ::close(fd_);
  }
  bool ok() const { return fd_ >= 0; }
  const std::string& path() const { return path_; }
  // at least n bytes from the read position (nullptr: EOF or error first); `got` = bytes available
  const uint8_t* need(size_t n, size_t& got) {
    if (end_ - beg_ < n) {
      if (beg_ > 0) {  // compact
        memmove(blk_.data(), blk_.data() + beg_, end_ - beg_);
        end_ -= beg_;
        beg_ = 0;
      }
      if (n > blk_.size()) blk_.resize(n + (1u << 20));
      while (end_ < n && !eof_) {
        const ssize_t k = ::read(fd_, blk_.data() + end_, blk_.size() - end_);
        if (k < 0) {
          if (errno == EINTR) continue;
          eof_ = true;
          err_ = true;
          break;
        }
        if (k == 0) eof_ = true;
        end_ += (size_t)k;
      }
    }
    got = end_ - beg_;
    return got >= n ? blk_.data() + beg_ : nullptr;
  }
  void consume(size_t n) { beg_ += n; }
  bool io_error() const { return err_; }

 private:
  std::string path_;
  int fd_ = -1;
  std::vector<uint8_t> blk_;
  size_t beg_ = 0, end_ = 0;
  bool eof_ = false, err_ = false;
};

// One TFRecord, in place: rec / len point into the reader's block until the next call.
// returns 1 = record, 0 = clean EOF, -1 = error
// verify: 0 none, 1 length + data CRC, 2 length CRC only (the data CRC is checked on the GPU)
static int next_tfrecord_view(BlockReader& r, const uint8_t*& rec, uint64_t& len, int verify,
                              size_t& pending) {
  r.consume(pending);
  pending = 0;
  size_t got;
  const uint8_t* h = r.need(12, got);
  if (!h) {
    if (got == 0 && !r.io_error()) return 0;
    set_err((r.io_error() ? "read error in " : "truncated TFRecord header in ") + r.path());
    return -1;
  }
  memcpy(&len, h, 8);
  uint32_t hcrc;
  memcpy(&hcrc, h + 8, 4);
  if (verify && hcrc != masked(hfmio_crc32c(h, 8))) {
    set_err("TFRecord length CRC mismatch in " + r.path());
    return -1;
  }
  if (len > (1ull << 31)) {
    set_err("TFRecord too large in " + r.path());
    return -1;
  }
  const uint8_t* p = r.need(12 + len + 4, got);
  if (!p) {
    set_err("truncated TFRecord payload in " + r.path());
    return -1;
  }
  rec = p + 12;
  if (verify == 1) {
    uint32_t dcrc;
    memcpy(&dcrc, rec + len, 4);
    if (dcrc != masked(hfmio_crc32c(rec, len))) {
      set_err("TFRecord data CRC mismatch in " + r.path());
      return -1;
    }
  }
  pending = 12 + len + 4;
  return 1;
}

// returns 1 = record, 0 = clean EOF, -1 = error
static int next_tfrecord(ByteReader& r, std::vector<uint8_t>& buf, bool verify) {
  uint8_t hdr[12];
  size_t got = r.read(hdr, 12);
  if (got == 0) return 0;
  if (got < 12) {
    set_err("truncated TFRecord header in " + r.path());
    return -1;
  }
  uint64_t len;
  memcpy(&len, hdr, 8);
  uint32_t hcrc;
  memcpy(&hcrc, hdr + 8, 4);
  if (verify && hcrc != masked(hfmio_crc32c(hdr, 8))) {
    set_err("TFRecord length CRC mismatch in " + r.path());
    return -1;
  }
  if (len > (1ull << 31)) {
    set_err("TFRecord too large in " + r.path());
    return -1;
  }
  buf.resize(len + 4);
  if (r.read(buf.data(), len + 4) != len + 4) {
    set_err("truncated TFRecord payload in " + r.path());
    return -1;
  }
  if (verify) {
    uint32_t dcrc;
    memcpy(&dcrc, buf.data() + len, 4);
    if (dcrc != masked(hfmio_crc32c(buf.data(), len))) {
      set_err("TFRecord data CRC mismatch in " + r.path());
      return -1;
    }
  }
  buf.resize(len);
  return 1;
}

// ------------------------------------------------------------------------------ Example decode
static inline bool rd_varint(const uint8_t*& p, const uint8_t* e, uint64_t& v) {
  v = 0;
  int s = 0;
  while (p < e) {
    uint8_t c = *p++;
    v |= (uint64_t)(c & 0x7F) << s;
    if (!(c & 0x80)) return true;
    s += 7;
    if (s > 63) return false;
  }
  return false;
}

// true if [p, p + n) lies inside [p, e)  (length compare: no out-of-range pointer arithmetic,
// found by the UBSan self-test, csrc/io/io_selftest.cpp)
static inline bool fits(const uint8_t* p, const uint8_t* e, uint64_t n) {
  return n <= (uint64_t)(e - p);
}

static bool skip_field(const uint8_t*& p, const uint8_t* e, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return rd_varint(p, e, v);
    case 1: if (!fits(p, e, 8)) return false; p += 8; return true;
    case 2: if (!rd_varint(p, e, v) || !fits(p, e, v)) return false; p += v; return true;
    case 5: if (!fits(p, e, 4)) return false; p += 4; return true;
    default: return false;
  }
}

// decode FloatList / Int64List payload (packed or not) into dst; returns count or -1
static long decode_list(const uint8_t* p, const uint8_t* e, bool is_float, float* fdst,
                        int64_t* idst, long cap) {
  long n = 0;
  while (p < e) {
    uint64_t key;
    if (!rd_varint(p, e, key)) return -1;
    int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f != 1) {
      if (!skip_field(p, e, wt)) return -1;
      continue;
    }
    if (is_float) {
      if (wt == 2) {
        uint64_t ln;
        if (!rd_varint(p, e, ln) || !fits(p, e, ln)) return -1;
        long k = (long)(ln / 4);
        if (n + k > cap) return -2;
        memcpy(fdst + n, p, k * 4);
        n += k;
        p += ln;
      } else if (wt == 5) {
        if (!fits(p, e, 4)) return -1;
        if (n + 1 > cap) return -2;
        memcpy(fdst + n, p, 4);
        n++;
        p += 4;
      } else return -1;
    } else {
      if (wt == 2) {
        uint64_t ln;
        if (!rd_varint(p, e, ln) || !fits(p, e, ln)) return -1;
        const uint8_t* q = p;
        const uint8_t* qe = p + ln;
        while (q < qe) {
          uint64_t v;
          if (!rd_varint(q, qe, v)) return -1;
          if (n + 1 > cap) return -2;
          idst[n++] = (int64_t)v;
        }
        p = qe;
      } else if (wt == 0) {
        uint64_t v;
        if (!rd_varint(p, e, v)) return -1;
        if (n + 1 > cap) return -2;
        idst[n++] = (int64_t)v;
      } else return -1;
    }
  }
  return n;
}

// Fixed-schema decode of one serialized tf.train.Example (label f32[1], ids i64[F], values f32[F]).
static bool decode_example(const uint8_t* p, size_t len, int F, float* label, int64_t* ids,
                           float* vals) {
  const uint8_t* e = p + len;
  int have = 0;
  while (p < e) {
    uint64_t key;
    if (!rd_varint(p, e, key)) return false;
    if ((key >> 3) != 1 || (key & 7) != 2) {
      if (!skip_field(p, e, key & 7)) return false;
      continue;
    }
    uint64_t ln;
    if (!rd_varint(p, e, ln) || !fits(p, e, ln)) return false;
    const uint8_t* fp = p;           // Features
    const uint8_t* fe = p + ln;
    p = fe;
    while (fp < fe) {
      uint64_t k2;
      if (!rd_varint(fp, fe, k2)) return false;
      if ((k2 >> 3) != 1 || (k2 & 7) != 2) {
        if (!skip_field(fp, fe, k2 & 7)) return false;
        continue;
      }
      uint64_t l2;
      if (!rd_varint(fp, fe, l2) || !fits(fp, fe, l2)) return false;
      const uint8_t* mp = fp;        // map entry {key=1, value=2}
      const uint8_t* me = fp + l2;
      fp = me;
      const char* name = nullptr;
      size_t nlen = 0;
      const uint8_t* vp = nullptr;
      const uint8_t* ve = nullptr;
      while (mp < me) {
        uint64_t k3;
        if (!rd_varint(mp, me, k3)) return false;
        uint64_t l3;
        if ((k3 & 7) != 2) {
          if (!skip_field(mp, me, k3 & 7)) return false;
          continue;
        }
        if (!rd_varint(mp, me, l3) || !fits(mp, me, l3)) return false;
        if ((k3 >> 3) == 1) {
          name = (const char*)mp;
          nlen = l3;
        } else if ((k3 >> 3) == 2) {
          vp = mp;
          ve = mp + l3;
        }
        mp += l3;
      }
      if (!name || !vp) continue;
      // Feature { oneof bytes=1 float=2 int64=3 }
      const uint8_t* q = vp;
      uint64_t k4, l4;
      if (!rd_varint(q, ve, k4) || (k4 & 7) != 2 || !rd_varint(q, ve, l4) || !fits(q, ve, l4)) return false;
      const int kind = (int)(k4 >> 3);
      if (nlen == 5 && !memcmp(name, "label", 5) && kind == 2) {
        if (decode_list(q, q + l4, true, label, nullptr, 1) != 1) return false;
        have |= 1;
      } else if (nlen == 3 && !memcmp(name, "ids", 3) && kind == 3) {
        if (decode_list(q, q + l4, false, nullptr, ids, F) != F) return false;
        have |= 2;
      } else if (nlen == 6 && !memcmp(name, "values", 6) && kind == 2) {
        if (decode_list(q, q + l4, true, vals, nullptr, F) != F) return false;
        have |= 4;
      }
    }
  }
  return have == 7;
}

HFMIO_API int hfmio_decode_example(const uint8_t* p, size_t len, int F, float* label, int64_t* ids,
                                   float* vals) {
  return decode_example(p, len, F, label, ids, vals) ? 0 : -1;
}

// ------------------------------------------------------------------------------ libsvm
static bool parse_libsvm(const std::string& line, int F, float* label, int64_t* ids, float* vals) {
  const char* s = line.c_str();
  char* end;
  *label = strtof(s, &end);
  if (end == s) return false;
  s = end;
  int n = 0;
  while (*s) {
    while (*s == ' ' || *s == '\t' || *s == '\r') ++s;
    if (!*s) break;
    long long id = strtoll(s, &end, 10);
    if (end == s || *end != ':') return false;
    s = end + 1;
    float v = strtof(s, &end);
    if (end == s) return false;
    s = end;
    if (n >= F) return false;
    ids[n] = id;
    vals[n] = v;
    ++n;
  }
  return n == F;
}

// ------------------------------------------------------------------------------ loader
struct Chunk {
  int n = 0;
  std::vector<float> label;
  std::vector<int64_t> ids;     // (empty when the loader narrows at decode time: ids32)
  std::vector<int32_t> ids32;
  std::vector<float> vals;
  uint64_t vmask = 0;           // bit f: some row of the chunk has a field-f value other than 1.0
  // raw mode (Loader::raw): each record's serialized Example, decoded later on the GPU
  // (csrc/kernels/decode.hip).  Records of a mapped file stay in the mapping (rptr); records read
  // from a stream (FIFO) are copied into `raw` (rptr null, rcopy = offset); `maps` keeps the
  // mappings alive until the chunk has been assembled
  std::vector<uint8_t> raw;
  std::vector<const uint8_t*> rptr;
  std::vector<uint32_t> rcopy, rlen;
  std::vector<std::shared_ptr<struct Mapping>> maps;
  size_t rbytes = 0;            // sum of rlen
  void add_mapped(const uint8_t* p, uint32_t len) {
    rptr.push_back(p);
    rcopy.push_back(0);
    rlen.push_back(len);
    rbytes += len;
  }
  void add_copied(const uint8_t* p, uint32_t len) {
    rptr.push_back(nullptr);
    rcopy.push_back((uint32_t)raw.size());
    rlen.push_back(len);
    raw.insert(raw.end(), p, p + len);
    rbytes += len;
  }
  const uint8_t* rec(int i) const { return rptr[i] ? rptr[i] : raw.data() + rcopy[i]; }
};

// A read-only private mapping of a whole regular file (pre-faulted, sequential read-ahead).
struct Mapping {
  const uint8_t* p = nullptr;
  size_t n = 0;
  ~Mapping() {
    if (p) munmap((void*)p, n);
  }
};

struct WorkerQueue {
  std::mutex m;
  std::condition_variable cv_put, cv_get;
  std::deque<std::unique_ptr<Chunk>> q;
  bool done = false;
  bool failed = false;
  std::string err;
};

// Parallel copy of one batch's chunk pieces into the caller's (pinned) buffers: a batch is 16+
// pieces (1024-record chunks), each memcpy'd / narrowed by whichever pool thread takes it.  The
// single consumer thread copying 5-10 MB per batch capped ingest below the decode workers' rate.
class CopyPool {
 public:
  explicit CopyPool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size(); }
  // run f(0..n-1) on the pool and the calling thread; returns when every call finished
  void run(int n, std::function<void(int)> f) {
    auto job = std::make_shared<Job>();
    job->f = std::move(f);
    job->n = n;
    {
      std::lock_guard<std::mutex> lk(m_);
      cur_ = job;
      ++gen_;
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> lk(job->m);
    job->cv.wait(lk, [&] { return job->done == job->n; });
  }

 private:
  struct Job {
    std::function<void(int)> f;
    int n = 0;
    std::atomic<int> next{0};
    std::mutex m;
    std::condition_variable cv;
    int done = 0;
  };
  static void work(Job& j) {
    int i;
    while ((i = j.next.fetch_add(1)) < j.n) {
      j.f(i);
      std::lock_guard<std::mutex> lk(j.m);
      if (++j.done == j.n) j.cv.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        j = cur_;
      }
      work(*j);   // (a job this thread joins late just finds its pieces taken)
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::shared_ptr<Job> cur_;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

struct Loader {
  std::vector<std::string> paths;
  int format = 0, F = 0, B = 0, drop_remainder = 1, verify = 1;
  int shard_n = 1, shard_i = 0;   // record-level shard (1 = off)
  int64_t id_limit = 0;            // > 0: every id must lie in [0, id_limit) (feature_size V)
  int raw = 0;                     // workers only frame + CRC-check TFRecords and keep the Example
                                   // bytes; batches ship raw records + offsets (next_raw)
  int narrow32 = 0;                // workers narrow ids to int32 while decoding (the device id type):
                                   // batch assembly is then a plain copy (it was the ingest bound)
  int depth = 4;
  int chunk = 1024;
  std::vector<std::unique_ptr<WorkerQueue>> queues;
  std::vector<std::thread> threads;
  std::atomic<bool> stop{false};
  // consumer state
  int turn = 0;
  std::unique_ptr<Chunk> cur;
  int cur_off = 0;
  std::string err;
  std::unique_ptr<CopyPool> pool;            // parallel batch assembly (null: the consumer copies)

  // Assembly ring (start_ring): an assembler thread fills caller-registered (pinned) buffers in
  // cyclic slot order ahead of the consumer, so batch i+1 is assembled while the consumer issues
  // batch i's device copy (with next() the assembly and the caller's per-batch work alternate on
  // one thread: the streamed epochs ran at ~65 % of the loader's own rate).  take() returns the
  // slots in order; give() hands one back once the caller is done with its contents.
  struct Ring {
    int n = 0;
    bool compact = false;
    std::vector<float*> lab, vals;
    std::vector<int32_t*> ids;
    std::vector<uint8_t*> rawb;  // raw mode: record bytes + offsets per slot, `cap` bytes each
    std::vector<uint32_t*> offs;
    size_t cap = 0;
    std::vector<int> state;      // 0 free, 1 assembling, 2 assembled
    std::vector<int> rows;
    std::vector<uint64_t> mask;
    std::deque<int> ready;
    int fill = 0;                // next slot the assembler fills
    std::mutex m;
    std::condition_variable cv_free, cv_ready;
    std::thread th;
  } ring;

  void assemble_loop() {
    Ring& R = ring;
    for (;;) {
      int s;
      {
        std::unique_lock<std::mutex> lk(R.m);
        R.cv_free.wait(lk, [&] { return stop.load() || R.state[R.fill] == 0; });
        if (stop.load()) return;
        s = R.fill;
        R.state[s] = 1;
        R.fill = (s + 1) % R.n;
      }
      uint64_t mk = 0;
      const int r = raw ? next_raw(R.rawb[s], R.cap, R.offs[s], &mk)
                        : next(R.lab[s], nullptr, R.vals[s], R.ids[s], R.compact ? &mk : nullptr);
      {
        std::lock_guard<std::mutex> lk(R.m);
        R.rows[s] = r;
        R.mask[s] = mk;
        R.state[s] = 2;
        R.ready.push_back(s);
      }
      R.cv_ready.notify_all();
      if (r <= 0) return;        // end of data (0) or error (-1, err holds it): the last slot says so
    }
  }

  // raw mode: slot s receives up to `cap` record bytes in rawb[s] and B + 1 offsets in offs[s];
  // ring_take's mask then returns the slot's byte count
  int start_ring_raw(int n, uint8_t** rawb, size_t cap, uint32_t** offs) {
    if (!raw || ring.n || n < 2) return -1;
    ring.rawb.assign(rawb, rawb + n);
    ring.offs.assign(offs, offs + n);
    ring.cap = cap;
    ring.n = n;
    ring.state.assign(n, 0);
    ring.rows.assign(n, 0);
    ring.mask.assign(n, 0);
    ring.th = std::thread(&Loader::assemble_loop, this);
    return 0;
  }

  int start_ring(int n, float** lab, int32_t** ids, float** vals, int compact) {
    if (raw || ring.n || n < 2 || (compact && F > 64)) return -1;
    ring.n = n;
    ring.compact = compact != 0;
    ring.lab.assign(lab, lab + n);
    ring.ids.assign(ids, ids + n);
    ring.vals.assign(vals, vals + n);
    ring.state.assign(n, 0);
    ring.rows.assign(n, 0);
    ring.mask.assign(n, 0);
    ring.th = std::thread(&Loader::assemble_loop, this);
    return 0;
  }

  // next assembled slot in order: rows (B, fewer for a final partial batch, 0 at end, -1 error)
  int ring_take(int* slot, uint64_t* mask) {
    std::unique_lock<std::mutex> lk(ring.m);
    ring.cv_ready.wait(lk, [&] { return !ring.ready.empty() || stop.load(); });
    if (ring.ready.empty()) return 0;
    const int s = ring.ready.front();
    const int r = ring.rows[s];
    if (r > 0) ring.ready.pop_front();   // (the end / error slot stays: every later take sees it)
    *slot = s;
    *mask = ring.mask[s];
    return r;
  }

  void ring_give(int slot) {
    {
      std::lock_guard<std::mutex> lk(ring.m);
      if (slot >= 0 && slot < ring.n && ring.state[slot] == 2) ring.state[slot] = 0;
    }
    ring.cv_free.notify_all();
  }

  // Chunk recycling: a chunk's buffers (160-512 KB each) come from a free list instead of a fresh
  // allocation per 1024 records -- glibc serves such sizes with mmap, so every chunk paid ~128 page
  // faults on first touch and a munmap at free (~125 ns per record: a lone worker managed ~5 M
  // records/s whatever the record format).
  std::mutex pool_m;
  std::vector<std::unique_ptr<Chunk>> pool_free;

  std::unique_ptr<Chunk> get_chunk() {
    std::unique_ptr<Chunk> c;
    {
      std::lock_guard<std::mutex> lk(pool_m);
      if (!pool_free.empty()) {
        c = std::move(pool_free.back());
        pool_free.pop_back();
      }
    }
    if (!c) {
      c = std::make_unique<Chunk>();
      if (raw) {
        c->rptr.reserve(chunk);
        c->rcopy.reserve(chunk);
        c->rlen.reserve(chunk);
      } else {
        c->label.resize(chunk);
        if (narrow32) c->ids32.resize((size_t)chunk * F);
        else c->ids.resize((size_t)chunk * F);
        c->vals.resize((size_t)chunk * F);
      }
    }
    c->n = 0;
    c->vmask = 0;
    if (raw) {
      c->raw.clear();                    // (vectors keep their capacity)
      c->rptr.clear();
      c->rcopy.clear();
      c->rlen.clear();
      c->maps.clear();
      c->rbytes = 0;
    }
    return c;
  }

  void put_chunk(std::unique_ptr<Chunk> c) {
    if (!c) return;
    c->maps.clear();                     // (the last chunk of a file unmaps it)
    std::lock_guard<std::mutex> lk(pool_m);
    if (pool_free.size() < 512) pool_free.push_back(std::move(c));
  }

  struct Recycle {                       // chunks an assembly finished with go back to the pool
    Loader* L;
    std::vector<std::unique_ptr<Chunk>> v;
    ~Recycle() {
      for (auto& c : v) L->put_chunk(std::move(c));
    }
  };

  // raw mode, one regular file: mapped once; framing + CRC in place, each chunk records where its
  // payloads lie in the mapping -- the only copy of a record's bytes on the host is the assembly
  // into the caller's pinned slot (read(2) into a block, a copy into the chunk and the assembly
  // moved every byte three times)
  template <class Push, class Fresh, class Fail>
  int worker_raw_mapped(const std::string& path, std::unique_ptr<Chunk>& c, long long& rec, Push& push,
                        Fresh& fresh, Fail& fail) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return -1;                              // (the caller reports it)
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
      ::close(fd);
      return 0;                                         // not a regular file: stream it instead
    }
    auto m = std::make_shared<Mapping>();
    m->n = (size_t)st.st_size;
    if (m->n > 0) {
      void* a = mmap(nullptr, m->n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (a == MAP_FAILED) {
        ::close(fd);
        return 0;
      }
      madvise(a, m->n, MADV_SEQUENTIAL);
      m->p = (const uint8_t*)a;
    }
    ::close(fd);
    const uint8_t* p = m->p;
    size_t at = 0;
    while (at < m->n && !stop.load()) {
      if (m->n - at < 12) {
        fail("truncated TFRecord header in " + path);
        return -2;
      }
      uint64_t len;
      memcpy(&len, p + at, 8);
      uint32_t hcrc;
      memcpy(&hcrc, p + at + 8, 4);
      if (verify && hcrc != masked(hfmio_crc32c(p + at, 8))) {
        fail("TFRecord length CRC mismatch in " + path);
        return -2;
      }
      if (len > (1ull << 31) || m->n - at - 12 < len + 4) {
        fail("truncated TFRecord payload in " + path);
        return -2;
      }
      const uint8_t* rp = p + at + 12;
      if (verify == 1) {
        uint32_t dcrc;
        memcpy(&dcrc, rp + len, 4);
        if (dcrc != masked(hfmio_crc32c(rp, len))) {
          fail("TFRecord data CRC mismatch in " + path);
          return -2;
        }
      }
      at += 12 + len + 4;
      if (shard_n > 1 && (rec++ % shard_n) != shard_i) continue;
      if (c->maps.empty() || c->maps.back() != m) c->maps.push_back(m);   // (a chunk may span files)
      // verify 2: the record travels with its 4-byte masked data CRC (the decode kernel checks it)
      c->add_mapped(rp, (uint32_t)len + (verify == 2 ? 4u : 0u));
      if (++c->n == chunk) {
        if (!push(std::move(c))) return -2;
        c = fresh();
      }
    }
    return 1;
  }

  // raw mode, one file: framing + CRC only, the Example bytes appended to the chunk
  template <class Push, class Fresh, class Fail>
  bool worker_raw_file(const std::string& path, std::unique_ptr<Chunk>& c, long long& rec, Push& push,
                       Fresh& fresh, Fail& fail) {
    const int mr = worker_raw_mapped(path, c, rec, push, fresh, fail);
    if (mr == 1) return true;
    if (mr == -2) return false;
    BlockReader br(path);
    if (!br.ok()) {
      fail("cannot open " + path);
      return false;
    }
    size_t pending = 0;
    while (!stop.load()) {
      const uint8_t* rp;
      uint64_t rlen;
      const int rc = next_tfrecord_view(br, rp, rlen, verify, pending);
      if (rc == 0) break;
      if (rc < 0) {
        fail(g_err);
        return false;
      }
      if (shard_n > 1 && (rec++ % shard_n) != shard_i) continue;
      const uint64_t rl = rlen + (verify == 2 ? 4u : 0u);   // (+ the data CRC: contiguous in the view)
      if (c->raw.size() + rl > 0xFFFFFFFFull) {
        fail("raw chunk exceeds 4 GB in " + path);
        return false;
      }
      c->add_copied(rp, (uint32_t)rl);
      if (++c->n == chunk) {
        if (!push(std::move(c))) return false;
        c = fresh();
      }
    }
    return true;
  }

  void worker(int w, int W) {
    WorkerQueue& Q = *queues[w];
    auto push = [&](std::unique_ptr<Chunk> c) {
      std::unique_lock<std::mutex> lk(Q.m);
      Q.cv_put.wait(lk, [&] { return (int)Q.q.size() < depth || stop.load(); });
      if (stop.load()) return false;
      Q.q.push_back(std::move(c));
      Q.cv_get.notify_one();
      return true;
    };
    auto fail = [&](const std::string& e) {
      std::lock_guard<std::mutex> lk(Q.m);
      Q.failed = true;
      Q.err = e;
      Q.done = true;
      Q.cv_get.notify_all();
    };
    auto fresh = [&] { return get_chunk(); };
    std::vector<int64_t> idrow((size_t)F);   // one record's ids before narrowing
    std::unique_ptr<Chunk> c = fresh();
    std::string line;
    long long rec = 0;   // record index in this worker's stream (record sharding uses W == 1)
    for (size_t fi = w; fi < paths.size() && !stop.load(); fi += W) {
      if (raw) {
        if (!worker_raw_file(paths[fi], c, rec, push, fresh, fail)) return;
        continue;
      }
      std::unique_ptr<ByteReader> lr;       // libsvm lines
      std::unique_ptr<BlockReader> br;      // TFRecords, parsed in place
      if (format == 0) br = std::make_unique<BlockReader>(paths[fi]);
      else lr = std::make_unique<ByteReader>(paths[fi]);
      if (format == 0 ? !br->ok() : !lr->ok()) {
        fail("cannot open " + paths[fi]);
        return;
      }
      size_t pending = 0;
      long long frec = -1;   // record index within this file (every record, sharded or not)
      while (!stop.load()) {
        float* lab = c->label.data() + c->n;
        int64_t* ids = narrow32 ? idrow.data() : c->ids.data() + (size_t)c->n * F;
        float* vals = c->vals.data() + (size_t)c->n * F;
        bool okrec;
        if (format == 0) {
          const uint8_t* rp;
          uint64_t rlen;
          int rc = next_tfrecord_view(*br, rp, rlen, verify, pending);
          if (rc == 0) break;
          if (rc < 0) {
            fail(g_err);
            return;
          }
          ++frec;
          if (shard_n > 1 && (rec++ % shard_n) != shard_i) continue;
          okrec = decode_example(rp, rlen, F, lab, ids, vals);
          if (!okrec) {
            fail("Example does not match the fixed schema (label, ids[F], values[F]) in " + paths[fi]);
            return;
          }
        } else {
          if (!lr->getline(line)) break;
          if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
          ++frec;
          if (shard_n > 1 && (rec++ % shard_n) != shard_i) continue;
          if (!parse_libsvm(line, F, lab, ids, vals)) {
            fail("bad libsvm line (expected label + " + std::to_string(F) + " id:val) in " + paths[fi]);
            return;
          }
        }
        if (id_limit > 0) {
          // the device gathers / updates table rows by id unchecked: reject out-of-vocabulary
          // ids here, where the file and record are known (TF's CPU gather raises likewise)
          for (int f = 0; f < F; ++f) {
            if (ids[f] < 0 || ids[f] >= id_limit) {
              fail("feature id " + std::to_string((long long)ids[f]) + " (field " + std::to_string(f) +
                   ") outside [0, feature_size=" + std::to_string((long long)id_limit) + ") in " +
                   paths[fi] + " record " + std::to_string(frec));
              return;
            }
          }
        }
        if (F <= 64) {
          // per-chunk mask of the fields whose values are not all exactly 1.0 (bit pattern, so
          // -0 / NaN / denormals count as values): the compact wire format ships only those columns
          uint64_t m = 0;
          for (int f = 0; f < F; ++f) {
            uint32_t u;
            memcpy(&u, vals + f, 4);
            m |= (uint64_t)(u != 0x3F800000u) << f;
          }
          c->vmask |= m;
        }
        if (narrow32) {
          int32_t* d = c->ids32.data() + (size_t)c->n * F;
          for (int f = 0; f < F; ++f) {
            if (ids[f] < 0 || ids[f] > 0x7FFFFFFF) {
              fail("feature id " + std::to_string((long long)ids[f]) + " outside [0, 2^31) for the int32 "
                   "device path in " + paths[fi] + " record " + std::to_string(frec));
              return;
            }
            d[f] = (int32_t)ids[f];
          }
        }
        if (++c->n == chunk) {
          if (!push(std::move(c))) return;
          c = fresh();
        }
      }
    }
    if (c->n > 0) push(std::move(c));
    std::lock_guard<std::mutex> lk(Q.m);
    Q.done = true;
    Q.cv_get.notify_all();
  }

  // next chunk in deterministic round-robin order; nullptr at end
  std::unique_ptr<Chunk> take() {
    const int W = (int)queues.size();
    int idle = 0;
    while (idle < W) {
      WorkerQueue& Q = *queues[turn];
      std::unique_lock<std::mutex> lk(Q.m);
      Q.cv_get.wait(lk, [&] { return !Q.q.empty() || Q.done || stop.load(); });
      if (Q.q.empty() && !Q.done) return nullptr;   // shutting down (a stopped worker never sets done)
      if (Q.failed) {
        err = Q.err;
        return nullptr;
      }
      if (!Q.q.empty()) {
        auto c = std::move(Q.q.front());
        Q.q.pop_front();
        Q.cv_put.notify_one();
        turn = (turn + 1) % W;
        return c;
      }
      // this worker is exhausted; skip it for good
      ++idle;
      turn = (turn + 1) % W;
    }
    return nullptr;
  }

  // returns rows written (B, or < B for the final partial batch), 0 at end, -1 error.
  // ids32 != null: ids are narrowed to int32 (the device id type) while copying, straight into
  // the caller's (pinned) buffer; an id outside [0, 2^31) is an error.  The batch is assembled
  // from pieces (chunk, chunk row, batch row, rows) copied in parallel by the copy pool.
  // vmask != null: compact values -- only the columns of the fields whose values are not all
  // 1.0 in the batch's chunks (mask returned in *vmask, bit f = field f shipped; columns in field
  // order, ``vals`` then holds [rows, popcount(mask)]).  Requires F <= 64.  Lossless: the omitted
  // columns are exactly 1.0f in every row of the batch.
  // Raw mode batch: up to B records' Example bytes back to back into `dst` (at most `cap` bytes)
  // and their B + 1 start offsets into `offs` (offs[rows] = total bytes, also in *bytes).  Returns
  // rows as next() does.  The copy pool assembles the pieces in parallel.
  int next_raw(uint8_t* dst, size_t cap, uint32_t* offs, uint64_t* bytes) {
    struct Piece {
      const Chunk* c;
      int src, dst, k;
      size_t at;
    };
    std::vector<Piece> pieces;
    Recycle done{this, {}};
    int got = 0;
    size_t total = 0;
    while (got < B) {
      if (!cur || cur_off >= cur->n) {
        if (cur) done.v.push_back(std::move(cur));
        cur = take();
        cur_off = 0;
        if (!cur) {
          if (stop.load() && err.empty()) err = "loader stopped";
          if (!err.empty()) return -1;
          break;
        }
      }
      const int k = std::min(B - got, cur->n - cur_off);
      pieces.push_back({cur.get(), cur_off, got, k, total});
      for (int i = 0; i < k; ++i) total += cur->rlen[cur_off + i];
      got += k;
      cur_off += k;
    }
    if (got < B && drop_remainder) return 0;
    if (total > cap || total > 0xFFFFFFFFull) {
      err = "raw batch of " + std::to_string(total) + " bytes exceeds the " + std::to_string(cap) +
            "-byte staging buffer";
      return -1;
    }
    auto copy = [&](int pi) {
      const Piece& p = pieces[pi];
      size_t at = p.at;
      for (int i = 0; i < p.k; ++i) {
        const uint32_t n = p.c->rlen[p.src + i];
        memcpy(dst + at, p.c->rec(p.src + i), n);
        offs[p.dst + i] = (uint32_t)at;
        at += n;
      }
    };
    if (pool && pieces.size() > 1) {
      pool->run((int)pieces.size(), copy);
    } else {
      for (int i = 0; i < (int)pieces.size(); ++i) copy(i);
    }
    offs[got] = (uint32_t)total;
    *bytes = total;
    return got;
  }

  int next(float* lab, int64_t* ids, float* vals, int32_t* ids32 = nullptr, uint64_t* vmask = nullptr) {
    struct Piece {
      const Chunk* c;
      int src, dst, k;
    };
    std::vector<Piece> pieces;
    Recycle done{this, {}};
    int got = 0;
    while (got < B) {
      if (!cur || cur_off >= cur->n) {
        if (cur) done.v.push_back(std::move(cur));
        cur = take();
        cur_off = 0;
        if (!cur) {
          // (a shutdown is not the end of the data: never publish a batch it cut short)
          if (stop.load() && err.empty()) err = "loader stopped";
          if (!err.empty()) return -1;
          break;
        }
      }
      int k = std::min(B - got, cur->n - cur_off);
      pieces.push_back({cur.get(), cur_off, got, k});
      got += k;
      cur_off += k;
    }
    if (got < B && drop_remainder) return 0;
    int cols[64];
    int nc = F;
    if (vmask) {
      if (F > 64) {
        err = "compact values need F <= 64 fields";
        return -1;
      }
      uint64_t m = 0;
      for (const Piece& p : pieces) m |= p.c->vmask;
      nc = 0;
      for (int f = 0; f < F; ++f)
        if ((m >> f) & 1) cols[nc++] = f;
      *vmask = m;
    }
    std::atomic<int64_t> bad{0};
    auto copy = [&](int pi) {
      const Piece& p = pieces[pi];
      memcpy(lab + p.dst, p.c->label.data() + p.src, p.k * 4);
      const size_t m = (size_t)p.k * F;
      if (ids32 && !p.c->ids32.empty()) {
        memcpy(ids32 + (size_t)p.dst * F, p.c->ids32.data() + (size_t)p.src * F, m * 4);
      } else if (ids32) {
        const int64_t* src = p.c->ids.data() + (size_t)p.src * F;
        int32_t* dst = ids32 + (size_t)p.dst * F;
        int64_t b = 0;
        for (size_t i = 0; i < m; ++i) {
          const int64_t v = src[i];
          b |= v >> 31;  // non-zero for negatives and ids >= 2^31
          dst[i] = (int32_t)v;
        }
        if (b) bad.store(1);
      } else if (p.c->ids.empty()) {  // narrowed at decode, read back as int64
        const int32_t* src = p.c->ids32.data() + (size_t)p.src * F;
        int64_t* dst = ids + (size_t)p.dst * F;
        for (size_t i = 0; i < m; ++i) dst[i] = src[i];
      } else {
        memcpy(ids + (size_t)p.dst * F, p.c->ids.data() + (size_t)p.src * F, m * 8);
      }
      if (nc == F) {
        memcpy(vals + (size_t)p.dst * F, p.c->vals.data() + (size_t)p.src * F, m * 4);
      } else {
        const float* src = p.c->vals.data() + (size_t)p.src * F;
        float* dst = vals + (size_t)p.dst * nc;
        for (int i = 0; i < p.k; ++i, src += F, dst += nc)
          for (int j = 0; j < nc; ++j) dst[j] = src[cols[j]];
      }
    };
    if (pool && pieces.size() > 1) {
      pool->run((int)pieces.size(), copy);
    } else {
      for (int i = 0; i < (int)pieces.size(); ++i) copy(i);
    }
    if (bad.load()) {
      err = "feature id outside [0, 2^31) for the int32 device path";
      return -1;
    }
    return got;
  }

  void shutdown() {
    stop.store(true);
    for (auto& q : queues) {
      std::lock_guard<std::mutex> lk(q->m);
      q->cv_put.notify_all();
      q->cv_get.notify_all();
    }
    {
      std::lock_guard<std::mutex> lk(ring.m);
      ring.cv_free.notify_all();
      ring.cv_ready.notify_all();
    }
    if (ring.th.joinable()) ring.th.join();
    for (auto& t : threads)
      if (t.joinable()) t.join();
  }
};

HFMIO_API void* hfmio_loader_create(const char** paths, int npaths, int format, int F, int batch,
                                    int drop_remainder, int num_threads, int shard_n, int shard_i,
                                    int verify_crc, int queue_depth, int64_t id_limit, int narrow32) {
  auto* L = new Loader();
  L->id_limit = id_limit;
  L->narrow32 = narrow32 ? 1 : 0;
  for (int i = 0; i < npaths; ++i) L->paths.emplace_back(paths[i]);
  L->format = format;
  L->F = F;
  L->B = batch;
  L->drop_remainder = drop_remainder;
  L->verify = verify_crc ? 1 : 0;        // (2 = device-side data CRC: raw loaders only)
  L->shard_n = shard_n < 1 ? 1 : shard_n;
  L->shard_i = shard_i;
  L->depth = queue_depth < 1 ? 4 : queue_depth;
  int W = num_threads < 1 ? 1 : num_threads;
  if (L->shard_n > 1) W = 1;                 // record-level shard needs the sequential stream
  if (W > npaths) W = npaths < 1 ? 1 : npaths;
  for (int w = 0; w < W; ++w) L->queues.emplace_back(new WorkerQueue());
  for (int w = 0; w < W; ++w) L->threads.emplace_back(&Loader::worker, L, w, W);
  return L;
}

// Raw-record loader (TFRecord only): workers frame + CRC-check, batches carry the serialized
// Examples + offsets for the GPU decoder (csrc/kernels/decode.hip); ids are checked there.
HFMIO_API void* hfmio_loader_create_raw(const char** paths, int npaths, int F, int batch, int drop_remainder,
                                        int num_threads, int shard_n, int shard_i, int verify_crc,
                                        int queue_depth) {
  auto* L = new Loader();
  L->raw = 1;
  for (int i = 0; i < npaths; ++i) L->paths.emplace_back(paths[i]);
  L->format = 0;
  L->F = F;
  L->B = batch;
  L->drop_remainder = drop_remainder;
  // 2: the length CRC here, the data CRC on the GPU (each record shipped with its 4 CRC bytes)
  L->verify = verify_crc == 2 ? 2 : (verify_crc ? 1 : 0);
  L->shard_n = shard_n < 1 ? 1 : shard_n;
  L->shard_i = shard_i;
  L->depth = queue_depth < 1 ? 4 : queue_depth;
  int W = num_threads < 1 ? 1 : num_threads;
  if (L->shard_n > 1) W = 1;
  if (W > npaths) W = npaths < 1 ? 1 : npaths;
  for (int w = 0; w < W; ++w) L->queues.emplace_back(new WorkerQueue());
  for (int w = 0; w < W; ++w) L->threads.emplace_back(&Loader::worker, L, w, W);
  return L;
}

HFMIO_API int hfmio_loader_next_raw(void* h, uint8_t* dst, size_t cap, uint32_t* offs, uint64_t* bytes) {
  auto* L = (Loader*)h;
  if (!L->raw) {
    set_err("next_raw on a decoding loader");
    return -1;
  }
  int r = L->next_raw(dst, cap, offs, bytes);
  if (r < 0) set_err(L->err);
  return r;
}

HFMIO_API int hfmio_loader_start_ring_raw(void* h, int n, uint8_t** rawb, size_t cap, uint32_t** offs) {
  auto* L = (Loader*)h;
  int r = L->start_ring_raw(n, rawb, cap, offs);
  if (r < 0) set_err("raw assembly ring: a raw loader, >= 2 slots, once per loader");
  return r;
}

HFMIO_API int hfmio_loader_next(void* h, float* labels, int64_t* ids, float* vals) {
  auto* L = (Loader*)h;
  int r = L->next(labels, ids, vals);
  if (r < 0) set_err(L->err);
  return r;
}

HFMIO_API int hfmio_loader_next32(void* h, float* labels, int32_t* ids, float* vals) {
  auto* L = (Loader*)h;
  int r = L->next(labels, nullptr, vals, ids);
  if (r < 0) set_err(L->err);
  return r;
}

// next32 with compact values (Loader::next): vals_c gets [rows, popcount(*mask)] floats.
HFMIO_API int hfmio_loader_next32c(void* h, float* labels, int32_t* ids, float* vals_c, uint64_t* mask) {
  auto* L = (Loader*)h;
  int r = L->next(labels, nullptr, vals_c, ids, mask);
  if (r < 0) set_err(L->err);
  return r;
}

// Assembly ring over n caller buffers (Loader::start_ring); vals[i] receives [B, nc] compact
// columns when compact != 0 (hfmio_loader_next32c), else [B, F].  Ids are int32.
HFMIO_API int hfmio_loader_start_ring(void* h, int n, float** labels, int32_t** ids, float** vals, int compact) {
  auto* L = (Loader*)h;
  int r = L->start_ring(n, labels, ids, vals, compact);
  if (r < 0) set_err("assembly ring: needs >= 2 slots, once per loader (compact: F <= 64)");
  return r;
}
HFMIO_API int hfmio_loader_ring_take(void* h, int* slot, uint64_t* mask) {
  auto* L = (Loader*)h;
  int r = L->ring_take(slot, mask);
  if (r < 0) set_err(L->err);
  return r;
}
HFMIO_API void hfmio_loader_ring_give(void* h, int slot) { ((Loader*)h)->ring_give(slot); }

// Assemble batches with n copy threads (the consumer plus n - 1 pool threads); 1: serial.
HFMIO_API void hfmio_loader_set_copy_threads(void* h, int n) {
  auto* L = (Loader*)h;
  L->pool.reset(n > 1 ? new CopyPool(n - 1) : nullptr);
}

HFMIO_API void hfmio_loader_destroy(void* h) {
  auto* L = (Loader*)h;
  L->shutdown();
  delete L;
}

// ------------------------------------------------------------------------------ writers
static void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
static void put_ld(std::string& s, int field, const std::string& payload) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, payload.size());
  s += payload;
}

static std::string encode_example(float label, const int64_t* ids, const float* vals, int F) {
  std::string fl;
  put_ld(fl, 1, std::string((const char*)&label, 4));
  std::string flab;
  put_ld(flab, 2, fl);
  std::string packed_ids;
  for (int i = 0; i < F; ++i) put_varint(packed_ids, (uint64_t)ids[i]);
  std::string il;
  put_ld(il, 1, packed_ids);
  std::string fids;
  put_ld(fids, 3, il);
  std::string vl;
  put_ld(vl, 1, std::string((const char*)vals, (size_t)F * 4));
  std::string fvals;
  put_ld(fvals, 2, vl);
  std::string entries;
  auto entry = [&](const char* k, const std::string& v) {
    std::string e;
    put_ld(e, 1, std::string(k));
    put_ld(e, 2, v);
    put_ld(entries, 1, e);
  };
  entry("label", flab);
  entry("ids", fids);
  entry("values", fvals);
  std::string ex;
  put_ld(ex, 1, entries);
  return ex;
}

static bool write_record(FILE* f, const std::string& d) {
  uint64_t len = d.size();
  uint32_t hc = masked(hfmio_crc32c((const uint8_t*)&len, 8));
  uint32_t dc = masked(hfmio_crc32c((const uint8_t*)d.data(), d.size()));
  return fwrite(&len, 8, 1, f) == 1 && fwrite(&hc, 4, 1, f) == 1 &&
         fwrite(d.data(), 1, d.size(), f) == d.size() && fwrite(&dc, 4, 1, f) == 1;
}

HFMIO_API int hfmio_write_examples(const char* path, const float* labels, const int64_t* ids,
                                   const float* vals, long n, int F, int append) {
  FILE* f = fopen(path, append ? "ab" : "wb");
  if (!f) {
    set_err(std::string("cannot open ") + path);
    return -1;
  }
  for (long i = 0; i < n; ++i)
    if (!write_record(f, encode_example(labels[i], ids + (size_t)i * F, vals + (size_t)i * F, F))) {
      fclose(f);
      set_err("write failed");
      return -1;
    }
  fclose(f);
  return 0;
}

// native libsvm -> TFRecord converter (C36); returns records written or -1
HFMIO_API long hfmio_libsvm_to_tfrecord(const char* src, const char* dst, int F) {
  ByteReader r(src);
  if (!r.ok()) {
    set_err(std::string("cannot open ") + src);
    return -1;
  }
  FILE* f = fopen(dst, "wb");
  if (!f) {
    set_err(std::string("cannot open ") + dst);
    return -1;
  }
  std::string line;
  std::vector<int64_t> ids(F);
  std::vector<float> vals(F);
  long n = 0;
  while (r.getline(line)) {
    if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
    float lab;
    if (!parse_libsvm(line, F, &lab, ids.data(), vals.data())) {
      set_err("bad libsvm line " + std::to_string(n + 1));
      fclose(f);
      return -1;
    }
    write_record(f, encode_example(lab, ids.data(), vals.data(), F));
    ++n;
  }
  fclose(f);
  return n;
}

HFMIO_API long hfmio_count_records(const char* path, int format, int verify) {
  ByteReader r(path);
  if (!r.ok()) {
    set_err(std::string("cannot open ") + path);
    return -1;
  }
  long n = 0;
  if (format == 0) {
    std::vector<uint8_t> buf;
    int rc;
    while ((rc = next_tfrecord(r, buf, verify)) == 1) ++n;
    return rc < 0 ? -1 : n;
  }
  std::string line;
  while (r.getline(line))
    if (line.find_first_not_of(" \t\r") != std::string::npos) ++n;
  return n;
}
