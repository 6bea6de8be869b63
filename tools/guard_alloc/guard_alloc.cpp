// Guard-zone device allocator for torch.cuda.memory.CUDAPluggableAllocator (GPU AddressSanitizer
// is not available on this pool): every allocation gets GUARD bytes before and after it, and the
// allocation itself, filled with a byte pattern.  A kernel that reads past a buffer sees the
// pattern (NaN for fp32 / bf16, -1 for int32 with 0xFF) instead of a neighbour's data; a kernel
// that writes past it is reported when the buffer is freed (guard bytes compared on the host).
//
// Build: hipcc --offload-arch=gfx950 -O2 -fPIC -shared tools/guard_alloc/guard_alloc.cpp -o
//        tools/guard_alloc/libguard_alloc.so
// Env:   HFM_GUARD_BYTES (default 65536), HFM_GUARD_FILL (default 255)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace {
size_t guard_bytes() {
  static size_t g = [] {
    const char* s = std::getenv("HFM_GUARD_BYTES");
    return s ? (size_t)std::strtoull(s, nullptr, 10) : (size_t)65536;
  }();
  return g;
}
int fill_byte() {
  static int f = [] {
    const char* s = std::getenv("HFM_GUARD_FILL");
    return s ? std::atoi(s) & 0xFF : 0xFF;
  }();
  return f;
}
std::mutex mu;
size_t n_alloc = 0, n_bad = 0;
}  // namespace

extern "C" {

void* hfm_guard_malloc(ssize_t size, int device, hipStream_t stream) {
  const size_t g = guard_bytes();
  const size_t tot = (size_t)size + 2 * g;
  void* p = nullptr;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  if (hipMalloc(&p, tot) != hipSuccess) {
    (void)hipSetDevice(prev);
    return nullptr;
  }
  (void)hipMemset(p, fill_byte(), tot);  // synchronous: the pattern is in place before first use
  (void)hipSetDevice(prev);
  std::lock_guard<std::mutex> lk(mu);
  ++n_alloc;
  (void)stream;
  return static_cast<char*>(p) + g;
}

void hfm_guard_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  const size_t g = guard_bytes();
  char* base = static_cast<char*>(ptr) - g;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  (void)hipDeviceSynchronize();
  if (g > 0) {
    std::vector<unsigned char> h(2 * g);
    (void)hipMemcpy(h.data(), base, g, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h.data() + g, base + g + size, g, hipMemcpyDeviceToHost);
    size_t first = (size_t)-1, cnt = 0;
    for (size_t i = 0; i < 2 * g; ++i)
      if (h[i] != (unsigned char)fill_byte()) {
        if (first == (size_t)-1) first = i;
        ++cnt;
      }
    if (cnt) {
      std::lock_guard<std::mutex> lk(mu);
      ++n_bad;
      const bool before = first < g;
      std::fprintf(stderr, "[guard_alloc] %zu guard bytes overwritten around %p (size %zd): first at %s%zu\n", cnt,
                   ptr, size, before ? "-" : "+", before ? g - first : first - g);
    }
  }
  (void)hipFree(base);
  (void)hipSetDevice(prev);
  (void)stream;
}

size_t hfm_guard_bad() {
  std::lock_guard<std::mutex> lk(mu);
  return n_bad;
}
}
