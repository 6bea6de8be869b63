// Same-device collective transport: N training PROCESSES on ONE GPU exchange through IPC-mapped
// device memory, behind the same grouped-collective interface as the RCCL engine (comm.hip).
//
// Why: the multi-rank step (row-sharded all-to-alls, dense gradient exchange, run-level routing,
// HIP graphs of whole runs) is the production path of the 8-GPU job, and RCCL refuses two ranks
// on one device ("Duplicate GPU detected").  This engine lets the one-GPU box run that path with
// real processes -- every rank its own HIP context, queues, graphs and caching allocator, exactly
// as on 8 GPUs -- so the first 8-GPU run is not the first time the path executes
// (HIPFM_SAME_DEVICE=1, parallel/dist.py).  Only the transport differs from RCCL.
//
// Protocol of one group (hfm_lb_group), enqueued on the caller's stream, capturable:
//   1. pack kernel   : every op's send buffer -> this rank's staging half h (h = op counter & 1)
//   2. host node     : cross-process barrier on a shared-memory counter (all ranks packed op k)
//   3. pull kernel   : every op's recv buffer <- the peers' staging halves h (all-to-all block r
//                      of peer p, peer p's all-gather block, or the f32 sum over ranks IN RANK
//                      ORDER: every rank computes the same bits); its last workgroup advances
//                      the op counter.
// Two staging halves make one barrier per group enough: rank r packs op k+2 into half h only
// after passing barrier k+1, and every peer reaches barrier k+1 only after its pull of op k has
// finished (a host node runs when the stream's earlier work is complete).
// The barrier never spins forever: after HIPFM_LB_TIMEOUT_MS it poisons the shared word, every
// rank's later barriers return at once (the queued work drains), and the engine's error word
// makes the Python side raise (no silent wrong step goes unreported).
#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>

#include "common.h"

namespace {

constexpr int LB_MAX_RANKS = 16;
constexpr int LB_MAX_OPS = 4;
constexpr int LB_THREADS = 256;
constexpr int LB_BLOCKS = 1024;       // 4 workgroups per CU: enough to stream the copies at HBM rate

struct LbShared {                     // the shared-memory page every rank maps
  std::atomic<uint32_t> count;        // arrivals at the current barrier
  std::atomic<uint32_t> gen;          // barrier generation
  std::atomic<uint32_t> poison;       // a rank timed out: every barrier returns at once
  uint32_t nranks;
};

struct LbOp {
  int kind;                           // 0 all-to-all, 1 all-gather, 2 f32 sum all-reduce
  int pad;
  const char* send;
  char* recv;
  size_t bytes;                       // per peer / per rank / in total (multiple of 4)
  size_t off;                         // offset of this op's block in a staging half
};

struct LbArgs {
  const char* peers[LB_MAX_RANKS];    // every rank's staging base (this rank's own included)
  char* stage;                        // this rank's staging base
  unsigned* ctr;                      // device op counter (parity selects the half)
  unsigned* ticket;                   // pull launch: finished workgroups
  size_t half;                        // bytes per staging half
  int rank, nranks, nops;
  int pad;
  LbOp ops[LB_MAX_OPS];
};

struct LbEngine {
  int rank = 0, nranks = 0, timeout_ms = 60000;
  LbShared* shm = nullptr;
  char* stage = nullptr;
  size_t half = 0;
  char* peers[LB_MAX_RANKS] = {};
  unsigned* dev_words = nullptr;      // [0] op counter, [1] ticket
  std::atomic<int> err{0};            // 1: this rank timed out, 2: a peer timed out
  unsigned long long groups = 0;
};

// a staging half holds the ops of a group: all-to-all N x bytes, all-gather / all-reduce bytes
size_t op_stage_bytes(int kind, size_t bytes, int nranks) {
  const size_t b = kind == 0 ? bytes * (size_t)nranks : bytes;
  return (b + 255) & ~(size_t)255;
}

// copy `n` 4-byte words with 16-B accesses where both ends allow it
__device__ __forceinline__ void copy_words(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                           size_t n, size_t tid, size_t nth) {
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const size_t n4 = n / 4;
    uint4* d4 = (uint4*)dst;
    const uint4* s4 = (const uint4*)src;
    for (size_t i = tid; i < n4; i += nth) d4[i] = s4[i];
    for (size_t i = n4 * 4 + tid; i < n; i += nth) dst[i] = src[i];
  } else {
    for (size_t i = tid; i < n; i += nth) dst[i] = src[i];
  }
}

__global__ void __launch_bounds__(LB_THREADS) lb_pack_kernel(LbArgs a) {
  const unsigned h = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u;
  char* base = a.stage + h * a.half;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
  for (int o = 0; o < a.nops; ++o) {
    const LbOp& op = a.ops[o];
    const size_t b = op.kind == 0 ? op.bytes * (size_t)a.nranks : op.bytes;
    copy_words((uint32_t*)(base + op.off), (const uint32_t*)op.send, b / 4, tid, nth);
  }
  // the peers read this half from other processes: make the writes visible device-wide (the
  // end-of-kernel release does too; this states it where the protocol needs it)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

__global__ void __launch_bounds__(LB_THREADS) lb_pull_kernel(LbArgs a) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // the peers' halves were written elsewhere
  const unsigned h = __hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
  const int N = a.nranks;
  for (int o = 0; o < a.nops; ++o) {
    const LbOp& op = a.ops[o];
    if (op.kind == 2) {
      // f32 sum over ranks in rank order (identical bits on every rank)
      const size_t n = op.bytes / 4;
      float* dst = (float*)op.recv;
      for (size_t i = tid; i < n; i += nth) {
        float s = 0.f;
        for (int p = 0; p < N; ++p) s += ((const float*)(a.peers[p] + h * a.half + op.off))[i];
        dst[i] = s;
      }
    } else {
      for (int p = 0; p < N; ++p) {
        const char* src = a.peers[p] + h * a.half + op.off + (op.kind == 0 ? (size_t)a.rank * op.bytes : 0);
        copy_words((uint32_t*)(op.recv + (size_t)p * op.bytes), (const uint32_t*)src, op.bytes / 4, tid, nth);
      }
    }
  }
  // the last workgroup to finish advances the op counter (every workgroup read it above)
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// host node: sense-counting barrier over the shared page, bounded by the engine's timeout
void lb_barrier(void* p) {
  LbEngine* e = (LbEngine*)p;
  LbShared* s = e->shm;
  if (s->poison.load(std::memory_order_acquire)) {
    e->err.store(2);
    return;
  }
  const uint32_t g = s->gen.load(std::memory_order_acquire);
  if (s->count.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)e->nranks - 1) {
    s->count.store(0, std::memory_order_relaxed);
    s->gen.fetch_add(1, std::memory_order_release);
    return;
  }
  const double t0 = now_ms();
  for (unsigned spin = 0; s->gen.load(std::memory_order_acquire) == g; ++spin) {
    if (s->poison.load(std::memory_order_acquire)) {
      e->err.store(2);
      return;
    }
    if (spin < 2000) continue;
    if ((spin & 63) == 0 && now_ms() - t0 > e->timeout_ms) {
      s->poison.store(1, std::memory_order_release);
      e->err.store(1);
      fprintf(stderr, "[hipfm loopback] rank %d: barrier of group %llu timed out after %d ms; "
              "poisoning the transport\n", e->rank, e->groups, e->timeout_ms);
      return;
    }
    if (spin < 20000) sched_yield();
    else {
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
    }
  }
}

}  // namespace

HFM_API int hfm_lb_shared_bytes() { return (int)sizeof(LbShared); }

// `path`: a file under /dev/shm; rank 0 creates it (create = 1) before the others open it.
HFM_API int hfm_lb_create(void** out, int nranks, int rank, const char* path, int create, int timeout_ms) {
  if (nranks < 1 || nranks > LB_MAX_RANKS || rank < 0 || rank >= nranks) return (int)hipErrorInvalidValue;
  const int fd = open(path, create ? (O_RDWR | O_CREAT | O_EXCL) : O_RDWR, 0600);
  if (fd < 0) return (int)hipErrorInvalidValue;
  if (create && ftruncate(fd, 4096) != 0) {
    close(fd);
    return (int)hipErrorInvalidValue;
  }
  void* m = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return (int)hipErrorInvalidValue;
  LbEngine* e = new LbEngine();
  e->rank = rank;
  e->nranks = nranks;
  e->timeout_ms = timeout_ms > 0 ? timeout_ms : 60000;
  e->shm = (LbShared*)m;
  if (create) {
    e->shm->count.store(0);
    e->shm->gen.store(0);
    e->shm->poison.store(0);
    e->shm->nranks = (uint32_t)nranks;
  }
  hipError_t r = hipMalloc((void**)&e->dev_words, 256);
  if (r == hipSuccess) r = hipMemset(e->dev_words, 0, 256);
  if (r != hipSuccess) {
    munmap(m, 4096);
    delete e;
    return (int)r;
  }
  *out = e;
  return 0;
}

// Host-only exercise of the engine's barrier (no GPU: tests/test_loopback_barrier.py runs it in
// several CPU processes): `iters` barriers over the shared page at `path` (rank 0 creates it);
// before barrier i every rank adds 1 to a check word in the page's spare half and after it reads
// the word back, which must be >= (i + 1) * nranks (no rank passes a barrier before all arrive).
// Rank `stall_rank` sleeps `stall_ms` before barrier `stall_at` (timeout / poison path).
// Returns the engine's error word (0 ok, 1 this rank timed out, 2 a peer poisoned the page),
// 3 on a check-word violation, -1 on setup failure.
HFM_API int hfm_lb_barrier_selftest(const char* path, int nranks, int rank, int create, int timeout_ms, int iters,
                                    int stall_rank, int stall_at, int stall_ms) {
  if (nranks < 1 || nranks > LB_MAX_RANKS || rank < 0 || rank >= nranks) return -1;
  const int fd = open(path, create ? (O_RDWR | O_CREAT | O_EXCL) : O_RDWR, 0600);
  if (fd < 0) return -1;
  if (create && ftruncate(fd, 4096) != 0) {
    close(fd);
    return -1;
  }
  void* m = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return -1;
  LbEngine e;
  e.rank = rank;
  e.nranks = nranks;
  e.timeout_ms = timeout_ms > 0 ? timeout_ms : 60000;
  e.shm = (LbShared*)m;
  auto* chk = reinterpret_cast<std::atomic<uint32_t>*>((char*)m + 2048);
  if (create) {
    e.shm->count.store(0);
    e.shm->gen.store(0);
    e.shm->poison.store(0);
    e.shm->nranks = (uint32_t)nranks;
    chk->store(0);
  }
  int rc = 0;
  for (int i = 0; i < iters && rc == 0; ++i) {
    if (rank == stall_rank && i == stall_at) {
      timespec ts{stall_ms / 1000, (long)(stall_ms % 1000) * 1000000L};
      nanosleep(&ts, nullptr);
    }
    chk->fetch_add(1, std::memory_order_acq_rel);
    e.groups = (unsigned long long)i;
    lb_barrier(&e);
    rc = e.err.load();
    if (rc == 0 && chk->load(std::memory_order_acquire) < (uint32_t)((i + 1) * nranks)) rc = 3;
  }
  munmap(m, 4096);
  return rc;
}

HFM_API int hfm_lb_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// (Re)allocate this rank's staging (2 halves of `half` bytes) and export its IPC handle.  Every
// rank calls it at the same point of its host program with the same size; the previous staging
// is NOT freed (graphs captured on it may still be replayed: it stays mapped until destroy).
HFM_API int hfm_lb_alloc_stage(void* eng, size_t half, void* handle_out) {
  LbEngine* e = (LbEngine*)eng;
  half = (half + 4095) & ~(size_t)4095;
  char* p = nullptr;
  hipError_t r = hipMalloc((void**)&p, 2 * half);
  if (r != hipSuccess) return (int)r;
  r = hipMemset(p, 0, 2 * half);
  if (r == hipSuccess) r = hipDeviceSynchronize();
  if (r == hipSuccess) r = hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, p);
  if (r != hipSuccess) {
    hipFree(p);
    return (int)r;
  }
  e->stage = p;
  e->half = half;
  return 0;
}

// Map every peer's staging from the gathered handles ([nranks] hipIpcMemHandle_t).
HFM_API int hfm_lb_open_peers(void* eng, const void* handles) {
  LbEngine* e = (LbEngine*)eng;
  const hipIpcMemHandle_t* h = (const hipIpcMemHandle_t*)handles;
  for (int p = 0; p < e->nranks; ++p) {
    if (p == e->rank) {
      e->peers[p] = e->stage;
      continue;
    }
    void* q = nullptr;
    const hipError_t r = hipIpcOpenMemHandle(&q, h[p], hipIpcMemLazyEnablePeerAccess);
    if (r != hipSuccess) return (int)r;
    e->peers[p] = (char*)q;
  }
  return 0;
}

struct CommOpIn {                      // layout of comm.hip's CommOp (ops/_lib.py CommOp)
  int kind;
  int pad;
  const void* send;
  void* recv;
  size_t bytes;
};

HFM_API int hfm_lb_group(void* eng, const CommOpIn* ops, int nops, hipStream_t st) {
  LbEngine* e = (LbEngine*)eng;
  if (nops < 0 || nops > LB_MAX_OPS) return (int)hipErrorInvalidValue;
  LbArgs a;
  memset(&a, 0, sizeof(a));
  for (int p = 0; p < e->nranks; ++p) a.peers[p] = e->peers[p];
  a.stage = e->stage;
  a.ctr = e->dev_words;
  a.ticket = e->dev_words + 1;
  a.half = e->half;
  a.rank = e->rank;
  a.nranks = e->nranks;
  size_t off = 0;
  int n = 0;
  for (int i = 0; i < nops; ++i) {
    if (ops[i].bytes % 4 || ops[i].kind < 0 || ops[i].kind > 2) return (int)hipErrorInvalidValue;
    if (ops[i].bytes == 0) continue;
    LbOp& o = a.ops[n++];
    o.kind = ops[i].kind;
    o.send = (const char*)ops[i].send;
    o.recv = (char*)ops[i].recv;
    o.bytes = ops[i].bytes;
    o.off = off;
    off += op_stage_bytes(o.kind, o.bytes, e->nranks);
  }
  a.nops = n;
  if (n == 0) return 0;
  if (off > e->half || e->stage == nullptr) return (int)hipErrorInvalidValue;   // caller reserves first
  ++e->groups;
  hipLaunchKernelGGL(lb_pack_kernel, dim3(LB_BLOCKS), dim3(LB_THREADS), 0, st, a);
  hipError_t r = hipGetLastError();
  if (r != hipSuccess) return (int)r;
  r = hipLaunchHostFunc(st, lb_barrier, e);
  if (r != hipSuccess) return (int)r;
  hipLaunchKernelGGL(lb_pull_kernel, dim3(LB_BLOCKS), dim3(LB_THREADS), 0, st, a);
  HFM_LAUNCH_CHECK();
}

// bytes per staging half, in KiB (halves are page multiples)
HFM_API int hfm_lb_stage_half_kb(void* eng) { return (int)(((LbEngine*)eng)->half >> 10); }

// 0 ok, 1 this rank's barrier timed out, 2 a peer's did (the transport is poisoned)
HFM_API int hfm_lb_error(void* eng) { return ((LbEngine*)eng)->err.load(); }

// Unmaps the peers and the shared page; the staging stays allocated until process exit (graphs
// captured on it may outlive the engine object).
HFM_API int hfm_lb_destroy(void* eng) {
  LbEngine* e = (LbEngine*)eng;
  if (!e) return 0;
  for (int p = 0; p < e->nranks; ++p)
    if (p != e->rank && e->peers[p]) hipIpcCloseMemHandle(e->peers[p]);
  munmap(e->shm, 4096);
  delete e;
  return 0;
}
