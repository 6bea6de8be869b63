// In-launch hand-offs between workgroups (gfx950: 8 XCDs with private L2s; L1 per CU).
//
// Two forms.  (1) Small payloads: stored write-through (relaxed agent-scope atomic stores, sc1),
// a drain of EVERY storing wave, a barrier, ONE relaxed atomic flag store; the consumer polls
// relaxed, runs ONE agent-scope acquire after the match (its workgroups share CUs: the fence-free
// sc1-load form is validated for one workgroup per CU only -- without it the sparse look-back
// and the wgfin split-K combine read stale partials now and then) and reads the payload with
// relaxed agent-scope atomic loads (sc1).  A release fence per producer workgroup writes back its
// XCD's whole L2 -- with 1248 producers that cost the sparse kernel 2x -- so producers stay
// write-through.  (2) Bulk payloads: plain stores, drain, barrier, ONE agent-scope
// release fence (+ a second drain) and ONE relaxed atomic on the counter; the consumer polls
// relaxed with s_sleep back-off, then ONE agent-scope acquire before plain loads.
// Waits are only ever on workgroups with a LOWER linear id (dispatched earlier on every XCD), so
// they always make progress; every spin is still bounded and reports a timeout through an error
// word instead of hanging the GPU.
//
// Sync words never need a reset between launches: a launch publishes a tag that is unique to it
// (the training step's index), so words written by earlier launches never match; the host zeroes
// them when it rewrites the step counter (checkpoint restore).  (A per-launch done counter that
// advances an epoch costs one contended atomic per workgroup: measured ~2x slower on a
// 1248-workgroup launch.)
#pragma once
#include "common.h"

#define HFM_RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

constexpr unsigned HFM_SPIN_LIMIT = 1u << 22;  // x s_sleep(2) ~ 0.5 s: far beyond any real wait

// every wave of the producer workgroup calls this after its last payload store
__device__ __forceinline__ void hx_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// form (1): write-through payload stores
__device__ __forceinline__ void hx_stf(float* p, float v) { __hip_atomic_store(p, v, HFM_RLX_AGENT); }
__device__ __forceinline__ void hx_sti(int* p, int v) { __hip_atomic_store(p, v, HFM_RLX_AGENT); }

// form (1): one lane stores the flag after hx_drain() in every storing wave and a __syncthreads()
__device__ __forceinline__ void hx_flag(unsigned* word, unsigned value) {
  asm volatile("" ::: "memory");
  __hip_atomic_store(word, value, HFM_RLX_AGENT);
}

// form (2): one lane publishes after hx_drain() in every wave and a __syncthreads()
__device__ __forceinline__ void hx_publish(unsigned* word, unsigned value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(word, value, HFM_RLX_AGENT);
}

__device__ __forceinline__ unsigned hx_add(unsigned* word, unsigned v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return __hip_atomic_fetch_add(word, v, HFM_RLX_AGENT);
}

__device__ __forceinline__ unsigned hx_load(const unsigned* word) {
  return __hip_atomic_load(const_cast<unsigned*>(word), HFM_RLX_AGENT);
}

// handed-off words read at a wave-uniform address: an atomic load keeps them on the vector path
// (a plain load of a uniform address may become a scalar-cache load, which the acquire does not
// refresh)
__device__ __forceinline__ int hx_ldi(const int* p) {
  return __hip_atomic_load(const_cast<int*>(p), HFM_RLX_AGENT);
}
__device__ __forceinline__ float hx_ldf(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), HFM_RLX_AGENT);
}

// one acquire after the poll succeeded; then (several reading waves) drain + __syncthreads()
__device__ __forceinline__ void hx_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// wave-uniform poll of one word until it is >= target; false on timeout (err |= code)
__device__ __forceinline__ bool hx_wait_geq(const unsigned* word, unsigned target, unsigned* err,
                                            unsigned code) {
  for (unsigned spins = 0; hx_load(word) < target; ++spins) {
    if (spins >= HFM_SPIN_LIMIT) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, code);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}
