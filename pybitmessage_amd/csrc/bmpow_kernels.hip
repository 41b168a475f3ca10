// bmpow_kernels.hip -- gfx950 kernels for the Bitmessage double-SHA-512 proof of work.
//
// Hot path: reference src/proofofwork.py:100-111 (_doSafePoW: first n >= 1 with
// trial(n) <= target) whose trial is proofofwork.py:106-107.  Replaces the OpenCL kernel
// src/bitmsghash/bitmsghash.cl:254-275 and the pthread loop bitmsghash.cpp:39-74.
//
// Execution model (one launch = one bounded "step" of the host scheduler, bmpow_host.hip):
//   * the launch covers a list of work items; item = (object, contiguous nonce window);
//   * each item is cut into CHUNKs of BM_BLOCK x BM_ITERS nonces; one workgroup per chunk;
//     lane l of iteration i hashes nonce  chunk_first + i*BM_BLOCK + l;
//   * a hit does atomicMin(best[obj], nonce) -- the per-object minimum over the launch;
//   * exact first-nonce semantics: a chunk whose first nonce is above best[obj] cannot
//     hold the minimum, so it is skipped (checked at chunk start and after every iteration
//     with an agent-scope load: the early exit never skips a nonce below the answer);
//   * pure integer VALU -- no LDS, no MFMA, no HBM traffic beyond ~100 B per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

// Out-of-line trial for the small kernels (resolve, trials): one compiled copy of the ~6,500-
// instruction body instead of one inlined per kernel (the search kernel keeps its own inline
// copy, with the per-object words hoisted out of its nonce loop).
__device__ __noinline__ uint64_t trial_ool(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint64_t w4,
                                           uint64_t w5, uint64_t w6, uint64_t w7, uint64_t nonce) {
  const uint64_t ihw[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  return trial_of(ihw, nonce);
}

__device__ uint64_t trial_obj(const bm_obj* o, uint64_t nonce) {
  return trial_ool(o->w[0], o->w[1], o->w[2], o->w[3], o->w[4], o->w[5], o->w[6], o->w[7], nonce);
}

// ---------------------------------------------------------------------------------------
// Search kernel.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(BM_BLOCK) void bm_search_kernel(const bm_obj* __restrict__ objs,
                                                             const bm_item* __restrict__ items,
                                                             uint32_t nitems,
                                                             unsigned long long* __restrict__ best,
                                                             unsigned long long* __restrict__ trials_done,
                                                             uint32_t iters) {
  const uint32_t b = blockIdx.x;
  const uint64_t chunk = (uint64_t)BM_BLOCK * iters;  // nonces per workgroup in this launch
  // largest item index with chunk_base <= b (items sorted by chunk_base, uniform search)
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  const bm_item it = items[lo];
  const uint64_t off = (uint64_t)(b - it.chunk_base) * chunk;
  if (off >= it.count) return;
  const uint64_t cnt = (it.count - off < chunk) ? (it.count - off) : chunk;
  const uint64_t first = it.start + off;
  unsigned long long* bestp = best + it.obj;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < first) return;

  const bm_obj* o = objs + it.obj;
  uint64_t ihw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ihw[i] = o->w[i];
  const uint64_t target = o->target;

  uint32_t done = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    const uint64_t base = (uint64_t)i * BM_BLOCK;
    if (base >= cnt) break;
    // Early exit, one iteration of granularity at no stall: the running minimum is read
    // before this iteration's hashing (its latency hides behind ~6,500 VALU instructions)
    // and tested after it.  A value older by one iteration is only conservative.
    const uint64_t seen = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t j = base + threadIdx.x;
    const uint64_t nonce = first + j;
    const uint64_t tv = trial_of(ihw, nonce);
    if (j < cnt && tv <= target) atomicMin(bestp, (unsigned long long)nonce);
    done += (cnt - base < BM_BLOCK) ? (uint32_t)(cnt - base) : BM_BLOCK;
    if (seen < first + base + BM_BLOCK) break;  // every later nonce of this chunk is above it
  }
  if (threadIdx.x == 0) atomicAdd(trials_done, (unsigned long long)done);
}

// For each launched item whose object has a hit, recompute the trial value at the winning
// nonce (one thread per item).  res[k] = {nonce, trial} or {UINT64_MAX, 0}.
__global__ void bm_resolve_kernel(const bm_obj* __restrict__ objs, const bm_item* __restrict__ items,
                                  uint32_t nitems, const unsigned long long* __restrict__ best,
                                  bm_result* __restrict__ res) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nitems) return;
  const uint32_t obj = items[k].obj;
  const uint64_t n = best[obj];
  bm_result r;
  r.nonce = n;
  r.trial = 0;
  if (n != ~0ULL) r.trial = trial_obj(objs + obj, n);
  res[k] = r;
}

// Trial values for an arbitrary list of nonces of one object (parity probe / verification).
__global__ __launch_bounds__(BM_BLOCK) void bm_trials_kernel(const bm_obj* __restrict__ obj,
                                                             const uint64_t* __restrict__ nonces,
                                                             uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * BM_BLOCK + threadIdx.x;
  if (k >= n) return;
  out[k] = trial_obj(obj, nonces[k]);
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bm_launch_search(hipStream_t st, uint32_t nchunks, uint32_t iters, const bm_obj* objs,
                            const bm_item* items, uint32_t nitems, unsigned long long* best,
                            unsigned long long* trials_done) {
  hipLaunchKernelGGL(bm_search_kernel, dim3(nchunks), dim3(BM_BLOCK), 0, st, objs, items, nitems, best,
                     trials_done, iters);
  return hipGetLastError();
}

hipError_t bm_launch_resolve(hipStream_t st, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                             const unsigned long long* best, bm_result* res) {
  const uint32_t bs = 64;
  hipLaunchKernelGGL(bm_resolve_kernel, dim3((nitems + bs - 1) / bs), dim3(bs), 0, st, objs, items, nitems,
                     best, res);
  return hipGetLastError();
}

hipError_t bm_launch_trials(hipStream_t st, const bm_obj* obj, const uint64_t* nonces, uint64_t n,
                            uint64_t* out) {
  const uint64_t nb = (n + BM_BLOCK - 1) / BM_BLOCK;
  hipLaunchKernelGGL(bm_trials_kernel, dim3((uint32_t)nb), dim3(BM_BLOCK), 0, st, obj, nonces, n, out);
  return hipGetLastError();
}
