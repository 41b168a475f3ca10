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
//   * a hit does atomicMin(best[obj], nonce) -- the per-object minimum over the launch -- and
//     sets found[obj]: best[] starts at UINT64_MAX, which is also a legal nonce (2^64-1), so
//     "no hit" is found[obj] == 0, never a best[] value;
//   * exact first-nonce semantics: a chunk whose first nonce is above best[obj] cannot
//     hold the minimum, so it is skipped (checked at chunk start and after every iteration
//     with an agent-scope load: the early exit never skips a nonce below the answer);
//   * pure integer VALU -- no LDS, no MFMA, no HBM traffic beyond ~100 B per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

// ---------------------------------------------------------------------------------------
// Search kernel.
// ---------------------------------------------------------------------------------------
// Register budget for 5 waves per SIMD (<= 96 VGPRs; the allocator keeps 12 dwords of loop-invariant
// per-object terms in scratch, 6 scratch_load_dwordx2 per iteration, L1-resident).  Same-box A/B, C3
// 2^35 nonces, on three boxes: 6.53-6.59 GH/s against 6.30-6.39 at the 4 waves of 120 VGPRs
// (profiles/r02/search_kernel_ab_waves*.txt).  The gain needs the per-object words in VGPRs too: with
// them in SGPRs (BM_IHW_SGPR) 5 waves fit without scratch but run no faster than 4.
#ifndef BM_SEARCH_WAVES
#define BM_SEARCH_WAVES 5
#endif
__global__ __launch_bounds__(BM_BLOCK, BM_SEARCH_WAVES) void bm_search_kernel(const bm_obj* __restrict__ objs,
                                                             const bm_item* __restrict__ items,
                                                             uint32_t nitems,
                                                             unsigned long long* __restrict__ best,
                                                             uint32_t* __restrict__ found,
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

#ifdef BM_PRIO_MOD
  if (b % BM_PRIO_MOD == 0) __builtin_amdgcn_s_setprio(2);  // A/B knob: a share of the waves issue first
#endif
#ifdef BM_STAGGER
  for (uint32_t z = 0; z < (b & 3); ++z) __builtin_amdgcn_s_sleep(BM_STAGGER);  // A/B knob: de-phase the waves sharing a SIMD
#endif
  const bm_obj* o = objs + it.obj;
  uint64_t ihw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ihw[i] = o->w[i];
    // The per-object words, and the terms hoisted from them, live in VGPRs: left in SGPRs they
    // overflow the SGPR budget and every trial pays v_readlane reloads of the spilled ones (32 per
    // trial -> 18).  Same-box A/B, C3: 6.345 vs 6.302 GH/s (profiles/r02/search_kernel_ab*.txt).
#ifndef BM_IHW_SGPR
    asm volatile("" : "+v"(ihw[i]));
#endif
  }
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
    if (j < cnt && tv <= target) {
      atomicMin(bestp, (unsigned long long)nonce);
      __hip_atomic_store(found + it.obj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    done += (cnt - base < BM_BLOCK) ? (uint32_t)(cnt - base) : BM_BLOCK;
    if (seen < first + base + BM_BLOCK) break;  // every later nonce of this chunk is above it
  }
  if (threadIdx.x == 0) atomicAdd(trials_done, (unsigned long long)done);
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bm_launch_search(hipStream_t st, uint32_t nchunks, uint32_t iters, const bm_obj* objs,
                            const bm_item* items, uint32_t nitems, unsigned long long* best, uint32_t* found,
                            unsigned long long* trials_done) {
  hipLaunchKernelGGL(bm_search_kernel, dim3(nchunks), dim3(BM_BLOCK), 0, st, objs, items, nitems, best, found,
                     trials_done, iters);
  return hipGetLastError();
}
