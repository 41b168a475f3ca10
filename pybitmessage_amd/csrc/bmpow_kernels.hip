// bmpow_kernels.hip -- gfx950 kernels for the Bitmessage double-SHA-512 proof of work.
//
// Hot path: reference src/proofofwork.py:100-111 (_doSafePoW: first n >= 1 with
// trial(n) <= target) whose trial is proofofwork.py:106-107.  Replaces the OpenCL kernel
// src/bitmsghash/bitmsghash.cl:254-275 and the pthread loop bitmsghash.cpp:39-74.
//
// Execution model (one launch = one bounded "step" of the host scheduler, bmpow_host.hip):
//   * the launch covers a list of work items; item = (object, nonce window, its columns);
//   * the window is cut into blocks of BM_BLOCK nonces, one per lane; the item's workgroups take them
//     IN ORDER from the item's block queue (a per-item counter, bm_block_of in bmpow_kernels.h), so
//     the hashed set is always a prefix of the window plus the blocks in flight, however unevenly
//     the workgroups progress (the SIMD arbiter favours older waves);
//   * each wave reduces its hits to its lowest hitting lane (its 64 nonces are consecutive) and does
//     one atomicMin(best[obj], nonce) -- the per-object minimum over the launch -- and sets
//     found[obj]: best[] starts at UINT64_MAX, which is also a legal nonce (2^64-1), so "no hit" is
//     found[obj] == 0, never a best[] value;
//   * exact first-nonce semantics: a workgroup whose next block starts above the running minimum
//     stops (an agent-scope load after each block: the early exit never skips a nonce below the
//     answer); for a window split over shards the launch's relay workgroup folds the other shards'
//     hits (the host-pinned cross-shard bound) into that running minimum;
//   * pure integer VALU -- no MFMA, 16 B of LDS (the block index), and memory traffic of one queue
//     atomic per 256 trials plus ~100 B per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#ifdef BM_MID_SYNC  // A/B knob: a workgroup barrier between a trial's two compressions (wave phasing)
#define BM_TRIAL_MID() __syncthreads()
#endif
#include "sha512_dev.h"

using namespace bm;

// ---------------------------------------------------------------------------------------
// Search kernel.
// ---------------------------------------------------------------------------------------
// Register budget for 4 waves per SIMD (<= 128 VGPRs, no scratch).  With the static chunks of round 2,
// 5 waves (96 VGPRs, 12 dwords of loop-invariant terms spilled to scratch) ran 3 % faster than 4
// (profiles/r02/search_kernel_ab_waves*.txt); with the block queue the order reversed.  Same box, C3
// 2^35 nonces, twice each (profiles/r03/waves_queue_ab/): 4 waves 6.7025 / 6.7026 GH/s, 5 waves
// 6.691 / 6.684, 512-lane workgroups at 4 waves 6.695 / 6.691 and at 6 waves 6.662 / 6.666, 1,024-lane
// workgroups 6.28 / 6.29 -- and 4 waves carry no scratch traffic.
#ifndef BM_GRAB
#define BM_GRAB 1
#endif
#ifndef BM_SEARCH_WAVES
#define BM_SEARCH_WAVES 4
#endif
// One workgroup of a launch: it takes blocks of its item from the item's queue (bm_block_of), in
// order, until the window ends or the next block lies above the running minimum.
// kX: the launch holds windows split over shards, whose hits are published to the cross-shard bound.
template <bool kX>
__device__ __forceinline__ void search_column(const bm_obj* __restrict__ objs, const bm_item* __restrict__ items,
                                              uint32_t nitems, unsigned long long* __restrict__ best,
                                              uint32_t* __restrict__ found, unsigned long long* __restrict__ trials_done,
                                              unsigned long long* __restrict__ queue, unsigned long long* __restrict__ xb,
                                              uint32_t xrows, uint32_t b) {
  // largest item index with chunk_base <= b (items sorted by chunk_base, uniform search)
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  const bm_item it = items[lo];
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;  // blocks of the window
  // the queue hands out units of BM_GRAB blocks (1 by default; larger is an A/B knob)
  const uint64_t nunit = (nblk + BM_GRAB - 1) / BM_GRAB;
  unsigned long long* bestp = best + it.obj;
  unsigned long long* qp = queue + lo;
  __shared__ unsigned long long s_k[2];  // the unit taken, alternating slots (one barrier per unit)
  if (threadIdx.x == 0) s_k[0] = atomicAdd(qp, 1ull);
  __syncthreads();
  uint64_t unit = bm_block_of(it, s_k[0]);
  if (unit >= nunit) return;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < it.start + unit * (BM_GRAB * BM_BLOCK))
    return;

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
  for (uint32_t slot = 1;; slot ^= 1) {
    // the next unit, taken while this one is hashed (its latency hides behind ~6,200 VALU
    // instructions per block)
    unsigned long long kn = 0;
    if (threadIdx.x == 0) kn = atomicAdd(qp, 1ull);
#if BM_GRAB > 1
#pragma unroll 1
    for (uint32_t g = 0; g < BM_GRAB; ++g) {
      const uint64_t blk = unit * BM_GRAB + g;
      if (blk >= nblk) break;
#else
    {
      const uint64_t blk = unit;
#endif
      const uint64_t off = blk * BM_BLOCK;
      const uint64_t first = it.start + off;
      const uint64_t nonce = first + threadIdx.x;
      const uint64_t tv = trial_of(ihw, nonce);
#ifndef BM_LANE_ATOMICS
      // Wavefront min-reduction of the hits: a wave's 64 nonces are consecutive, so its smallest hit
      // is its lowest hitting lane -- one atomicMin per wave instead of one per hitting lane.  Same
      // box (profiles/r03/waves_queue_ab/wave_min_ab.txt): C3 6.713-6.718 against 6.709-6.718 GH/s
      // with lane atomics (BM_LANE_ATOMICS), C2 6.674-6.681 against 6.678, and the hit-heavy C5
      // flood at test-mode difficulty 5.816-5.837 against 5.761-5.835.
      const uint64_t hits = __builtin_amdgcn_ballot_w64(off + threadIdx.x < it.count && tv <= target);
      if (hits) {
        const uint64_t wmin = first + (threadIdx.x & ~63u) + (uint64_t)__builtin_ctzll(hits);
        if ((threadIdx.x & 63) == 0) {
          const unsigned long long prev = atomicMin(bestp, (unsigned long long)wmin);
          __hip_atomic_store(found + it.obj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (kX && it.xslot != BM_NO_XSLOT) bm_publish(bestp, xb, it.xslot, xrows, prev < wmin ? prev : wmin);
        }
      }
#else
      if (off + threadIdx.x < it.count && tv <= target) {
        const unsigned long long prev = atomicMin(bestp, (unsigned long long)nonce);
        __hip_atomic_store(found + it.obj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kX && it.xslot != BM_NO_XSLOT) bm_publish(bestp, xb, it.xslot, xrows, prev < nonce ? prev : nonce);
      }
#endif
      done += (it.count - off < BM_BLOCK) ? (uint32_t)(it.count - off) : BM_BLOCK;
    }
    // Early exit: the running minimum (for a split window also the other shards' hits, folded in by
    // the launch's relay) is tested against the next unit.  It is read after the hash, so a hit
    // published while this unit was hashed stops the workgroup now rather than one unit later; the
    // load's latency overlaps the wait at the barrier below.  Same box (profiles/r03/fresh_bound_ab.txt):
    // C1 waste 1.3-1.4 % against 2.1 % with the load issued before the hash; C3 6.705-6.707 against
    // 6.703-6.708 GH/s.  A stale value is only conservative.
    //
    // Each wave reads it itself, so two waves of the workgroup may see different values and part:
    // one stops, another goes on.  That is safe.  The one that stops saw a real hit below the next
    // block, so the lanes it leaves unhashed lie above an answer; the one that goes on finds its
    // slots no longer refreshed by thread 0 and re-hashes blocks it already hashed (their hits are
    // real ones) until its own read shows the hit -- within two blocks, since the last slot written
    // holds the block the other wave stopped at.  Sharing thread 0's read through LDS instead keeps
    // the waves in step but exposes the load's latency before the barrier: 4.7 % slower (C3 6.39
    // against 6.70 GH/s, same box, profiles/r03/steal_ab/lds_bound_ab.txt).
    const uint64_t seen = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) s_k[slot] = kn;
    __syncthreads();
    const uint64_t nu = bm_block_of(it, s_k[slot]);
    // a unit taken and not hashed lies past the window or above a hit: no nonce below the answer
    // is skipped
    if (nu >= nunit || seen < it.start + nu * (BM_GRAB * BM_BLOCK)) break;
    unit = nu;
  }
  if (threadIdx.x == 0) atomicAdd(trials_done, (unsigned long long)done);
}

// kX = false: every launch without split windows (one shard; as many objects as shards) -- the hot
// loop carries nothing of the cross-shard bound.  kX = true: workgroup 0 is the relay (bm_relay),
// columns are workgroups 1.., and each column counts itself in trials_done[1] as it ends.
template <bool kX>
__global__ __launch_bounds__(BM_BLOCK, BM_SEARCH_WAVES) void bm_search_kernel(const bm_obj* __restrict__ objs,
                                                             const bm_item* __restrict__ items,
                                                             uint32_t nitems,
                                                             unsigned long long* __restrict__ best,
                                                             uint32_t* __restrict__ found,
                                                             unsigned long long* __restrict__ trials_done,
                                                             unsigned long long* __restrict__ queue,
                                                             unsigned long long* __restrict__ xb,
                                                             uint32_t xrow, uint32_t xrows) {
  if constexpr (kX) {
    if (blockIdx.x == 0) {
      bm_relay(items, nitems, best, xb, xrow, trials_done + 1, gridDim.x - 1);
      return;
    }
    search_column<true>(objs, items, nitems, best, found, trials_done, queue, xb, xrows, blockIdx.x - 1);
    if (threadIdx.x == 0) atomicAdd(trials_done + 1, 1ull);
  } else {
    search_column<false>(objs, items, nitems, best, found, trials_done, queue, nullptr, 0, blockIdx.x);
  }
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bm_launch_search(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                            unsigned long long* best, uint32_t* found, unsigned long long* trials_done,
                            unsigned long long* queue, const bm_xbound& xb) {
  if (xb.table)
    hipLaunchKernelGGL(bm_search_kernel<true>, dim3(nwg + 1), dim3(BM_BLOCK), 0, st, objs, items, nitems, best, found,
                       trials_done, queue, xb.table, xb.row, xb.rows);
  else
    hipLaunchKernelGGL(bm_search_kernel<false>, dim3(nwg), dim3(BM_BLOCK), 0, st, objs, items, nitems, best, found,
                       trials_done, queue, nullptr, 0u, 0u);
  return hipGetLastError();
}

int bm_search_resident_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bm_search_kernel<false>, BM_BLOCK, 0) != hipSuccess) return 0;
  return n;
}
