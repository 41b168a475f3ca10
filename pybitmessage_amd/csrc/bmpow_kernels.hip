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
#ifndef BM_LOG_RELEASE
#define BM_LOG_RELEASE 0
#endif
#ifndef BM_LAG_PRIO  // A/B knob: issue priority for workgroups behind the queue (sweep)
#define BM_LAG_PRIO 0
#endif
#ifndef BM_CUT  // the single-object kernel's mid-trial bound check (sweep's kOne); 0 for A/B builds
#define BM_CUT 1
#endif
// One workgroup's sweep of a work item: it takes the item's blocks from the item's queue (bm_block_of),
// in order, until the window ends or the next block lies above the running minimum.
// kX: the launch holds items with a cross-shard bound slot, whose hits are published there.
// log (the single-object kernel): each hit's trial value is logged, so the result needs no re-hash.
// kOne (the single-object kernel): the running minimum is read again between a block's two
// compressions (BM_CUT); a block that starts above it skips its second (every nonce of it lies above
// a hit), so a wave stops half a trial sooner after the answer is published.  Such lanes are counted
// in cut, not in the trials hashed.  The kernel folds its waves' counts per workgroup (bm_fold_leave).
// Returns this wave's own counts (every wave counts itself, whichever of the workgroup's waves leaves
// first).
struct bm_swept {
  uint32_t done;  // trials hashed by this wave's lanes
  uint32_t cut;   // lanes whose block skipped its second compression
  uint32_t hit;   // 1: this wave published a hit
};
template <bool kX, bool kOne = false>
__device__ __forceinline__ bm_swept sweep(const bm_item& it, uint32_t qi, const uint64_t* __restrict__ wsrc,
                                          uint64_t target, unsigned long long* __restrict__ bestp,
                                          uint32_t* __restrict__ foundp, unsigned long long* __restrict__ queue,
                                          unsigned long long* __restrict__ xb, uint32_t xrows,
                                          bm_one_call* __restrict__ log) {
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;  // blocks of the window
  // the queue hands out units of BM_GRAB blocks (1 by default; larger is an A/B knob)
  const uint64_t nunit = (nblk + BM_GRAB - 1) / BM_GRAB;
  unsigned long long* qp = queue + qi;
  __shared__ unsigned long long s_k[2];  // the unit taken, alternating slots (one barrier per unit)
  if (threadIdx.x == 0) {
    s_k[0] = atomicAdd(qp, 1ull);
    if constexpr (kOne) bm_fold_init();
  }
  __syncthreads();
  bm_swept r = {0, 0, 0};
#if BM_LAG_PRIO
  unsigned long long kprev = s_k[0];
#endif
  uint64_t unit = bm_block_of(it, s_k[0]);
  if (unit >= nunit) return r;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < it.start + unit * (BM_GRAB * BM_BLOCK))
    return r;

#ifdef BM_PRIO_MOD
  if (blockIdx.x % BM_PRIO_MOD == 0) __builtin_amdgcn_s_setprio(2);  // A/B knob: a share of the waves issue first
#endif
  uint64_t ihw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ihw[i] = wsrc[i];
    // The per-object words, and the terms hoisted from them, live in VGPRs: left in SGPRs they
    // overflow the SGPR budget and every trial pays v_readlane reloads of the spilled ones (32 per
    // trial -> 18).  Same-box A/B, C3: 6.345 vs 6.302 GH/s (profiles/r02/search_kernel_ab*.txt).
#ifndef BM_IHW_SGPR
    asm volatile("" : "+v"(ihw[i]));
#endif
  }

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
      bool live = off + threadIdx.x < it.count;
#ifdef BM_HETERO  // A/B variant: odd waves run the other instruction order (sha512_dev.h)
      const uint64_t tv = ((threadIdx.x >> 6) & 1) ? trial_of_b(ihw, nonce) : trial_of(ihw, nonce);
#else
      uint64_t tv;
      if constexpr (kOne && BM_CUT) {
        bool c = false;
        tv = trial_of_cut(
            ihw, nonce, [&] { return __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < first; }, c);
        if (c) {
          r.cut += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(live));
          live = false;
        }
      } else {
        tv = trial_of(ihw, nonce);
      }
#endif
      // Wavefront min-reduction of the hits: a wave's 64 nonces are consecutive, so its smallest hit
      // is its lowest hitting lane -- one atomicMin per wave instead of one per hitting lane.  Same
      // box (profiles/r03/waves_queue_ab/wave_min_ab.txt): C3 6.713-6.718 against 6.709-6.718 GH/s
      // with lane atomics, C2 6.674-6.681 against 6.678, and the hit-heavy C5 flood at test-mode
      // difficulty 5.816-5.837 against 5.761-5.835.
      const uint64_t hits = __builtin_amdgcn_ballot_w64(live && tv <= target);
      if (hits) {
        r.hit = 1;
        const uint32_t lane = (uint32_t)__builtin_ctzll(hits);
        const uint64_t wmin = first + (threadIdx.x & ~63u) + lane;
        uint64_t wtv = 0;
        if (log)  // the hit lane's trial value, for the single-object result
          wtv = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(tv >> 32), (int)lane) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tv, (int)lane);
        if ((threadIdx.x & 63) == 0) {
          const unsigned long long prev = atomicMin(bestp, (unsigned long long)wmin);
          __hip_atomic_store(foundp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (log) {
            const uint32_t k = atomicAdd(&log->nhits, 1u);
            if (k < BM_ONE_LOG) {
              // plain stores: the workgroup's fold and its release at the end carry them to the
              // launch's last workgroup (bm_search1_kernel)
              log->hit_trial[k] = wtv;
#if BM_LOG_RELEASE  // A/B knob: a release per logged hit
              __hip_atomic_store(&log->hit_nonce[k], (unsigned long long)wmin, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#else
              __hip_atomic_store(&log->hit_nonce[k], (unsigned long long)wmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
            }
          }
          if (kX && it.xslot != BM_NO_XSLOT) bm_publish(bestp, xb, it.xslot, xrows, prev < wmin ? prev : wmin);
        }
      }
      r.done += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(live));
    }
    // Early exit: the running minimum (for a shared object also the other shards' hits, folded in by
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
    // holds the block the other wave stopped at.  The barrier below then waits only for the waves
    // still running: a wave that has ended no longer counts at s_barrier (the hardware drops ended
    // waves from the workgroup's barrier).  Sharing thread 0's read through LDS instead keeps the
    // waves in step but exposes the load's latency before the barrier: 4.7 % slower (C3 6.39 against
    // 6.70 GH/s, same box, profiles/r03/steal_ab/lds_bound_ab.txt).
    const uint64_t seen = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) s_k[slot] = kn;
    __syncthreads();
#if BM_LAG_PRIO
    {
      // A workgroup that fell behind -- more of the queue's units taken by the item's workgroups
      // during its last unit than 5/4 of their count -- issues first for its next unit.  The SIMD
      // arbiter otherwise favours older waves, and a starved workgroup holding the unit with the
      // answer delays the answer by its whole unit time (the long tail of C1 calls).
      const unsigned long long kr = s_k[slot];
      const uint32_t taken = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(kr - kprev));
      kprev = kr;
      if (taken > it.nwg + (it.nwg >> 2)) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
    const uint64_t nu = bm_block_of(it, s_k[slot]);
    // a unit taken and not hashed lies past the window or above a hit: no nonce below the answer
    // is skipped
    if (nu >= nunit || seen < it.start + nu * (BM_GRAB * BM_BLOCK)) break;
    unit = nu;
  }
  return r;
}

// One workgroup of a batch launch: the item holding workgroup b (the largest item index with
// chunk_base <= b; items sorted by chunk_base, a uniform binary search), then its sweep.
template <bool kX>
__device__ __forceinline__ void search_column(const bm_obj* __restrict__ objs, const bm_item* __restrict__ items,
                                              uint32_t nitems, unsigned long long* __restrict__ best,
                                              uint32_t* __restrict__ found, unsigned long long* __restrict__ trials_done,
                                              unsigned long long* __restrict__ queue, unsigned long long* __restrict__ xb,
                                              uint32_t xrows, uint32_t b) {
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  const bm_item it = items[lo];
  const bm_obj* o = objs + it.obj;
  const bm_swept r = sweep<kX>(it, lo, o->w, o->target, best + it.obj, found + it.obj, queue, xb, xrows, nullptr);
  // Each wave adds its own count: no workgroup fold here.  The fold of the single-object kernel,
  // though it runs only as the waves leave, cut this kernel's VALU dual issue from 6.1 % to 1.6 % of
  // its instructions and its rate by 4.7 % (PMC, same box: profiles/r04/eng9/) -- a launch-long effect
  // of a change outside the loop, measured, not understood -- while 4,096 atomics at the end of an
  // 80 ms launch cost it ~0.06 %.
  if ((threadIdx.x & 63) == 0) {
    if (r.done) atomicAdd(trials_done, (unsigned long long)r.done);
    if (kX) atomicAdd(trials_done + 1, 1ull);  // a column wave has finished (bm_relay)
  }
}

// kX = false: every launch without shared objects -- the hot loop carries nothing of the
// cross-shard bound.  kX = true: workgroup 0 is the relay (bm_relay), columns are workgroups 1..,
// and each of their waves counts itself in trials_done[1] as it leaves (search_column).
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
      bm_relay(items, nitems, best, xb, xrow, trials_done + 1, (gridDim.x - 1) * (BM_BLOCK / 64));
      return;
    }
    search_column<true>(objs, items, nitems, best, found, trials_done, queue, xb, xrows, blockIdx.x - 1);
  } else {
    search_column<false>(objs, items, nitems, best, found, trials_done, queue, nullptr, 0, blockIdx.x);
  }
}

// The trial value of the single-object result when the hit log overflowed (a very easy object): out
// of line, so its registers are not the sweep's.
__device__ __noinline__ uint64_t trial_one(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint64_t w4,
                                           uint64_t w5, uint64_t w6, uint64_t w7, uint64_t nonce) {
  const uint64_t ihw[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  return trial_of(ihw, nonce);
}

// The single-object kernel of run() (bm_one_args, bmpow_layout.h): one window (or, with kX, one
// device's piece of it), the object in the arguments; the launch's last workgroup to finish writes the
// result into host-mapped memory -- the minimum, its trial value from the hit log (re-hashed only when
// the log overflowed), the trials hashed and the launch's start and end on the 100 MHz realtime clock
// -- and then its sequence number, which the host polls.  (The argument's fields are read into locals:
// taking the address of a by-value kernel argument copies it to scratch.)
//
// kX (a run() split over several physical devices): workgroup 0 is the relay.  One lane polls this
// piece's row of the cross-device table (a system-scope load every few microseconds) and folds what the
// other devices' pieces published into this device's running minimum, which every column reads once
// per block; it leaves once every column workgroup has counted itself in ctr->acc, adds itself, and so
// is the launch's last workgroup -- it writes the result.  Columns publish their hits into every row
// (bm_publish).  Every value in the table is a real hit of the object, so it only stops columns above
// an answer.  kX = false is the one-device kernel, with none of this in its code.
template <bool kX>
__device__ __forceinline__ void one_result(const bm_one_args& a, bm_one_ctr* ctr, bm_one_call* call, const uint64_t (&w)[8],
                                           uint64_t acc) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // the last workgroup's last wave (lane 0): every workgroup's counts and hits are in
  const uint64_t best = __hip_atomic_load(&call->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t found = __hip_atomic_load(&call->found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t nh = __hip_atomic_load(&call->nhits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t trial = 0;
  bool have = false;
  for (uint32_t k = 0; found && k < nh && k < BM_ONE_LOG && !have; ++k)
    if (__hip_atomic_load(&call->hit_nonce[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == best) {
      trial = call->hit_trial[k];
      have = true;
    }
  // the log overflowed, or (kX) the minimum is another device's hit folded in by the relay
  if (found && !have) trial = trial_one(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], best);
  bm_one_out* const o = a.out;
  const uint64_t t1 = (uint64_t)__builtin_amdgcn_s_memrealtime();
  uint64_t t0 = __hip_atomic_load(&ctr->t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t0 == 0 || t0 > t1) t0 = t1;  // workgroup 0 not seen yet: no span rather than a wrong one
  __hip_atomic_store(&o->nonce, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->trial, trial, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->trials, acc >> 31, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->t0, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->t1, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->found, found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&o->cut, (uint32_t)((acc >> 12) & 0x7ffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // the launch's counters, for the launch that next uses this ring entry
  ctr->queue = 0;
  ctr->acc = 0;
  ctr->t0 = 0;
  __hip_atomic_store(&o->seq, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool kX>
__global__ __launch_bounds__(BM_BLOCK, BM_SEARCH_WAVES) void bm_search1_kernel(const bm_one_args a) {
  bm_one_ctr* const ctr = a.ctr;
  bm_one_call* const call = a.call;
  uint64_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = a.w[i];
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    // the call two ahead starts from "no hit" (no launch in flight uses it)
    bm_one_call* const r = a.reset;
    r->best = ~0ULL;
    r->found = 0;
    r->nhits = 0;
    __hip_atomic_store(&ctr->t0, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (kX) {
    if (blockIdx.x == 0) {
      if (threadIdx.x != 0) return;
      unsigned long long* const slot = a.xb + (size_t)a.xrow * BM_XSLOTS + a.xslot;
      uint64_t seen = ~0ULL;
      // bounded (2^26 polls, over a minute) so a lost column cannot keep the relay forever; the last
      // column then writes the result instead
      for (uint32_t spin = 0; spin < (1u << 26); ++spin) {
        const uint64_t v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v < seen) {
          atomicMin(&call->best, (unsigned long long)v);
          seen = v;
        }
        if ((__hip_atomic_load(&ctr->acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xfffu) >= a.nwg) break;
        __builtin_amdgcn_s_sleep(2);
      }
      const uint64_t old = __hip_atomic_fetch_add(&ctr->acc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((old & 0xfffu) == a.nwg) one_result<kX>(a, ctr, call, w, old + 1);
      return;
    }
  }
  bm_item it;
  it.start = a.start;
  it.count = a.count;
  it.obj = 0;
  it.chunk_base = 0;
  it.g0 = kX ? a.g0 : 0;
  it.gn = kX ? a.gn : a.nwg;
  it.nwg = a.nwg;
  it.xslot = kX ? a.xslot : BM_NO_XSLOT;
  it.pad = 0;
  const bm_swept r = sweep<kX, true>(it, 0, w, a.target, &call->best, &call->found, &ctr->queue, kX ? a.xb : nullptr,
                                     kX ? a.xrows : 0, call);
  if ((threadIdx.x & 63) != 0) return;
  bm_fold tot;
  if (!bm_fold_leave(r.done, r.cut, r.hit, tot)) return;
  // one device atomic per workgroup (bm_one_ctr.acc: trials << 31 | cut << 12 | workgroups); a release
  // only from a workgroup whose waves published hits, so the last workgroup's acquire sees them all
  const uint64_t add = ((uint64_t)tot.done << 31) | ((uint64_t)tot.cut << 12) | 1u;
  uint64_t old;
  if (tot.hits) old = __hip_atomic_fetch_add(&ctr->acc, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  else old = __hip_atomic_fetch_add(&ctr->acc, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the launch's workgroups: the columns, and with kX the relay
  if ((old & 0xfffu) != a.nwg - (kX ? 0u : 1u)) return;
  one_result<kX>(a, ctr, call, w, old + add);
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

hipError_t bm_launch_search1(hipStream_t st, const bm_one_args& a) {
  if (a.xb)
    hipLaunchKernelGGL(bm_search1_kernel<true>, dim3(a.nwg + 1), dim3(BM_BLOCK), 0, st, a);
  else
    hipLaunchKernelGGL(bm_search1_kernel<false>, dim3(a.nwg), dim3(BM_BLOCK), 0, st, a);
  return hipGetLastError();
}

int bm_search_resident_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bm_search_kernel<false>, BM_BLOCK, 0) != hipSuccess) return 0;
  return n;
}
