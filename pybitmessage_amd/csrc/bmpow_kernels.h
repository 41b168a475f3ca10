// bmpow_kernels.h -- device data layout shared by the kernels and the host scheduler.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_layout.h"
#include "secp256k1_dev.h"

hipError_t bv_launch_pow(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out);
hipError_t bv_launch_pow_binned(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out,
                                const uint32_t* bins, uint32_t nbins);

// The cross-shard bound as a launch sees it: the table (host-pinned, coherent, mapped; null when the
// step splits no window), this shard's row and the number of rows.
struct bm_xbound {
  unsigned long long* table = nullptr;
  uint32_t row = 0, rows = 0;
};

// Publish a hit of a split window: store this device's running minimum into the window's slot of
// EVERY shard's row (plain system-scope vector stores, no PCIe atomics; a hit is rare, so the S stores
// are too), then re-read the device minimum and store again while it is lower, so the last writer
// leaves a value no larger than its device's minimum when stores of two hits cross.  Any value stored
// is a real hit of the window, so a stale larger one only stops fewer columns.
__device__ __forceinline__ void bm_publish(unsigned long long* bestp, unsigned long long* xb, uint32_t xslot,
                                           uint32_t xrows, uint64_t v) {
  for (;;) {
    for (uint32_t r = 0; r < xrows; ++r)
      __hip_atomic_store(xb + (size_t)r * BM_XSLOTS + xslot, (unsigned long long)v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t now = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (now >= v) break;
    v = now;
  }
}

// The launch's relay of the cross-shard bound (workgroup 0 of a launch with split windows; one wave):
// while the launch's columns run, it polls this shard's row of the table -- one system-scope load per
// split window every few microseconds, not one per column and block -- and folds what the other shards
// published into the device's own running minimum (atomicMin on best[obj]), which every column already
// reads once per block from L2.  A value it folds in is a real hit of the window: the columns above it
// stop, and the found[] flag stays the device's own, so the step's results are unchanged.  Exit: every
// column wave has finished (cols_done, counted by each wave of the column workgroups as it leaves), or
// 2^24 polls.
__device__ __forceinline__ void bm_relay(const bm_item* __restrict__ items, uint32_t nitems,
                                         unsigned long long* __restrict__ best, unsigned long long* xb,
                                         uint32_t xrow, unsigned long long* cols_done, uint32_t ncols) {
  if (threadIdx.x >= 64) return;
  uint64_t seen = ~0ULL;  // lane k's last folded value for item k (k < 64)
  for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
    if (__hip_atomic_load(cols_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ncols) break;
    for (uint32_t k = threadIdx.x; k < nitems; k += 64) {
      const bm_item& it = items[k];
      if (it.xslot == BM_NO_XSLOT) continue;
      const uint64_t v = __hip_atomic_load(xb + (size_t)xrow * BM_XSLOTS + it.xslot, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (v < seen || k >= 64) {
        atomicMin(best + it.obj, (unsigned long long)v);
        if (k < 64) seen = v;
      }
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// A workgroup's totals at the end of its sweep (the single-object kernel).  Its waves leave at
// different blocks (a wave that saw a hit stops while a sibling may go on for a block), so they cannot
// meet at a barrier: each wave adds its counts to the workgroup's LDS fold as it leaves, and the last
// one to leave carries the workgroup's totals -- one device atomic per workgroup at the end of a launch
// instead of two per wave.  A C1 launch lasts 1.7 ms and drains in ~20 us, into which 8,192 atomics on
// two addresses (~100 us at 83 M atomics/s) would not fit: the kernel's C1 span fell from 1.775 to
// 1.70 ms with the fold (profiles/r04/eng7/).
struct bm_fold {
  uint32_t done;  // trials hashed
  uint32_t cut;   // lanes whose block skipped its second compression
  uint32_t hits;  // waves that published a hit
  uint32_t left;  // waves that have left
};
__device__ __forceinline__ bm_fold& bm_fold_lds() {
  __shared__ bm_fold f;
  return f;
}
// Thread 0, before the sweep's first barrier.
__device__ __forceinline__ void bm_fold_init() {
  bm_fold& f = bm_fold_lds();
  f.done = 0;
  f.cut = 0;
  f.hits = 0;
  f.left = 0;
}
// Lane 0 of each wave as it leaves; true in the workgroup's last wave, with the totals in tot.
__device__ __forceinline__ bool bm_fold_leave(uint32_t done, uint32_t cut, uint32_t hit, bm_fold& tot) {
  bm_fold& f = bm_fold_lds();
  if (done) __hip_atomic_fetch_add(&f.done, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (cut) __hip_atomic_fetch_add(&f.cut, cut, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (hit) __hip_atomic_fetch_add(&f.hits, hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  // acq_rel: the last wave sees the others' counts (and their hits' memory effects at workgroup scope)
  if (__hip_atomic_fetch_add(&f.left, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) != BM_BLOCK / 64 - 1)
    return false;
  tot.done = __hip_atomic_load(&f.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  tot.cut = __hip_atomic_load(&f.cut, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  tot.hits = __hip_atomic_load(&f.hits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return true;
}

// The block queue of a work item (round 3).  A static column layout (column c hashing blocks c,
// c + gn, ...) keeps the columns in step only while every column progresses at the same rate, and
// they do not: the SIMD's arbiter favours its older waves, so of five column workgroups sharing a
// SIMD the oldest runs several times faster than the youngest.  A lone C1 object on one shard
// (1,280 columns) hashed 29 M trials for its 10.9 M useful, and 62.7 M with 1,024 columns
// (profiles/r03/c1_columns_static.jsonl): the column holding the answer lagged dozens of rows behind the
// fast ones.  So an item's workgroups now take its blocks IN ORDER from a per-item counter
// (queue[item], zeroed before each launch): the k-th block taken is the k-th block of the item's
// own columns, row by row, and the hashed set is always a prefix of the item's blocks plus the
// blocks in flight, however unevenly the workgroups run.  A workgroup fetches its next block while
// it hashes the current one (lane 0's atomicAdd, ~1 per 256 trials: 26 M/s device-wide for one
// item, against 83 M/s measured for one address, profiles/r03/atomic_rate.jsonl) and shares it
// through LDS at one barrier per block.
// A window on one shard (every item with gn == nwg has g0 == 0) takes its blocks as they come; only a
// window split over shards maps through its columns (a uniform 64-bit division, once per block).
__device__ __forceinline__ uint64_t bm_block_of(const bm_item& it, uint64_t k) {
  if (it.gn == it.nwg) return k;
  const uint64_t row = k / it.nwg;
  return row * it.gn + it.g0 + (k - row * it.nwg);
}

hipError_t bm_launch_search(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                            unsigned long long* best, uint32_t* found, unsigned long long* trials_done,
                            unsigned long long* queue, const bm_xbound& xb);
// trials_done points at two counters: [0] trials hashed, [1] column waves finished (the relay's
// exit; both zeroed before each launch).  With xb.table set, the grid is nwg + 1 workgroups (the relay).
// workgroups of bm_search_kernel resident per CU (its occupancy): the columns a shard's window
// gets at most, so a sweep is on the chip at once
int bm_search_resident_per_cu();
// the single-object kernel of run() (bm_one_args, bmpow_layout.h): grid a.nwg
hipError_t bm_launch_search1(hipStream_t st, const bm_one_args& a);
hipError_t bm_launch_search_var(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items,
                                uint32_t nitems, unsigned long long* best, uint32_t* found,
                                unsigned long long* trials_done, unsigned long long* queue, const bm_xbound& xb,
                                const uint64_t* vpool);
// vpool: the batch's var pool (may be null when no object of the launch is var-form)
// Writes each item's result (best/found are left as they are: they persist across the launches of a
// stream); res[nitems].nonce = trials[0] (the step's trial count, so one copy brings both home).
hipError_t bm_launch_resolve(hipStream_t st, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                             unsigned long long* best, uint32_t* found, bm_result* res,
                             const uint64_t* vpool, const unsigned long long* trials);
// objs[slots[i]] = recs[i], best = UINT64_MAX, found = 0 (recs, slots: pinned host memory)
hipError_t bm_launch_slots_init(hipStream_t st, bm_obj* objs, unsigned long long* best, uint32_t* found,
                                const bm_obj* recs, const uint32_t* slots, uint32_t n);
hipError_t bm_launch_mintrial(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                              bm_minpart* parts);
hipError_t bm_launch_mintrial_var(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items,
                                  uint32_t nitems, bm_minpart* parts, const uint64_t* vpool);
hipError_t bm_launch_trials(hipStream_t st, const bm_obj* obj, const uint64_t* nonces, uint64_t n,
                            uint64_t* out, const uint64_t* vpool);

// RIPE-prefix address search (ar_*, bmpow_addr.hip).  Parameters are uniform per search.
struct ar_params {
  uint64_t mid[8];     // SHA-512 state after the key seed's full 128-byte blocks (device-written)
  uint64_t tmpl[32];   // the seed's tail bytes (tail_len of them) as big-endian words, zero elsewhere
  uint64_t total_len;  // key-seed bytes (passphrase, or the random seed)
  uint32_t tail_len;   // total_len % 128
  uint32_t null_bytes; // leading zero bytes demanded of the ripe
  uint32_t mode;       // 0: deterministic (keys from 2k, 2k+1); 1: fixed signing key, encryption key from k
  uint32_t pad;
  ec::ge pub_s;        // mode 1: the signing public key (device-written)
};

struct ar_result {
  uint64_t k;
  uint64_t priv_s[4], priv_e[4];  // 32-byte private keys as big-endian words
  ec::ge pub_s, pub_e;
  uint32_t ripe[5];               // RIPEMD-160 state words (bytes little-endian)
  uint32_t ok;
};

size_t ar_table_entries(int wbits);  // allocation size (entries) of the comb of width wbits
hipError_t ar_launch_table(hipStream_t st, ec::ge* table, int wbits);
// mode: prm->mode (sizes the grid: 2 tries per lane in mode 0, 4 in mode 1)
hipError_t ar_launch_search(hipStream_t st, const ar_params* prm, uint32_t mode, const ec::ge* table, int wbits,
                            uint64_t start, uint32_t count, unsigned long long* best);
hipError_t ar_launch_resolve(hipStream_t st, const ar_params* prm, const ec::ge* table, int wbits, uint64_t k,
                             ar_result* out);
hipError_t ar_launch_pubkeys(hipStream_t st, const uint64_t* privs, uint32_t n, const ec::ge* table, ec::ge* pubs,
                             uint32_t* ok);
hipError_t ar_launch_fe_probe(hipStream_t st, int op, const ec::fe* a, const ec::fe* b, ec::fe* out, uint32_t n);
hipError_t ar_launch_midstate(hipStream_t st, const uint8_t* pass, uint64_t nfull, uint64_t* mid);
