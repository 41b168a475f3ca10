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

// Running minimum hit of an item's object as a column sees it: the device's own (agent scope: other
// CUs' atomics through L2), and for a window split over shards every shard's published hit (system
// scope: host-pinned memory, written by other devices).  Every value read is a real hit of the window
// or UINT64_MAX, so it only ever stops columns above an answer.
__device__ __forceinline__ uint64_t bm_bound(unsigned long long* bestp, bool xs, unsigned long long* xb,
                                             uint32_t xslot, uint32_t xrows) {
  uint64_t m = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (xs) {
    for (uint32_t r = 0; r < xrows; ++r) {
      const uint64_t v = __hip_atomic_load(xb + (size_t)r * BM_XSLOTS + xslot, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
      m = v < m ? v : m;
    }
  }
  return m;
}

// Publish this shard's running minimum of a split window to its slot of the cross-shard bound: a plain
// system-scope store (no PCIe atomics), then re-read the device minimum and store again while it is
// lower, so the last writer leaves the true minimum even when stores of two hits cross.
__device__ __forceinline__ void bm_publish(unsigned long long* bestp, unsigned long long* slot, uint64_t v) {
  for (;;) {
    __hip_atomic_store(slot, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t now = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (now >= v) break;
    v = now;
  }
}

hipError_t bm_launch_search(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                            unsigned long long* best, uint32_t* found, unsigned long long* trials_done,
                            const bm_xbound& xb);
// workgroups of bm_search_kernel resident per CU (its occupancy): the columns a shard's window
// gets at most, so a sweep is on the chip at once
int bm_search_resident_per_cu();
hipError_t bm_launch_search_var(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items,
                                uint32_t nitems, unsigned long long* best, uint32_t* found,
                                unsigned long long* trials_done, const bm_xbound& xb, const uint64_t* vpool);
// vpool: the batch's var pool (may be null when no object of the launch is var-form)
hipError_t bm_launch_resolve(hipStream_t st, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                             const unsigned long long* best, const uint32_t* found, bm_result* res,
                             const uint64_t* vpool);
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
