// bmpow_var.hip -- gfx950 search and min-trial kernels for an initialHash of any length other than
// 64 bytes (the reference's _doSafePoW hashes pack('>Q', nonce) + initialHash as given,
// src/proofofwork.py:100-111; every caller in the reference passes a 64-byte digest, which
// bm_search_kernel serves).
//
// Same execution model as bm_search_kernel (bmpow_kernels.hip): workgroups taking an item's blocks
// in order from its queue, atomicMin of hits into best[obj], early exit above the running minimum.
// Per object the message words come from the batch's var pool (bmsched::pack_var): block 0's
// W1..W15 are loaded once per workgroup (loop-invariant, so their sigma terms are hoisted out of
// the nonce loop), the K+W words of the further blocks are read per round with uniform loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

namespace {

__device__ __forceinline__ uint32_t item_of(const bm_item* __restrict__ items, uint32_t nitems, uint32_t b) {
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ bool lex_less(uint64_t t1, uint64_t n1, uint64_t t2, uint64_t n2) {
  return t1 < t2 || (t1 == t2 && n1 < n2);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, mask);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), mask);
  return ((uint64_t)hi << 32) | lo;
}

}  // namespace

__device__ __forceinline__ void search_var_column(const bm_obj* __restrict__ objs, const bm_item* __restrict__ items,
                                                  uint32_t nitems, unsigned long long* __restrict__ best,
                                                  uint32_t* __restrict__ found,
                                                  unsigned long long* __restrict__ trials_done,
                                                  unsigned long long* __restrict__ queue,
                                                  unsigned long long* __restrict__ xb, uint32_t xrows,
                                                  const uint64_t* __restrict__ vpool, uint32_t b) {
  const uint32_t li = item_of(items, nitems, b);
  const bm_item it = items[li];
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
  unsigned long long* bestp = best + it.obj;
  unsigned long long* qp = queue + li;
  __shared__ unsigned long long s_k[2];  // the item's block queue, as in bm_search_kernel (bmpow_kernels.h)
  if (threadIdx.x == 0) s_k[0] = atomicAdd(qp, 1ull);
  __syncthreads();
  uint64_t blk = bm_block_of(it, s_k[0]);
  if (blk >= nblk) return;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < it.start + blk * BM_BLOCK) return;
  const bm_obj* o = objs + it.obj;
  const uint64_t* m = vpool + o->vword;
  const uint32_t nb = o->nblk;
  const uint64_t target = o->target;
  uint64_t mw[16];
  mw[0] = 0;
#pragma unroll
  for (int i = 1; i < 16; ++i) mw[i] = m[i];
  uint32_t done = 0;
  for (uint32_t slot = 1;; slot ^= 1) {
    unsigned long long kn = 0;
    if (threadIdx.x == 0) kn = atomicAdd(qp, 1ull);
    const uint64_t off = blk * BM_BLOCK;
    const uint64_t first = it.start + off;
    const uint64_t nonce = first + threadIdx.x;
    const uint64_t tv = trial_var(mw, m + 16, nb, nonce);
    // the wave's smallest hit is its lowest hitting lane (consecutive nonces): one atomicMin per wave
    const uint64_t hits = __builtin_amdgcn_ballot_w64(off + threadIdx.x < it.count && tv <= target);
    if (hits) {
      const uint64_t wmin = first + (threadIdx.x & ~63u) + (uint64_t)__builtin_ctzll(hits);
      if ((threadIdx.x & 63) == 0) {
        const unsigned long long prev = atomicMin(bestp, (unsigned long long)wmin);
        __hip_atomic_store(found + it.obj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (xb && it.xslot != BM_NO_XSLOT) bm_publish(bestp, xb, it.xslot, xrows, prev < wmin ? prev : wmin);
      }
    }
    const uint64_t seen = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    done += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(off + threadIdx.x < it.count));  // this wave's
    if (threadIdx.x == 0) s_k[slot] = kn;
    __syncthreads();
    const uint64_t nxt = bm_block_of(it, s_k[slot]);
    if (nxt >= nblk || seen < it.start + nxt * BM_BLOCK) break;
    blk = nxt;
  }
  // every wave counts its own lanes (waves of one workgroup may leave at different blocks)
  if ((threadIdx.x & 63) == 0 && done) atomicAdd(trials_done, (unsigned long long)done);
}

// xb set (split windows): workgroup 0 is the relay and columns are workgroups 1.., as in
// bm_search_kernel<true>.
__global__ __launch_bounds__(BM_BLOCK) void bm_search_var_kernel(const bm_obj* __restrict__ objs,
                                                                 const bm_item* __restrict__ items,
                                                                 uint32_t nitems,
                                                                 unsigned long long* __restrict__ best,
                                                                 uint32_t* __restrict__ found,
                                                                 unsigned long long* __restrict__ trials_done,
                                                                 unsigned long long* __restrict__ queue,
                                                                 unsigned long long* __restrict__ xb,
                                                                 uint32_t xrow, uint32_t xrows,
                                                                 const uint64_t* __restrict__ vpool) {
  if (xb) {
    if (blockIdx.x == 0) {
      bm_relay(items, nitems, best, xb, xrow, trials_done + 1, (gridDim.x - 1) * (BM_BLOCK / 64));
      return;
    }
    search_var_column(objs, items, nitems, best, found, trials_done, queue, xb, xrows, vpool, blockIdx.x - 1);
    if ((threadIdx.x & 63) == 0) atomicAdd(trials_done + 1, 1ull);
  } else {
    search_var_column(objs, items, nitems, best, found, trials_done, queue, nullptr, 0, vpool, blockIdx.x);
  }
}

// Min-trial probe over var-form objects: bm_mintrial_kernel (bmpow_mintrial.hip) with trial_var.
__global__ __launch_bounds__(BM_BLOCK) void bm_mintrial_var_kernel(const bm_obj* __restrict__ objs,
                                                                   const bm_item* __restrict__ items,
                                                                   uint32_t nitems, bm_minpart* __restrict__ parts,
                                                                   const uint64_t* __restrict__ vpool) {
  const uint32_t b = blockIdx.x;
  const bm_item it = items[item_of(items, nitems, b)];
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
  uint64_t blk = (uint64_t)it.g0 + (b - it.chunk_base);
  uint64_t bt = ~0ULL, bn = ~0ULL;
  if (blk < nblk) {
    const bm_obj* o = objs + it.obj;
    const uint64_t* m = vpool + o->vword;
    const uint32_t nb = o->nblk;
    uint64_t mw[16];
    mw[0] = 0;
#pragma unroll
    for (int i = 1; i < 16; ++i) mw[i] = m[i];
    for (; blk < nblk; blk += it.gn) {
      const uint64_t j = blk * BM_BLOCK + threadIdx.x;
      const uint64_t nonce = it.start + j;
      const uint64_t tv = trial_var(mw, m + 16, nb, nonce);
      if (j < it.count && tv < bt) {
        bt = tv;
        bn = nonce;
      }
    }
  }
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    const uint64_t ot = shfl_xor64(bt, k), on = shfl_xor64(bn, k);
    if (lex_less(ot, on, bt, bn)) {
      bt = ot;
      bn = on;
    }
  }
  __shared__ uint64_t st[BM_BLOCK / 64], sn[BM_BLOCK / 64];
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    st[w] = bt;
    sn[w] = bn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < BM_BLOCK / 64; ++k)
      if (lex_less(st[k], sn[k], bt, bn)) {
        bt = st[k];
        bn = sn[k];
      }
    bm_minpart p;
    p.trial = bt;
    p.nonce = bn;
    parts[b] = p;
  }
}

hipError_t bm_launch_search_var(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items,
                                uint32_t nitems, unsigned long long* best, uint32_t* found,
                                unsigned long long* trials_done, unsigned long long* queue, const bm_xbound& xb,
                                const uint64_t* vpool) {
  hipLaunchKernelGGL(bm_search_var_kernel, dim3(nwg + (xb.table ? 1 : 0)), dim3(BM_BLOCK), 0, st, objs, items, nitems,
                     best, found, trials_done, queue, xb.table, xb.row, xb.rows, vpool);
  return hipGetLastError();
}

hipError_t bm_launch_mintrial_var(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items,
                                  uint32_t nitems, bm_minpart* parts, const uint64_t* vpool) {
  hipLaunchKernelGGL(bm_mintrial_var_kernel, dim3(nwg), dim3(BM_BLOCK), 0, st, objs, items, nitems, parts, vpool);
  return hipGetLastError();
}
