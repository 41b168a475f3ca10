// bmpow_var.hip -- gfx950 search and min-trial kernels for an initialHash of any length other than
// 64 bytes (the reference's _doSafePoW hashes pack('>Q', nonce) + initialHash as given,
// src/proofofwork.py:100-111; every caller in the reference passes a 64-byte digest, which
// bm_search_kernel serves).
//
// Same execution model as bm_search_kernel (bmpow_kernels.hip): one workgroup per chunk of an
// item's nonce window, atomicMin of hits into best[obj], early exit above the running minimum.
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

__global__ __launch_bounds__(BM_BLOCK) void bm_search_var_kernel(const bm_obj* __restrict__ objs,
                                                                 const bm_item* __restrict__ items,
                                                                 uint32_t nitems,
                                                                 unsigned long long* __restrict__ best,
                                                                 uint32_t* __restrict__ found,
                                                                 unsigned long long* __restrict__ trials_done,
                                                                 uint32_t iters,
                                                                 const uint64_t* __restrict__ vpool) {
  const uint32_t b = blockIdx.x;
  const uint64_t chunk = (uint64_t)BM_BLOCK * iters;
  const bm_item it = items[item_of(items, nitems, b)];
  const uint64_t off = (uint64_t)(b - it.chunk_base) * chunk;
  if (off >= it.count) return;
  const uint64_t cnt = (it.count - off < chunk) ? (it.count - off) : chunk;
  const uint64_t first = it.start + off;
  unsigned long long* bestp = best + it.obj;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < first) return;
  const bm_obj* o = objs + it.obj;
  const uint64_t* m = vpool + o->vword;
  const uint32_t nblk = o->nblk;
  const uint64_t target = o->target;
  uint64_t mw[16];
  mw[0] = 0;
#pragma unroll
  for (int i = 1; i < 16; ++i) mw[i] = m[i];
  uint32_t done = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    const uint64_t base = (uint64_t)i * BM_BLOCK;
    if (base >= cnt) break;
    const uint64_t seen = __hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t j = base + threadIdx.x;
    const uint64_t nonce = first + j;
    const uint64_t tv = trial_var(mw, m + 16, nblk, nonce);
    if (j < cnt && tv <= target) {
      atomicMin(bestp, (unsigned long long)nonce);
      __hip_atomic_store(found + it.obj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    done += (cnt - base < BM_BLOCK) ? (uint32_t)(cnt - base) : BM_BLOCK;
    if (seen < first + base + BM_BLOCK) break;
  }
  if (threadIdx.x == 0) atomicAdd(trials_done, (unsigned long long)done);
}

// Min-trial probe over var-form objects: bm_mintrial_kernel (bmpow_mintrial.hip) with trial_var.
__global__ __launch_bounds__(BM_BLOCK) void bm_mintrial_var_kernel(const bm_obj* __restrict__ objs,
                                                                   const bm_item* __restrict__ items,
                                                                   uint32_t nitems, bm_minpart* __restrict__ parts,
                                                                   uint32_t iters,
                                                                   const uint64_t* __restrict__ vpool) {
  const uint32_t b = blockIdx.x;
  const uint64_t chunk = (uint64_t)BM_BLOCK * iters;
  const bm_item it = items[item_of(items, nitems, b)];
  const uint64_t off = (uint64_t)(b - it.chunk_base) * chunk;
  uint64_t bt = ~0ULL, bn = ~0ULL;
  if (off < it.count) {
    const uint64_t cnt = (it.count - off < chunk) ? (it.count - off) : chunk;
    const uint64_t first = it.start + off;
    const bm_obj* o = objs + it.obj;
    const uint64_t* m = vpool + o->vword;
    const uint32_t nblk = o->nblk;
    uint64_t mw[16];
    mw[0] = 0;
#pragma unroll
    for (int i = 1; i < 16; ++i) mw[i] = m[i];
    for (uint32_t i = 0; i < iters; ++i) {
      const uint64_t j = (uint64_t)i * BM_BLOCK + threadIdx.x;
      if ((uint64_t)i * BM_BLOCK >= cnt) break;
      const uint64_t nonce = first + j;
      const uint64_t tv = trial_var(mw, m + 16, nblk, nonce);
      if (j < cnt && tv < bt) {
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

hipError_t bm_launch_search_var(hipStream_t st, uint32_t nchunks, uint32_t iters, const bm_obj* objs,
                                const bm_item* items, uint32_t nitems, unsigned long long* best, uint32_t* found,
                                unsigned long long* trials_done, const uint64_t* vpool) {
  hipLaunchKernelGGL(bm_search_var_kernel, dim3(nchunks), dim3(BM_BLOCK), 0, st, objs, items, nitems, best, found,
                     trials_done, iters, vpool);
  return hipGetLastError();
}

hipError_t bm_launch_mintrial_var(hipStream_t st, uint32_t nchunks, uint32_t iters, const bm_obj* objs,
                                  const bm_item* items, uint32_t nitems, bm_minpart* parts, const uint64_t* vpool) {
  hipLaunchKernelGGL(bm_mintrial_var_kernel, dim3(nchunks), dim3(BM_BLOCK), 0, st, objs, items, nitems, parts, iters,
                     vpool);
  return hipGetLastError();
}
