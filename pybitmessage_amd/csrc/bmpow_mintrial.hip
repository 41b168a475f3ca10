// bmpow_mintrial.hip -- the min-trial probe (gfx950): min over a nonce range of trial(n, ih) and
// the first nonce reaching it, for many (object, range) items in one launch.
//
// This is the size-independent minimality check of a search answer: n is the _doSafePoW answer
// (src/proofofwork.py:100-111) iff trial(n) <= target and min{trial(m) : 1 <= m < n} > target.
// It hashes every nonce of its range (no early exit, no target) and reduces instead of searching,
// so it shares the trial function with bm_search_kernel but none of its hit/exit logic: a search
// bug cannot hide behind the probe.  Layout is the search kernel's (bm_item list, one workgroup per
// column of an item, bmpow_layout.h); each workgroup writes one bm_minpart and the host reduces the
// parts per item.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

namespace {

__device__ __forceinline__ bool lex_less(uint64_t t1, uint64_t n1, uint64_t t2, uint64_t n2) {
  return t1 < t2 || (t1 == t2 && n1 < n2);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, mask);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), mask);
  return ((uint64_t)hi << 32) | lo;
}

}  // namespace

__global__ __launch_bounds__(BM_BLOCK) void bm_mintrial_kernel(const bm_obj* __restrict__ objs,
                                                               const bm_item* __restrict__ items,
                                                               uint32_t nitems, bm_minpart* __restrict__ parts) {
  const uint32_t b = blockIdx.x;
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  const bm_item it = items[lo];
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
  uint64_t blk = (uint64_t)it.g0 + (b - it.chunk_base);  // this workgroup's column (bmpow_layout.h)
  uint64_t bt = ~0ULL, bn = ~0ULL;  // no nonce of this lane (yet): sorts after every real pair
  if (blk < nblk) {
    const bm_obj* o = objs + it.obj;
    uint64_t ihw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ihw[i] = o->w[i];
    for (; blk < nblk; blk += it.gn) {
      const uint64_t j = blk * BM_BLOCK + threadIdx.x;
      const uint64_t nonce = it.start + j;
      const uint64_t tv = trial_of(ihw, nonce);
      if (j < it.count && tv < bt) {  // ascending nonces per lane: strict < keeps the first
        bt = tv;
        bn = nonce;
      }
    }
  }
  // wave reduction (64 lanes), then across the workgroup's waves through LDS
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t ot = shfl_xor64(bt, m), on = shfl_xor64(bn, m);
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

hipError_t bm_launch_mintrial(hipStream_t st, uint32_t nwg, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                              bm_minpart* parts) {
  hipLaunchKernelGGL(bm_mintrial_kernel, dim3(nwg), dim3(BM_BLOCK), 0, st, objs, items, nitems, parts);
  return hipGetLastError();
}
