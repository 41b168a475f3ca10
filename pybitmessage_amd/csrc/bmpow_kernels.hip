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

namespace bm {

// ---------------------------------------------------------------------------------------
// Generic fully-unrolled SHA-512 rounds.  State slot of a at round T is (-T) & 7; every
// index below is a compile-time constant after template expansion, so s[] and w[] live in
// VGPR/SGPR pairs (verified: no scratch in the ISA).
// ---------------------------------------------------------------------------------------
template <int T>
BM_DEV void round_step(uint64_t (&s)[8], uint64_t (&w)[16]) {
  constexpr int A = (8 - (T & 7)) & 7;
  constexpr int B = (A + 1) & 7, C = (A + 2) & 7, D = (A + 3) & 7;
  constexpr int E = (A + 4) & 7, F = (A + 5) & 7, G = (A + 6) & 7, H = (A + 7) & 7;
  if constexpr (T >= 16) {
    // grouped so the terms that do not depend on the nonce (per-object or compile-time)
    // are summed first and hoisted out of the nonce loop by LICM
    w[T & 15] = (w[(T - 7) & 15] + sig0(w[(T - 15) & 15]) + w[(T - 16) & 15]) + sig1(w[(T - 2) & 15]);
  }
  const uint64_t t1 = s[H] + Sig1(s[E]) + Ch(s[E], s[F], s[G]) + (K(T) + w[T & 15]);
  s[D] += t1;
  s[H] = t1 + Sig0(s[A]) + Maj(s[A], s[B], s[C]);
}

template <int T, int END>
BM_DEV void rounds(uint64_t (&s)[8], uint64_t (&w)[16]) {
  if constexpr (T < END) {
    round_step<T>(s, w);
    rounds<T + 1, END>(s, w);
  }
}

// trial(n, ih) with ih given as 8 big-endian words.  Round 0 of each block is folded:
// from the IV with W0 unknown, a1 = W0 + A1C and e1 = W0 + E1C.
BM_DEV uint64_t trial_of(const uint64_t (&ihw)[8], uint64_t nonce) {
  uint64_t w[16];
  w[0] = nonce;
#pragma unroll
  for (int i = 0; i < 8; ++i) w[1 + i] = ihw[i];
  w[9] = PAD;
#pragma unroll
  for (int i = 10; i < 15; ++i) w[i] = 0;
  w[15] = 72 * 8;
  // state after the folded round 0 (round 1 has A = 7: a=s7 b=s0 c=s1 d=s2 e=s3 f=s4 g=s5 h=s6)
  uint64_t s[8] = {IV(0), IV(1), IV(2), nonce + E1C, IV(4), IV(5), IV(6), nonce + A1C};
  rounds<1, 80>(s, w);
  // after 80 rounds A = 0: s[i] holds a..h in order
  uint64_t w2[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w2[i] = s[i] + IV(i);
  w2[8] = PAD;
#pragma unroll
  for (int i = 9; i < 15; ++i) w2[i] = 0;
  w2[15] = 64 * 8;
  uint64_t s2[8] = {IV(0), IV(1), IV(2), w2[0] + E1C, IV(4), IV(5), IV(6), w2[0] + A1C};
  rounds<1, 80>(s2, w2);
  return s2[0] + IV(0);
}

// One SHA-512 compression of a runtime block into the chaining state h.
BM_DEV void compress(uint64_t (&h)[8], uint64_t (&w)[16]) {
  uint64_t s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = h[i];
  rounds<0, 80>(s, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] += s[i];
}

// Big-endian 64-bit word from a little-endian 16-byte load: bytes b0..b3 are in x, b4..b7 in y.
BM_DEV uint64_t be64(uint32_t x, uint32_t y) { return mk64(__builtin_bswap32(y), __builtin_bswap32(x)); }

}  // namespace bm

using namespace bm;

// ---------------------------------------------------------------------------------------
// Search kernel.
// ---------------------------------------------------------------------------------------
#ifndef BM_MIN_WAVES
#define BM_MIN_WAVES 1
#endif
#if BM_MIN_WAVES > 0
#define BM_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(BM_MIN_WAVES, 8)))
#else
#define BM_WAVES_ATTR
#endif
__global__ __launch_bounds__(BM_BLOCK) BM_WAVES_ATTR void bm_search_kernel(const bm_obj* __restrict__ objs,
                                                             const bm_item* __restrict__ items,
                                                             uint32_t nitems,
                                                             unsigned long long* __restrict__ best,
                                                             unsigned long long* __restrict__ trials_done) {
  const uint32_t b = blockIdx.x;
  // largest item index with chunk_base <= b (items sorted by chunk_base, uniform search)
  uint32_t lo = 0, hi = nitems;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (items[mid].chunk_base <= b) lo = mid; else hi = mid;
  }
  const bm_item it = items[lo];
  const uint64_t off = (uint64_t)(b - it.chunk_base) * BM_CHUNK;
  if (off >= it.count) return;
  const uint64_t cnt = (it.count - off < BM_CHUNK) ? (it.count - off) : BM_CHUNK;
  const uint64_t first = it.start + off;
  unsigned long long* bestp = best + it.obj;
  if (__hip_atomic_load(bestp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < first) return;

  const bm_obj* o = objs + it.obj;
  uint64_t ihw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ihw[i] = o->w[i];
  const uint64_t target = o->target;

  uint32_t done = 0;
  for (uint32_t i = 0; i < BM_ITERS; ++i) {
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
  if (n != ~0ULL) {
    uint64_t ihw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ihw[i] = objs[obj].w[i];
    r.trial = trial_of(ihw, n);
  }
  res[k] = r;
}

// Trial values for an arbitrary list of nonces of one object (parity probe / verification).
__global__ __launch_bounds__(BM_BLOCK) void bm_trials_kernel(const bm_obj* __restrict__ obj,
                                                             const uint64_t* __restrict__ nonces,
                                                             uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * BM_BLOCK + threadIdx.x;
  if (k >= n) return;
  uint64_t ihw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ihw[i] = obj->w[i];
  out[k] = trial_of(ihw, nonces[k]);
}

// ---------------------------------------------------------------------------------------
// Receive-side PoW value, reference src/protocol.py:280-282:
//   POW = BE64(SHA512(SHA512(object[0:8] || SHA512(object[8:])))[0:8])
// One lane per object.  The inner SHA512(object[8:]) runs over the host-padded blocks of the
// pool (16-B loads, byte-swapped into the big-endian schedule words); its digest words are the
// initialHash words of the trial function, so the outer double hash is trial_of(H, nonce).
// Integer-VALU bound: ~3,300 VALU instructions per 128-B block, 0 bytes re-read.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(BV_BLOCK) void bv_pow_kernel(const bv_obj* __restrict__ objs, uint32_t n,
                                                          const uint4* __restrict__ pool,
                                                          uint64_t* __restrict__ pow_out) {
  const uint32_t k = blockIdx.x * BV_BLOCK + threadIdx.x;
  if (k >= n) return;
  const bv_obj o = objs[k];
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = IV(i);
  const uint4* p = pool + (uint64_t)o.blk * 8;
  for (uint32_t b = 0; b < o.nblk; ++b, p += 8) {
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 v = p[j];
      w[2 * j] = be64(v.x, v.y);
      w[2 * j + 1] = be64(v.z, v.w);
    }
    compress(h, w);
  }
  pow_out[k] = trial_of(h, o.nonce);
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bm_launch_search(hipStream_t st, uint32_t nchunks, const bm_obj* objs, const bm_item* items,
                            uint32_t nitems, unsigned long long* best, unsigned long long* trials_done) {
  hipLaunchKernelGGL(bm_search_kernel, dim3(nchunks), dim3(BM_BLOCK), 0, st, objs, items, nitems, best,
                     trials_done);
  return hipGetLastError();
}

hipError_t bm_launch_resolve(hipStream_t st, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                             const unsigned long long* best, bm_result* res) {
  const uint32_t bs = 64;
  hipLaunchKernelGGL(bm_resolve_kernel, dim3((nitems + bs - 1) / bs), dim3(bs), 0, st, objs, items, nitems,
                     best, res);
  return hipGetLastError();
}

hipError_t bv_launch_pow(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(bv_pow_kernel, dim3((n + BV_BLOCK - 1) / BV_BLOCK), dim3(BV_BLOCK), 0, st, objs, n, pool,
                     pow_out);
  return hipGetLastError();
}

hipError_t bm_launch_trials(hipStream_t st, const bm_obj* obj, const uint64_t* nonces, uint64_t n,
                            uint64_t* out) {
  const uint64_t nb = (n + BM_BLOCK - 1) / BM_BLOCK;
  hipLaunchKernelGGL(bm_trials_kernel, dim3((uint32_t)nb), dim3(BM_BLOCK), 0, st, obj, nonces, n, out);
  return hipGetLastError();
}
