// bmpow_verify.hip -- receive-side PoW verification kernel (gfx950).
//
// Reference: src/protocol.py:258-286 (isProofOfWorkSufficient), called per received object from
// src/network/bmobject.py:71-76.  Host side: bmpow_vbatch_* / bmpow_verify_batch in bmpow_host.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

// ---------------------------------------------------------------------------------------
// Receive-side PoW value, reference src/protocol.py:280-282:
//   POW = BE64(SHA512(SHA512(object[0:8] || SHA512(object[8:])))[0:8])
// One lane per object.  The inner SHA512(object[8:]) runs over the host-padded blocks of the
// pool (16-B loads, byte-swapped into the big-endian schedule words); its digest words are the
// initialHash words of the trial function, so the outer double hash is trial_of(H, nonce).
// Integer-VALU bound: ~3,300 VALU instructions per 128-B block, 0 bytes re-read.
// ---------------------------------------------------------------------------------------
//
// One copy of the compression body serves the whole object: the loop runs nblk + 2 blocks, the
// payload's from the pool, then the trial's two (trial_of's blocks, built in registers by selects:
// the state restarts at the IV and the previous digest becomes the message).  The specialised
// trial (trial_of, ~6,200 VALU against ~6,700 here; BV_TWO_BODY) puts two more unrolled
// compressions beside the loop's, 83 KB of code against 29 KB, and measured slower in the binned
// kernel: 1.17 vs 1.06 ms for the 500k-object flood (same box; profiles/r02/verify_binned_ab.txt).
#ifdef BV_TWO_BODY
// A/B variant: the payload loop, then the specialised trial_of
BM_DEV uint64_t pow_of(const bv_obj& o, const uint4* __restrict__ pool) {
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
  return trial_of(h, o.nonce);
}
#else
BM_DEV uint64_t pow_of(const bv_obj& o, const uint4* __restrict__ pool) {
  uint64_t h[8], d[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = IV(i), d[i] = 0;
  const uint4* base = pool + (uint64_t)o.blk * 8;
  const uint32_t nb = o.nblk;
  for (uint32_t b = 0; b < nb + 2; ++b) {
    const bool pay = b < nb, t1 = b == nb;
    const uint4* p = base + (uint64_t)(pay ? b : nb - 1) * 8;  // never past the object's blocks
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 v = p[j];
      w[2 * j] = be64(v.x, v.y);
      w[2 * j + 1] = be64(v.z, v.w);
    }
    if (!pay) {
      // trial block 1: nonce || payload digest || padding (72 B); block 2: digest 1 || padding (64 B)
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = h[i], h[i] = IV(i);
      w[0] = t1 ? o.nonce : d[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) w[i] = t1 ? d[i - 1] : d[i];
      w[8] = t1 ? d[7] : PAD;
      w[9] = t1 ? PAD : 0;
#pragma unroll
      for (int i = 10; i < 15; ++i) w[i] = 0;
      w[15] = t1 ? 72 * 8 : 64 * 8;
    }
    compress(h, w);
  }
  return h[0];
}
#endif

// One wave per object group of BV_BLOCK lanes, the groups dispatched in sorted order (small floods).
__global__ __launch_bounds__(BV_BLOCK) void bv_pow_kernel(const bv_obj* __restrict__ objs, uint32_t n,
                                                          const uint4* __restrict__ pool,
                                                          uint64_t* __restrict__ pow_out) {
  const uint32_t k = blockIdx.x * BV_BLOCK + threadIdx.x;
  if (k >= n) return;
  pow_out[k] = pow_of(objs[k], pool);
}

// Balanced floods.  A wave runs as long as its longest lane, so a SIMD's time is at least the sum
// over the waves it holds, and at least the latency of its longest wave: one wave alone issues a
// VALU instruction every ~5 clocks (7.0 us per block; tools/verify_uniform.py), and shares the SIMD
// fairly with the others (~4 x slower beside three busy waves).  In a 500k flood a 16 KB message
// group is ~85 % of a SIMD's share of the work, so the SIMD's time is that group's latency.  Here
// the host deals the groups to one bin per SIMD, longest first to the least-loaded bin
// (bmsched::plan_bins), so each SIMD gets one long group plus short ones; one workgroup per CU (its
// LDS request admits no second one; tools/hwid_probe.hip: 4 waves per SIMD id in every workgroup)
// runs 16 waves, each taking groups from the bin of the SIMD it runs on (HW_ID.SIMD_ID), then from
// the CU's other bins once its own is empty (so every bin drains whatever the placement: the SIMD
// id only steers the balance).  The wave holding a bin's first (longest) group raises its issue
// priority, so the short groups fill the long one's gaps instead of slowing it down.  Same box,
// 500k-object flood: 1.06 ms against 1.25 ms (the sorted one-wave-per-group launch) and 1.26 ms
// (binned without the priority).
constexpr uint32_t kBvBinnedLdsWords = (96u << 10) / 4;  // > half of the CU's 160 KiB

__global__ __launch_bounds__(BV_BINNED_WG) void bv_pow_binned_kernel(const bv_obj* __restrict__ objs, uint32_t n,
                                                                     const uint4* __restrict__ pool,
                                                                     uint64_t* __restrict__ pow_out,
                                                                     const uint32_t* __restrict__ bins,
                                                                     uint32_t nbins) {
  __shared__ uint32_t heads[kBvBinnedLdsWords];  // [0..3]: next group of each of the CU's 4 bins
  if (threadIdx.x < 4) heads[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  // s_getreg_b32 hwreg(HW_REG_HW_ID, 4, 2): SIMD_ID of this wave
  const uint32_t simd = __builtin_amdgcn_s_getreg((1u << 11) | (4u << 6) | 4u) & 3u;
  const uint32_t* list = bins + nbins + 1;
  for (uint32_t t = 0; t < 4; ++t) {
    const uint32_t s = (simd + t) & 3u;
    const uint32_t b = blockIdx.x * 4 + s;
    const uint32_t lo = bins[b], cnt = bins[b + 1] - lo;
    for (;;) {
      uint32_t idx = 0;
      if (lane == 0) idx = atomicAdd(&heads[s], 1u);
      idx = __builtin_amdgcn_readfirstlane(idx);
      if (idx >= cnt) break;
      const uint32_t k = list[lo + idx] * BV_BLOCK + lane;
#ifndef BV_NO_PRIO
      // the bin's first group is its longest: the SIMD's critical path, so it gets the issue priority
      if (idx == 0) __builtin_amdgcn_s_setprio(3);
#endif
      if (k < n) pow_out[k] = pow_of(objs[k], pool);
#ifndef BV_NO_PRIO
      if (idx == 0) __builtin_amdgcn_s_setprio(0);
#endif
    }
  }
}

// ---------------------------------------------------------------------------------------
// Launch wrapper (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bv_launch_pow(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(bv_pow_kernel, dim3((n + BV_BLOCK - 1) / BV_BLOCK), dim3(BV_BLOCK), 0, st, objs, n, pool,
                     pow_out);
  return hipGetLastError();
}

hipError_t bv_launch_pow_binned(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out,
                                const uint32_t* bins, uint32_t nbins) {
  if (n == 0) return hipSuccess;
  if (nbins == 0 || nbins % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bv_pow_binned_kernel, dim3(nbins / 4), dim3(BV_BINNED_WG), 0, st, objs, n, pool, pow_out, bins,
                     nbins);
  return hipGetLastError();
}

