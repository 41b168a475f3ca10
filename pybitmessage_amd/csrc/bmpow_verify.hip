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
// Launch wrapper (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bv_launch_pow(hipStream_t st, const bv_obj* objs, uint32_t n, const uint4* pool, uint64_t* pow_out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(bv_pow_kernel, dim3((n + BV_BLOCK - 1) / BV_BLOCK), dim3(BV_BLOCK), 0, st, objs, n, pool,
                     pow_out);
  return hipGetLastError();
}

