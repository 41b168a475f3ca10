// bmpow_trials.hip -- the small trial kernels beside the search (gfx950): bm_resolve_kernel
// (winning trial values after a step) and bm_trials_kernel (trial values of arbitrary nonces, the
// parity probe).  A translation unit of their own, so scheduler and flag experiments on the search
// kernel (tools/cmp_variants.sh) never touch them -- the iterative-ILP scheduler, for one, crashes
// the register allocator on trial_ool (ROCm 7.2 clang) once SHR64 is an inline-asm v_lshrrev_b64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "sha512_dev.h"

using namespace bm;

// Out-of-line trial for the small kernels (resolve, trials): one compiled copy of the ~6,500-
// instruction body instead of one inlined per kernel (the search kernel keeps its own inline
// copy, with the per-object words hoisted out of its nonce loop).
__device__ __noinline__ uint64_t trial_ool(uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3, uint64_t w4,
                                           uint64_t w5, uint64_t w6, uint64_t w7, uint64_t nonce) {
  const uint64_t ihw[8] = {w0, w1, w2, w3, w4, w5, w6, w7};
  return trial_of(ihw, nonce);
}

// The same for a var-form object (an initialHash of another length, bmpow_var.hip).
__device__ __noinline__ uint64_t trial_var_ool(const uint64_t* __restrict__ m, uint32_t nblk, uint64_t nonce) {
  uint64_t mw[16];
  mw[0] = 0;
#pragma unroll
  for (int i = 1; i < 16; ++i) mw[i] = m[i];
  return trial_var(mw, m + 16, nblk, nonce);
}

__device__ uint64_t trial_obj(const bm_obj* o, uint64_t nonce, const uint64_t* vpool) {
  if (o->ihlen != BM_IH_MAIN) return trial_var_ool(vpool + o->vword, o->nblk, nonce);
  return trial_ool(o->w[0], o->w[1], o->w[2], o->w[3], o->w[4], o->w[5], o->w[6], o->w[7], nonce);
}

// For each launched item whose object has a hit, recompute the trial value at the winning
// nonce (one thread per item).  res[k] = {nonce, trial, found = 1} or {UINT64_MAX, 0, found = 0}:
// the found flag, not the nonce, says whether there is a hit (2^64-1 is a legal answer).  res[k].pad =
// the units item k's block queue handed out (trials[2 + k], clipped to 32 bits): the host's estimate of
// the trials hashed past the answers (bmsched::WasteStats).
__global__ void bm_resolve_kernel(const bm_obj* __restrict__ objs, const bm_item* __restrict__ items,
                                  uint32_t nitems, unsigned long long* __restrict__ best,
                                  uint32_t* __restrict__ found, bm_result* __restrict__ res,
                                  const uint64_t* __restrict__ vpool,
                                  const unsigned long long* __restrict__ trials) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 0) {  // the step's trial count rides home after the results (one copy)
    bm_result t;
    t.nonce = trials[0];
    t.trial = 0;
    t.found = 0;
    t.pad = 0;
    res[nitems] = t;
  }
  if (k >= nitems) return;
  const uint32_t obj = items[k].obj;  // at most one item per object in a shard's step
  bm_result r;
  r.nonce = best[obj];
  r.trial = 0;
  r.found = found[obj];
  const unsigned long long taken = trials[2 + k];
  r.pad = taken > 0xffffffffULL ? 0xffffffffu : (uint32_t)taken;
  if (r.found) r.trial = trial_obj(objs + obj, r.nonce, vpool);
  res[k] = r;
  // best[] / found[] are left as they are: a launch queued behind this one on the stream (the
  // engine's lookahead, bmsched::Engine) stops at once above the hit; a slot is put back to (UINT64_MAX,
  // 0) when it gets a new object (bm_slots_init_kernel) or the batch is reset.
}

// Objects written into slots of a shard's table, stream-ordered behind the launches in flight
// (bmpow_host.hip init_slots): the record, and the "no hit" state.  recs / slots: pinned host memory.
__global__ void bm_slots_init_kernel(bm_obj* __restrict__ objs, unsigned long long* __restrict__ best,
                                     uint32_t* __restrict__ found, const bm_obj* __restrict__ recs,
                                     const uint32_t* __restrict__ slots, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = slots[i];
  objs[k] = recs[i];
  best[k] = ~0ULL;
  found[k] = 0;
}

// Trial values for an arbitrary list of nonces of one object, either form (parity probe).
__global__ __launch_bounds__(BM_BLOCK) void bm_trials_kernel(const bm_obj* __restrict__ obj,
                                                             const uint64_t* __restrict__ nonces,
                                                             uint64_t n, uint64_t* __restrict__ out,
                                                             const uint64_t* __restrict__ vpool) {
  const uint64_t k = (uint64_t)blockIdx.x * BM_BLOCK + threadIdx.x;
  if (k >= n) return;
  out[k] = trial_obj(obj, nonces[k], vpool);
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
hipError_t bm_launch_resolve(hipStream_t st, const bm_obj* objs, const bm_item* items, uint32_t nitems,
                             unsigned long long* best, uint32_t* found, bm_result* res,
                             const uint64_t* vpool, const unsigned long long* trials) {
  const uint32_t bs = 64;
  hipLaunchKernelGGL(bm_resolve_kernel, dim3((nitems + bs) / bs), dim3(bs), 0, st, objs, items, nitems,
                     best, found, res, vpool, trials);
  return hipGetLastError();
}

hipError_t bm_launch_slots_init(hipStream_t st, bm_obj* objs, unsigned long long* best, uint32_t* found,
                                const bm_obj* recs, const uint32_t* slots, uint32_t n) {
  if (n == 0) return hipSuccess;
  const uint32_t bs = 256;
  hipLaunchKernelGGL(bm_slots_init_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, st, objs, best, found, recs, slots, n);
  return hipGetLastError();
}

hipError_t bm_launch_trials(hipStream_t st, const bm_obj* obj, const uint64_t* nonces, uint64_t n,
                            uint64_t* out, const uint64_t* vpool) {
  const uint64_t nb = (n + BM_BLOCK - 1) / BM_BLOCK;
  hipLaunchKernelGGL(bm_trials_kernel, dim3((uint32_t)nb), dim3(BM_BLOCK), 0, st, obj, nonces, n, out, vpool);
  return hipGetLastError();
}
