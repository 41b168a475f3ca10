// bmpow_addr.hip -- RIPE-prefix address search on gfx950.
//
// Reference: src/class_addressGenerator.py:238-271 (deterministic addresses: try k = 0, 1, ...
// with privSigning = SHA512(passphrase || varint(2k))[:32], privEncryption =
// SHA512(passphrase || varint(2k+1))[:32], ripe = RIPEMD160(SHA512(pubSigning || pubEncryption))
// until ripe starts with numberOfNullBytesDemandedOnFrontOfRipeHash zero bytes) and :130-148
// (random addresses: fixed signing key, fresh encryption keys).
//
// One lane per try: two SHA-512 key derivations (from a per-passphrase midstate; the tail
// block is patched per lane with its varint), two fixed-base scalar multiplications
// (secp256k1_dev.h), SHA-512 over the two 65-byte keys, RIPEMD-160, prefix test,
// atomicMin(best, k).  Exact first-try semantics as the search kernel: a lane whose k is
// above a hit already recorded exits early; the host reports a hit only after the launch that
// covers every k below it has completed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bmpow_kernels.h"
#include "ripemd160_dev.h"
#include "secp256k1_dev.h"
#include "sha512_dev.h"

using namespace bm;
using ec::fe;
using ec::ge;
using ec::gej;

namespace {

// SHA-512 of (passphrase || varint(m)) given the midstate over the passphrase's full 128-byte
// blocks and the template block(s) holding its tail bytes (prm->tail_len of them).
BM_DEV void key_hash(uint64_t (&h)[8], const ar_params* __restrict__ prm, uint64_t m) {
  // varint(m) || 0x80 as a big-endian byte string in (hi, lo), top aligned
  uint64_t shi, slo = 0;
  uint32_t vlen;
  if (m < 253) {
    shi = (m << 56) | (0x80ULL << 48);
    vlen = 1;
  } else if (m < 65536) {
    shi = (0xfdULL << 56) | (m << 40) | (0x80ULL << 32);
    vlen = 3;
  } else if (m < 4294967296ULL) {
    shi = (0xfeULL << 56) | (m << 24) | (0x80ULL << 16);
    vlen = 5;
  } else {
    shi = (0xffULL << 56) | (m >> 8);
    slo = (m << 56) | (0x80ULL << 48);
    vlen = 9;
  }
  const uint32_t r = prm->tail_len;  // < 128
  const uint32_t q = r >> 3, sh = 8 * (r & 7);
  const uint64_t v0 = shi >> sh;
  const uint64_t v1 = sh ? ((shi << (64 - sh)) | (slo >> sh)) : slo;
  const uint64_t v2 = sh ? (slo << (64 - sh)) : 0;
  const uint32_t nblk = (r + vlen + 1 + 16 + 127) / 128;  // 1 or 2
  const uint64_t bits = 8 * (prm->total_len + vlen);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = prm->mid[i];
#pragma unroll 1
  for (uint32_t b = 0; b < nblk; ++b) {  // one compress body for both tail blocks
    uint64_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t jj = 16 * b + j;
      uint64_t x = prm->tmpl[jj];
      x |= (jj == q) ? v0 : ((jj == q + 1) ? v1 : ((jj == q + 2) ? v2 : 0));
      if (j == 15 && b + 1 == nblk) x |= bits;
      w[j] = x;
    }
    compress(h, w);
  }
}

// SHA-512 over 0x04||Xs||Ys||0x04||Xe||Ye (130 bytes, two blocks), then RIPEMD-160.
BM_DEV void ripe_of(uint32_t (&rh)[5], const uint64_t (&xs)[4], const uint64_t (&ys)[4], const uint64_t (&xe)[4],
                    const uint64_t (&ye)[4]) {
  uint64_t w[16];
  w[0] = (0x04ULL << 56) | (xs[0] >> 8);
  w[1] = (xs[0] << 56) | (xs[1] >> 8);
  w[2] = (xs[1] << 56) | (xs[2] >> 8);
  w[3] = (xs[2] << 56) | (xs[3] >> 8);
  w[4] = (xs[3] << 56) | (ys[0] >> 8);
  w[5] = (ys[0] << 56) | (ys[1] >> 8);
  w[6] = (ys[1] << 56) | (ys[2] >> 8);
  w[7] = (ys[2] << 56) | (ys[3] >> 8);
  w[8] = (ys[3] << 56) | (0x04ULL << 48) | (xe[0] >> 16);
  w[9] = (xe[0] << 48) | (xe[1] >> 16);
  w[10] = (xe[1] << 48) | (xe[2] >> 16);
  w[11] = (xe[2] << 48) | (xe[3] >> 16);
  w[12] = (xe[3] << 48) | (ye[0] >> 16);
  w[13] = (ye[0] << 48) | (ye[1] >> 16);
  w[14] = (ye[1] << 48) | (ye[2] >> 16);
  w[15] = (ye[2] << 48) | (ye[3] >> 16);
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = IV(i);
  const uint64_t tail0 = (ye[3] << 48) | (0x80ULL << 40);
#pragma unroll 1
  for (int b = 0; b < 2; ++b) {  // one compress body for both blocks
    compress(h, w);
    w[0] = tail0;
#pragma unroll
    for (int i = 1; i < 15; ++i) w[i] = 0;
    w[15] = 130 * 8;
  }
  rmd::of_sha512_digest(rh, h);
}

BM_DEV bool prefix_ok(const uint32_t (&rh)[5], uint32_t null_bytes) {
  // ripe bytes are h0..h4 little-endian: byte i = (h[i/4] >> 8*(i%4)) & 0xff
#pragma unroll
  for (int i = 0; i < 20; ++i)
    if ((uint32_t)i < null_bytes && ((rh[i >> 2] >> (8 * (i & 3))) & 0xff) != 0) return false;
  return true;
}

// The keys of one try.  mode 0 (deterministic): signing from m = 2k, encryption from 2k+1.
// mode 1 (random): fixed signing key prm->pub_s; encryption key from m = k of a random seed.
// Both public keys leave the comb in Jacobian coordinates and share one inversion (mode 1 feeds
// the given signing key in with Z = 1, so both modes run the same code).
template <int W>
BM_DEV bool try_keys(const ar_params* __restrict__ prm, const ge* __restrict__ table, uint64_t k,
                     uint64_t (&hs)[8], uint64_t (&he)[8], ge& ps, ge& pe) {
  const uint32_t first = prm->mode == 0 ? 0 : 1;  // mode 1: the signing key is given
  gej js, je;
  if (first) {
#pragma unroll
    for (int i = 0; i < 8; ++i) hs[i] = 0;
    js.x = prm->pub_s.x;
    js.y = prm->pub_s.y;
    ec::fe_set(js.z, 1);
    js.inf = false;
  }
  bool ok = true;
#pragma unroll 1
  for (uint32_t which = first; which < 2; ++which) {  // one hash + one comb body for both keys
    const uint64_t m = prm->mode == 0 ? 2 * k + which : k;
    uint64_t h[8];
    key_hash(h, prm, m);
    const uint64_t kw[4] = {h[0], h[1], h[2], h[3]};
    gej r;
    ec::scalar_mult_base_jac<W>(r, table, kw);
    ok = ok && !r.inf;
    if (which == 0) {
      js = r;
#pragma unroll
      for (int i = 0; i < 8; ++i) hs[i] = h[i];
    } else {
      je = r;
#pragma unroll
      for (int i = 0; i < 8; ++i) he[i] = h[i];
    }
  }
  if (!ok) return false;
  ec::gej_pair_to_ge(ps, pe, js, je);
  return true;
}

BM_DEV void ripe_of_points(uint32_t (&rh)[5], const ge& ps, const ge& pe) {
  uint64_t xs[4], ys[4], xe[4], ye[4];
  ec::fe_to_be64(xs, ps.x);
  ec::fe_to_be64(ys, ps.y);
  ec::fe_to_be64(xe, pe.x);
  ec::fe_to_be64(ye, pe.y);
  ripe_of(rh, xs, ys, xe, ye);
}


#ifndef AR_SINGLE
// ---- four keys per lane behind ONE inversion (the search path) ----
// Mode 0 (deterministic): the lane runs tries k0 and k0 + 1 -- keys 2k0 .. 2k0 + 3.  Mode 1
// (random): the signing key is the given affine point, so the lane runs FOUR tries k0 .. k0 + 3,
// one encryption key each.  Either way four combs end in Jacobian coordinates and Montgomery's
// trick converts them with one inversion: ZA = Z0 Z1, ZB = Z2 Z3, inv = (ZA ZB)^-1, iA = inv ZB,
// iB = inv ZA, Z0^-1 = iA Z1, Z1^-1 = iA Z0, Z2^-1 = iB Z3, Z3^-1 = iB Z2.  X, Y of keys 0..2 wait
// in LDS (lane-major, so the accesses are bank-conflict free); key 3 stays in registers.
constexpr int kPairLanes = 64;

BM_DEV void fe_sel(fe& r, bool c, const fe& a, const fe& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) r.d[j] = c ? a.d[j] : b.d[j];
}

BM_DEV void stash_put(uint32_t* st, int slot, uint32_t lane, const fe& x, const fe& y) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    st[(slot * 16 + j) * kPairLanes + lane] = x.d[j];
    st[(slot * 16 + 8 + j) * kPairLanes + lane] = y.d[j];
  }
}

BM_DEV void stash_get(const uint32_t* st, int slot, uint32_t lane, fe& x, fe& y) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x.d[j] = st[(slot * 16 + j) * kPairLanes + lane];
    y.d[j] = st[(slot * 16 + 8 + j) * kPairLanes + lane];
  }
}

// Jacobian (X, Y) with known Z^-1 -> affine (canonical)
BM_DEV void to_affine(ge& r, const fe& x, const fe& y, const fe& zi) {
  fe t;
  ec::fe_sqr(t, zi);
  ec::fe_mul(r.x, x, t);
  ec::fe_mul(t, t, zi);
  ec::fe_mul(r.y, y, t);
  ec::fe_normalize(r.x, r.x);
  ec::fe_normalize(r.y, r.y);
}

// Tries per lane of the search kernel for a mode.
__host__ __device__ inline uint32_t ar_tries_per_lane(uint32_t mode) { return mode == 0 ? 2u : 4u; }

// The first of the lane's ntries tries (k0, k0 + 1, ...) whose ripe has the prefix; 4 if none.
template <int W>
BM_DEV uint32_t try_quad(const ar_params* __restrict__ prm, const ge* __restrict__ table, uint64_t k0, uint32_t ntries,
                         uint32_t* st, uint32_t lane, bool fixed_sign) {
  fe z0, z1, z2;
  uint32_t bad = 0;  // bit t: a key of try t is 0 mod n
  gej r;             // after the loop: key 3 (no copy of it is kept live across the loop)
#pragma unroll 1
  for (int q = 0; q < 4; ++q) {  // one hash + one comb body for the four keys
    const uint64_t m = fixed_sign ? k0 + q : 2 * k0 + q;
    uint64_t h[8];
    key_hash(h, prm, m);
    const uint64_t kw[4] = {h[0], h[1], h[2], h[3]};
    ec::scalar_mult_base_jac<W>(r, table, kw);
    if (r.inf) {  // k = 0 mod n: keep the shared product invertible, drop the try
      ec::fe_set(r.z, 1);
      bad |= 1u << (fixed_sign ? q : q >> 1);
    }
    if (q < 3) stash_put(st, q, lane, r.x, r.y);
    fe_sel(z0, q == 0, r.z, z0);
    fe_sel(z1, q == 1, r.z, z1);
    fe_sel(z2, q == 2, r.z, z2);
  }
  const fe& z3 = r.z;
  fe za, zb, inv, ia, ib;
  ec::fe_mul(za, z0, z1);
  ec::fe_mul(zb, z2, z3);
  ec::fe_mul(inv, za, zb);
  ec::fe_inv(inv, inv);
  ec::fe_mul(ia, inv, zb);
  ec::fe_mul(ib, inv, za);
  uint32_t hit = 4;
  ge saved;  // mode 0: the encryption key (odd key) of the try being assembled; never read in mode 1
  ec::fe_set(saved.x, 0);  // (only through a select), but defined there too
  ec::fe_set(saved.y, 0);
#pragma unroll 1
  for (int q = 3; q >= 0; --q) {  // one affine + hash body for every key (key 3 first: it is live)
    fe it, zp, zi, x, y;
    fe_sel(it, q >= 2, ib, ia);
    fe_sel(zp, q == 0, z1, z0);  // the partner's Z: 0 <-> 1, 2 <-> 3
    fe_sel(zp, q == 2, z3, zp);
    fe_sel(zp, q == 3, z2, zp);
    ec::fe_mul(zi, it, zp);
    if (q == 3) {
      x = r.x;
      y = r.y;
    } else {
      stash_get(st, q, lane, x, y);
    }
    ge a;
    to_affine(a, x, y, zi);
    if (!fixed_sign && (q & 1)) {
      saved = a;
      continue;
    }
    const uint32_t t = fixed_sign ? (uint32_t)q : (uint32_t)q >> 1;
    ge ps, pe;  // selects, so the hashing is one inlined copy for both modes
    fe_sel(ps.x, fixed_sign, prm->pub_s.x, a.x);
    fe_sel(ps.y, fixed_sign, prm->pub_s.y, a.y);
    fe_sel(pe.x, fixed_sign, a.x, saved.x);
    fe_sel(pe.y, fixed_sign, a.y, saved.y);
    uint32_t rh[5];
    ripe_of_points(rh, ps, pe);
    if (t < ntries && !((bad >> t) & 1) && prefix_ok(rh, prm->null_bytes)) hit = t;  // q descends
  }
  return hit;
}
#endif  // AR_SINGLE

}  // namespace

// The comb table in two launches.  ar_base_kernel: bases[i] = 2^(W i) * G (affine), one thread per
// window.  ar_table_kernel: table[i << W | v] = v * bases[i] by double-and-add over v's W bits,
// one thread per entry (entries v = 0 are never read as points: the comb skips zero windows).
template <int W>
__global__ __launch_bounds__(64) void ar_base_kernel(ge* __restrict__ bases) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= (uint32_t)ec::comb<W>::kWindows) return;
  gej b;
  b.inf = false;
  // G
  const uint32_t gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                          0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const uint32_t gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                          0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
  for (int j = 0; j < 8; ++j) {
    b.x.d[j] = gx[j];
    b.y.d[j] = gy[j];
  }
  ec::fe_set(b.z, 1);
  for (uint32_t d = 0; d < (uint32_t)W * i; ++d) ec::gej_double(b, b);  // 2^(W i) * G
  ec::gej_to_ge(bases[i], b);
}

template <int W>
__global__ __launch_bounds__(64) void ar_table_kernel(const ge* __restrict__ bases, ge* __restrict__ table) {
  const size_t t = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (t >= ec::comb<W>::kEntries) return;
  const uint32_t i = (uint32_t)(t >> W), v = (uint32_t)t & ec::comb<W>::kMask;
  if (v == 0) return;
  const ge ba = bases[i];
  gej acc;
  acc.inf = true;
  for (int bit = 31 - __builtin_clz(v); bit >= 0; --bit) {  // v * B, MSB first
    ec::gej_double(acc, acc);
    if ((v >> bit) & 1) ec::gej_add_ge(acc, acc, ba);
  }
  ec::gej_to_ge(table[t], acc);
}

// Search: lanes try k in [start, start + count), two (mode 0) or four (mode 1) consecutive tries per
// lane (try_quad; one per lane when built with -DAR_SINGLE, the A/B baseline).  best: running minimum k with a hit.
// kResolve: the launch instead reports everything about the single try k = start (keys, public
// keys, ripe) -- the resolve step, sharing this kernel's code; a separate instantiation so the
// search never keeps the private-key digests live.
// 3 waves/SIMD (168 VGPRs, a few dwords spilled) beat 2 waves at 173 VGPRs: 206 vs 193 M tries/s
// end to end at 3 null bytes (r01p).
#ifndef AR_WAVES
#define AR_WAVES 3
#endif
#define AR_OCC __attribute__((amdgpu_waves_per_eu(AR_WAVES)))
template <bool kResolve, int W>
__global__ __launch_bounds__(64) AR_OCC void ar_search_kernel(const ar_params* __restrict__ prm, const ge* __restrict__ table,
                                                       uint64_t start, uint32_t count,
                                                       unsigned long long* __restrict__ best,
                                                       ar_result* __restrict__ out, uint32_t mode) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
#ifndef AR_SINGLE
  if (!kResolve) {  // lane g: tries start + T g .. start + T g + T - 1 below start + count (T = 2 or 4)
    __shared__ uint32_t stash[3 * 16 * kPairLanes];
    const uint32_t T = ar_tries_per_lane(mode);  // the host sized the grid with this same argument
    const uint64_t first = (uint64_t)T * g;
    if (first >= count) return;
    const uint64_t k0 = start + first;
    if (__hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k0) return;
    const uint32_t ntries = (uint32_t)min((uint64_t)T, count - first);
    const uint32_t hit = try_quad<W>(prm, table, k0, ntries, stash, threadIdx.x, mode != 0);
    if (hit < ntries) atomicMin(best, (unsigned long long)(k0 + hit));
    return;
  }
#endif
  if (g >= count) return;
  const uint64_t k = start + g;
  if (!kResolve && __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) return;
  uint64_t hs[8], he[8];
  ge ps, pe;
  const bool ok = try_keys<W>(prm, table, k, hs, he, ps, pe);
  uint32_t rh[5] = {0, 0, 0, 0, 0};
  if (ok) ripe_of_points(rh, ps, pe);
  if (kResolve) {
    out->k = k;
    out->ok = ok ? 1u : 0u;
    for (int i = 0; i < 4; ++i) {
      out->priv_s[i] = hs[i];
      out->priv_e[i] = he[i];
    }
    out->pub_s = ps;
    out->pub_e = pe;
    for (int i = 0; i < 5; ++i) out->ripe[i] = rh[i];
    return;
  }
  if (ok && prefix_ok(rh, prm->null_bytes)) atomicMin(best, (unsigned long long)k);
}

// pointMult parity probe: pub[i] = privs[i] * G (privs as 4 big-endian words each).
__global__ __launch_bounds__(64) void ar_pubkey_kernel(const uint64_t* __restrict__ privs, uint32_t n,
                                                       const ge* __restrict__ table, ge* __restrict__ pubs,
                                                       uint32_t* __restrict__ ok) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n) return;
  const uint64_t kw[4] = {privs[4 * g], privs[4 * g + 1], privs[4 * g + 2], privs[4 * g + 3]};
  ge r;
  ok[g] = ec::scalar_mult_base<ec::kCombSmall>(r, table, kw) ? 1u : 0u;
  pubs[g] = r;
}

// Field-arithmetic probe (tests only): out[i] = op(a[i], b[i]) on arbitrary 256-bit inputs, so the
// weak-reduction bounds are checked at the edges (values >= p, near 2^256) that random keys never
// reach.  op: 0 add, 1 sub, 2 mul, 3 sqr, 4 normalize, 5 inv, 6 is_zero (out limb 0 = 0/1).
__global__ __launch_bounds__(64) void ar_fe_probe_kernel(int op, const fe* __restrict__ a, const fe* __restrict__ b,
                                                         fe* __restrict__ out, uint32_t n) {
  const uint32_t g = blockIdx.x * 64 + threadIdx.x;
  if (g >= n) return;
  const fe x = a[g], y = b[g];
  fe r;
  ec::fe_set(r, 0);
  switch (op) {
    case 0: ec::fe_add(r, x, y); break;
    case 1: ec::fe_sub(r, x, y); break;
    case 2: ec::fe_mul(r, x, y); break;
    case 3: ec::fe_sqr(r, x); break;
    case 4: ec::fe_normalize(r, x); break;
    case 5: ec::fe_inv(r, x); break;
    case 6: ec::fe_set(r, ec::fe_is_zero(x) ? 1u : 0u); break;
    default: break;
  }
  out[g] = r;
}

// Midstate of the passphrase's first nfull 128-byte blocks (one thread).
__global__ void ar_midstate_kernel(const uint8_t* __restrict__ pass, uint64_t nfull, uint64_t* __restrict__ mid) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  uint64_t h[8];
  for (int i = 0; i < 8; ++i) h[i] = IV(i);
  for (uint64_t b = 0; b < nfull; ++b) {
    uint64_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint64_t x = 0;
      for (int q = 0; q < 8; ++q) x = (x << 8) | pass[b * 128 + 8 * j + q];
      w[j] = x;
    }
    compress(h, w);
  }
  for (int i = 0; i < 8; ++i) mid[i] = h[i];
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (C++ linkage, used by bmpow_host.hip).
// ---------------------------------------------------------------------------------------
// table: ec::comb<W>::kEntries entries followed by ec::comb<W>::kWindows scratch entries (the bases)
template <int W>
hipError_t launch_table(hipStream_t st, ge* table) {
  using C = ec::comb<W>;
  ge* bases = table + C::kEntries;
  hipLaunchKernelGGL(ar_base_kernel<W>, dim3(1), dim3(64), 0, st, bases);
  hipLaunchKernelGGL(ar_table_kernel<W>, dim3((uint32_t)((C::kEntries + 63) / 64)), dim3(64), 0, st,
                     (const ge*)bases, table);
  return hipGetLastError();
}

size_t ar_table_entries(int wbits) {
  return wbits == ec::kCombLarge ? ec::comb<ec::kCombLarge>::kEntries + ec::comb<ec::kCombLarge>::kWindows
                                 : ec::comb<ec::kCombSmall>::kEntries + ec::comb<ec::kCombSmall>::kWindows;
}

hipError_t ar_launch_table(hipStream_t st, ge* table, int wbits) {
  return wbits == ec::kCombLarge ? launch_table<ec::kCombLarge>(st, table) : launch_table<ec::kCombSmall>(st, table);
}

hipError_t ar_launch_search(hipStream_t st, const ar_params* prm, uint32_t mode, const ge* table, int wbits,
                            uint64_t start, uint32_t count, unsigned long long* best) {
  if (count == 0) return hipSuccess;
#ifndef AR_SINGLE
  const uint32_t tpl = ar_tries_per_lane(mode);  // the kernel takes the same mode argument
#else
  const uint32_t tpl = 1;
  (void)mode;
#endif
  const uint32_t lanes = (uint32_t)(((uint64_t)count + tpl - 1) / tpl);
  if (wbits == ec::kCombLarge)
    hipLaunchKernelGGL((ar_search_kernel<false, ec::kCombLarge>), dim3((lanes + 63) / 64), dim3(64), 0, st, prm, table,
                       start, count, best, (ar_result*)nullptr, mode);
  else
    hipLaunchKernelGGL((ar_search_kernel<false, ec::kCombSmall>), dim3((lanes + 63) / 64), dim3(64), 0, st, prm, table,
                       start, count, best, (ar_result*)nullptr, mode);
  return hipGetLastError();
}

// the resolve step runs with the search's comb (so the tests see that comb's public keys); the
// pointMult probe (ar_launch_pubkeys) always uses the small one
hipError_t ar_launch_resolve(hipStream_t st, const ar_params* prm, const ge* table, int wbits, uint64_t k,
                             ar_result* out) {
  if (wbits == ec::kCombLarge)
    hipLaunchKernelGGL((ar_search_kernel<true, ec::kCombLarge>), dim3(1), dim3(64), 0, st, prm, table, k, 1u,
                       (unsigned long long*)nullptr, out, 0u /* the resolve path (try_keys) reads prm->mode */);
  else
    hipLaunchKernelGGL((ar_search_kernel<true, ec::kCombSmall>), dim3(1), dim3(64), 0, st, prm, table, k, 1u,
                       (unsigned long long*)nullptr, out, 0u /* the resolve path (try_keys) reads prm->mode */);
  return hipGetLastError();
}

hipError_t ar_launch_pubkeys(hipStream_t st, const uint64_t* privs, uint32_t n, const ge* table, ge* pubs,
                             uint32_t* ok) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ar_pubkey_kernel, dim3((n + 63) / 64), dim3(64), 0, st, privs, n, table, pubs, ok);
  return hipGetLastError();
}

hipError_t ar_launch_fe_probe(hipStream_t st, int op, const ec::fe* a, const ec::fe* b, ec::fe* out, uint32_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ar_fe_probe_kernel, dim3((n + 63) / 64), dim3(64), 0, st, op, a, b, out, n);
  return hipGetLastError();
}

hipError_t ar_launch_midstate(hipStream_t st, const uint8_t* pass, uint64_t nfull, uint64_t* mid) {
  hipLaunchKernelGGL(ar_midstate_kernel, dim3(1), dim3(64), 0, st, pass, nfull, mid);
  return hipGetLastError();
}
