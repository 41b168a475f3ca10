// modinv_dev.h -- inversion mod p = 2^256 - 2^32 - 977 by Bernstein-Yang divsteps ("safegcd",
// Bernstein & Yang, "Fast constant-time gcd computation and modular inversion", TCHES 2019).
//
// The address search turns two Jacobian keys to affine with one inversion per try
// (secp256k1_dev.h gej_pair_to_ge).  Fermat's a^(p-2) costs 255 squarings + 15 products there
// (~52 k VALU instructions, 37 % of a try); this costs 600 divsteps on 32-bit words plus 20
// matrix applications to 9-limb numbers.  Constant time: every lane runs the same 20 x 30 steps
// (590 divsteps suffice for 256-bit inputs), so a wave never diverges.
//
// Numbers are 9 signed 30-bit limbs (value = sum v[i] 2^(30 i); after an update limbs 0..7 lie in
// [0, 2^30) and v[8] carries the sign).  p itself is {-977, -4, 0, 0, 0, 0, 0, 0, 65536}, so the
// multiples of p added to make a matrix product divisible by 2^30 touch three limbs only.
// Invariants: f = d x (mod p), g = e x (mod p); at the end g = 0, f = +-1, so x^-1 = +-d.
//
// The structure follows libsecp256k1's 32-bit safegcd implementation (src/modinv32_impl.h, MIT
// licence; the reference uses secp256k1 through OpenSSL, not libsecp256k1): zeta-form 30-divstep
// batches on the low words, and the update of d, e with the multiple of p chosen from
// p^-1 mod 2^30 so each product is exactly divisible by 2^30.  Rewritten here for a wave of 64
// lanes (branch-free selects, the 9-limb representation and p's three nonzero limbs).
//
// Plain C++ (int32/int64 only): the same source compiles for gfx950 and for the host, where
// tests/test_modinv.py checks it against Python's pow(x, -1, p).
#pragma once
#include <stdint.h>

#ifndef BM_HD
#if defined(__HIPCC__)
#define BM_HD __device__ __forceinline__
#else
#define BM_HD static inline
#endif
#endif

namespace mi {

constexpr int32_t M30 = 0x3FFFFFFF;
constexpr int32_t P0 = -977, P1 = -4, P8 = 65536;  // p in signed 30-bit limbs (others 0)
constexpr uint32_t PINV30 = 0x2DDACACFu;           // p^-1 mod 2^30

// 30 divsteps on the low words of f and g.  Returns the new zeta (= -(delta + 1/2)) and the
// transition matrix t = {u, v, q, r}, scaled by 2^30: [f', g'] 2^30 = t [f, g].
//   zeta < 0 and g odd:  (f, g) <- (g, (g - f) / 2), zeta <- -zeta - 2
//   otherwise:           (f, g) <- (f, (g + (g & 1) f) / 2), zeta <- zeta - 1
// Only bit 0 of g is ever inspected, and after i steps it depends on bits 0..i of the inputs, so
// 32-bit words carry 30 steps exactly.
BM_HD int32_t divsteps30(int32_t zeta, uint32_t f, uint32_t g, int32_t (&t)[4]) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);  // all ones: zeta < 0
    const uint32_t c2 = 0u - (g & 1u);           // all ones: g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;  // g +- f
    q += y & c2;
    r += z & c2;
    const uint32_t c3 = c1 & c2;  // swap
    zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
    f += g & c3;  // f <- old g
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return zeta;
}

// [f, g] <- t [f, g] / 2^30 (exact: the low 30 bits of both products are zero by construction)
BM_HD void update_fg(int32_t (&f)[9], int32_t (&g)[9], const int32_t (&t)[4]) {
  const int64_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = u * f[0] + v * g[0];
  int64_t cg = q * f[0] + r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cf += u * f[i] + v * g[i];
    cg += q * f[i] + r * g[i];
    f[i - 1] = (int32_t)cf & M30;
    g[i - 1] = (int32_t)cg & M30;
    cf >>= 30;
    cg >>= 30;
  }
  f[8] = (int32_t)cf;
  g[8] = (int32_t)cg;
}

// [d, e] <- (t [d, e] + p [md, me]) / 2^30 with md, me chosen so the division is exact
// (md = -p^-1 (u d + v e) mod 2^30); starting md/me from the sign terms keeps d, e in (-2p, p).
BM_HD void update_de(int32_t (&d)[9], int32_t (&e)[9], const int32_t (&t)[4]) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d[8] >> 31, se = e[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d[0] + (int64_t)v * e[0];
  int64_t ce = (int64_t)q * d[0] + (int64_t)r * e[0];
  md -= (int32_t)((PINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((PINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)P0 * md;
  ce += (int64_t)P0 * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    cd += (int64_t)u * d[i] + (int64_t)v * e[i];
    ce += (int64_t)q * d[i] + (int64_t)r * e[i];
    if (i == 1) {
      cd += (int64_t)P1 * md;
      ce += (int64_t)P1 * me;
    } else if (i == 8) {
      cd += (int64_t)P8 * md;
      ce += (int64_t)P8 * me;
    }
    d[i - 1] = (int32_t)cd & M30;
    e[i - 1] = (int32_t)ce & M30;
    cd >>= 30;
    ce >>= 30;
  }
  d[8] = (int32_t)cd;
  e[8] = (int32_t)ce;
}

// d <- d + (p & m), limbs renormalised (m = 0 or all ones)
BM_HD void add_p_masked(int32_t (&d)[9], int32_t m) {
  int64_t c = (int64_t)d[0] + (P0 & m);
  d[0] = (int32_t)c & M30;
  c >>= 30;
  c += (int64_t)d[1] + (P1 & m);
  d[1] = (int32_t)c & M30;
  c >>= 30;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    c += d[i];
    d[i] = (int32_t)c & M30;
    c >>= 30;
  }
  d[8] = (int32_t)(c + d[8] + (P8 & m));
}

// d <- -d when s is all ones, limbs renormalised
BM_HD void neg_masked(int32_t (&d)[9], int32_t s) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (int64_t)((d[i] ^ s) - s);
    d[i] = (int32_t)c & M30;
    c >>= 30;
  }
  d[8] = (int32_t)(c + ((d[8] ^ s) - s));
}

// r = a^-1 mod p for 0 < a < p (8 little-endian 32-bit limbs in and out; a = 0 gives 0)
BM_HD void inv_mod_p(uint32_t (&r)[8], const uint32_t (&a)[8]) {
  int32_t f[9] = {P0, P1, 0, 0, 0, 0, 0, 0, P8};
  int32_t g[9], d[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, e[9] = {1, 0, 0, 0, 0, 0, 0, 0, 0};
  // 8 x 32 -> 9 x 30 bits: limb i = bits [30i, 30i + 30)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int b = 30 * i, w = b >> 5, s = b & 31;
    const uint32_t lo = a[w] >> s;
    const uint32_t hi = (s && w + 1 < 8) ? (a[w + 1] << (32 - s)) : 0u;
    g[i] = (int32_t)((lo | hi) & (uint32_t)M30);
  }
  g[8] = (int32_t)(a[7] >> 16);
  int32_t zeta = -1;
#pragma unroll 1
  for (int it = 0; it < 20; ++it) {
    int32_t t[4];
    zeta = divsteps30(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    update_de(d, e, t);
    update_fg(f, g, t);
  }
  // d in (-2p, p); x^-1 = sign(f) d mod p
  add_p_masked(d, d[8] >> 31);
  neg_masked(d, f[8] >> 31);
  add_p_masked(d, d[8] >> 31);
  // 9 x 30 -> 8 x 32 bits
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int b = 32 * j, i = b / 30, s = b % 30;
    uint32_t w = (uint32_t)d[i] >> s;
    if (i + 1 < 9) w |= (uint32_t)d[i + 1] << (30 - s);
    if (s > 28 && i + 2 < 9) w |= (uint32_t)d[i + 2] << (60 - s);
    r[j] = w;
  }
}

}  // namespace mi
