// secp256k1_dev.h -- gfx950 field and group arithmetic for the RIPE-prefix address search.
//
// The reference turns a private key into a public key with OpenSSL EC_POINT_mul on secp256k1
// (src/highlevelcrypto.py:111-140, pointMult).  Here one lane computes k*G for its own k:
//   * field elements mod p = 2^256 - 2^32 - 977 as 8 x 32-bit little-endian limbs, WEAKLY reduced:
//     every fe is some value < 2^256 congruent to the element (so 0 and p both stand for zero);
//     products by v_mad_u64_u32 with its carry-out (product scanning, 2 instructions per 32x32
//     product), reduction by 2^256 = 2^32 + 977.  Only affine points (ge: table entries, keys
//     that get serialized) are canonical (< p): fe_normalize runs once per affine coordinate,
//     instead of a conditional subtraction at the end of every operation;
//   * k*G by a fixed-base comb: windows of W = 16 or 24 bits, table[i][v] = v * 2^(W i) * G in
//     affine coordinates (64 MB or 10.7 GB, built once per device by ar_table_kernel), so one
//     scalar multiplication is 16 or 11 mixed Jacobian+affine additions and one inversion (shared
//     by the two keys of an address try, gej_pair_to_ge);
//   * inversion by Bernstein-Yang divsteps (modinv_dev.h: 600 divsteps on 32-bit words + 20
//     updates of 9 x 30-bit limbs); Fermat (a^(p-2), 255 squarings + 15 products) is kept
//     behind -DAR_INV_FERMAT for A/B runs.
#pragma once
#include <stdint.h>

#include "modinv_dev.h"

#ifndef BM_DEV
#define BM_DEV __device__ __forceinline__
#endif

namespace ec {

struct fe {
  uint32_t d[8];
};

struct ge {  // affine point (table entry); 64 B
  fe x, y;
};

struct gej {  // Jacobian point; inf marks the point at infinity
  fe x, y, z;
  bool inf;
};

// 2^256 - p = 2^32 + 977
constexpr uint32_t C0 = 977;

BM_DEV void fe_set(fe& r, uint32_t v) {
  r.d[0] = v;
#pragma unroll
  for (int i = 1; i < 8; ++i) r.d[i] = 0;
}

// a = 0 mod p for a weakly reduced a, i.e. a == 0 or a == p
BM_DEV bool fe_is_zero(const fe& a) {
  uint32_t o = 0, n = (a.d[0] ^ 0xFFFFFC2Fu) | (a.d[1] ^ 0xFFFFFFFEu);
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.d[i];
#pragma unroll
  for (int i = 2; i < 8; ++i) n |= ~a.d[i];
  return o == 0 || n == 0;
}

// ---- carry primitives ----
// Limb chains use __builtin_addc/__builtin_subc (v_add_co/v_addc_co with the carry in VCC); the
// products use v_mad_u64_u32 directly for its carry-out (VOP3b sdst), which no builtin exposes:
// a 64-bit column accumulator plus a 32-bit top word absorb every product at 2 instructions
// (mad + addc), against ~4 (mad + 64-bit add + 2 moves to build zero-extended pairs) for the
// uint64_t operand-scanning form.

// (acc, top) += a * b
BM_DEV void mac(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cc, unused;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
  asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(top), "=s"(unused) : "s"(cc));
}

// acc += a * b; top = the carry out (first product of a column)
BM_DEV void mac_first(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cc, unused;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
  asm("v_addc_co_u32_e64 %0, %1, 0, 0, %2" : "=v"(top), "=s"(unused) : "s"(cc));
}

// acc += a (a 32-bit add into the 64-bit accumulator, as a * 1)
BM_DEV void add_nc(uint64_t& acc, uint32_t a) {
  uint64_t unused;
  asm("v_mad_u64_u32 %0, %1, %2, 1, %0" : "+v"(acc), "=s"(unused) : "v"(a));
}

// acc += a * 977 (977 = 2^256 mod p - 2^32, from an SGPR)
BM_DEV void mad977_nc(uint64_t& acc, uint32_t a) {
  uint64_t unused;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(unused) : "v"(a), "s"(C0));
}

// a * b as 64 bits
BM_DEV uint64_t mul_wide(uint32_t a, uint32_t b) {
  uint64_t r, unused;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(unused) : "v"(a), "v"(b));
  return r;
}

// r = t mod p for t < 2^256 + carry * 2^256 (carry in {0,1}, t < p when it is set): returns
// t - p when t >= p.  t >= p  <=>  t + (2^256 - p) carries out of 256 bits.
BM_DEV void fe_cond_sub_p(fe& r, const uint32_t (&t)[8], uint32_t carry) {
  uint32_t u[8], c;
  u[0] = __builtin_addc(t[0], C0, 0u, &c);
  u[1] = __builtin_addc(t[1], 1u, c, &c);
#pragma unroll
  for (int i = 2; i < 8; ++i) u[i] = __builtin_addc(t[i], 0u, c, &c);
  const bool ge_p = (c | carry) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.d[i] = ge_p ? u[i] : t[i];
}

// r = t - p when t >= p (t < 2^256): the canonical form of a weakly reduced element
BM_DEV void fe_normalize(fe& r, const fe& a) { fe_cond_sub_p(r, a.d, 0u); }

// r = a + b for a, b < 2^256: the carry out of 256 bits folds back as 2^256 = 2^32 + 977.  A
// second carry needs a + b >= 2^257 - (2^32 + 977); the sum left is then < 2^32 + 977, so the
// second fold ends in limb 1.
BM_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = __builtin_addc(a.d[i], b.d[i], c, &c);
  uint32_t m = 0u - c;
  t[0] = __builtin_addc(t[0], C0 & m, 0u, &c);
  t[1] = __builtin_addc(t[1], 1u & m, c, &c);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = __builtin_addc(t[i], 0u, c, &c);
  m = 0u - c;
  r.d[0] = __builtin_addc(t[0], C0 & m, 0u, &c);
  r.d[1] = t[1] + (1u & m) + c;
#pragma unroll
  for (int i = 2; i < 8; ++i) r.d[i] = t[i];
}

// r = a - b for a, b < 2^256: a borrow out of 256 bits adds p back as - (2^32 + 977) mod 2^256.
// A second borrow needs the difference t = a - b + 2^256 below 2^32 + 977 (b >= p + a, so b is
// unreduced); t + 2^256 - (2^32 + 977) is then >= 2^256 - 2^32 - 976, and subtracting
// 2^32 + 977 once more (= adding 2p in all) stays in limbs 0..1 without a borrow.
BM_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t t[8], bw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = __builtin_subc(a.d[i], b.d[i], bw, &bw);
  uint32_t m = 0u - bw;
  t[0] = __builtin_subc(t[0], C0 & m, 0u, &bw);
  t[1] = __builtin_subc(t[1], 1u & m, bw, &bw);
#pragma unroll
  for (int i = 2; i < 8; ++i) t[i] = __builtin_subc(t[i], 0u, bw, &bw);
  m = 0u - bw;
  r.d[0] = __builtin_subc(t[0], C0 & m, 0u, &bw);
  r.d[1] = t[1] - (1u & m) - bw;  // limb 1 >= 2^32 - 2 here: no borrow into limb 2
#pragma unroll
  for (int i = 2; i < 8; ++i) r.d[i] = t[i];
}

// r = 2a as an addition (cheap, exact)
BM_DEV void fe_dbl(fe& r, const fe& a) { fe_add(r, a, a); }

// r = p mod p_field (weakly) for a 512-bit product p (16 limbs): t = L + H * 977 + H * 2^32
// column by column (each column < 2^43, no carry out of the accumulator), then the overflow
// c < 2^33 above 2^256 folded once more the same way and a last 0/1 fold.
BM_DEV void fe_reduce512(fe& r, const uint32_t (&p)[16]) {
  uint32_t t[8];
  uint64_t acc = p[0];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i) add_nc(acc, p[i]);
    mad977_nc(acc, p[8 + i]);
    if (i) add_nc(acc, p[7 + i]);
    t[i] = (uint32_t)acc;
    acc >>= 32;
  }
  add_nc(acc, p[15]);  // value = t + acc * 2^256, acc = ah * 2^32 + al < 2^33
  const uint32_t al = (uint32_t)acc, ah = (uint32_t)(acc >> 32);
  // + acc * (2^32 + 977): al*977 into limb 0, al + ah*977 into limb 1, ah into limb 2
  uint64_t lo = t[0];
  mad977_nc(lo, al);
  t[0] = (uint32_t)lo;
  const uint32_t x = (uint32_t)(lo >> 32) + ah * C0;  // < 2^11
  uint32_t c, c2;
  t[1] = __builtin_addc(t[1], al, 0u, &c);
  t[1] = __builtin_addc(t[1], x, 0u, &c2);
  t[2] = __builtin_addc(t[2], ah, c, &c);
  t[2] = __builtin_addc(t[2], 0u, c2, &c2);
  c |= c2;  // at most one of them is set
#pragma unroll
  for (int i = 3; i < 8; ++i) t[i] = __builtin_addc(t[i], 0u, c, &c);
  // c in {0,1}: one more fold of 2^256.  The value was < 2^256 + 2^66 (t < 2^256 plus
  // acc (2^32 + 977)), so when c is set t < 2^66: limb 2 < 4 absorbs the last carry, and the
  // result is weakly reduced (< 2^256) either way -- no conditional subtraction.
  const uint32_t m = 0u - c;
  r.d[0] = __builtin_addc(t[0], C0 & m, 0u, &c);
  r.d[1] = __builtin_addc(t[1], 1u & m, c, &c);
  r.d[2] = t[2] + c;
#pragma unroll
  for (int i = 3; i < 8; ++i) r.d[i] = t[i];
}

// 512-bit product by columns (product scanning): column k sums a_i b_j over i + j = k.
BM_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t p[16];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    const int i0 = k < 8 ? 0 : k - 7, i1 = k < 8 ? k : 7;
    mac_first(acc, top, a.d[i0], b.d[k - i0]);
#pragma unroll
    for (int i = i0 + 1; i <= i1; ++i) mac(acc, top, a.d[i], b.d[k - i]);
    p[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  p[15] = (uint32_t)acc;
  fe_reduce512(r, p);
}

// r = a^2: the 28 cross products once (product scanning), doubled by a 1-bit funnel shift, plus
// the 8 squares -- the inversion is 255 of these per point.
BM_DEV void fe_sqr(fe& r, const fe& a) {
  uint32_t p[16];
  p[0] = 0;
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int k = 1; k < 14; ++k) {
    const int i0 = k < 8 ? 0 : k - 7, i1 = (k - 1) / 2;  // i < j = k - i
    mac_first(acc, top, a.d[i0], a.d[k - i0]);
#pragma unroll
    for (int i = i0 + 1; i <= i1; ++i) mac(acc, top, a.d[i], a.d[k - i]);
    p[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  p[14] = (uint32_t)acc;  // cross sum < 2^511: nothing above limb 14 but its carry bit
  p[15] = (uint32_t)(acc >> 32);
#pragma unroll
  for (int i = 15; i > 0; --i) p[i] = __builtin_amdgcn_alignbit(p[i], p[i - 1], 31);
  p[0] = 0;  // p[0] was 0 before the doubling too
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t sq = mul_wide(a.d[i], a.d[i]);
    p[2 * i] = __builtin_addc(p[2 * i], (uint32_t)sq, c, &c);
    p[2 * i + 1] = __builtin_addc(p[2 * i + 1], (uint32_t)(sq >> 32), c, &c);
  }
  fe_reduce512(r, p);
}

// a^-1 mod p (a != 0; a = 0 gives 0).
#ifndef AR_INV_FERMAT
BM_DEV void fe_inv(fe& r, const fe& a) {  // inv_mod_p wants 0 <= a < p
  fe n;
  fe_normalize(n, a);
  mi::inv_mod_p(r.d, n.d);
}
#else
// a^(p-2) = a^-1 (a != 0).  The exponent is [223 ones][0][22 ones][0000101101]; the 255-
// squaring / 15-multiplication addition chain (runs of 2^n - 1 ones: 1, 2, 3, 6, 9, 11, 22, 44,
// 88, 176, 220, 223) runs as a rolled loop of (squarings, multiplier) steps so the kernel holds
// one squaring and one multiplication body instead of 37 inlined copies.
BM_DEV void fe_inv(fe& r, const fe& a) {
  // step s: t = t^(2^N[s]) * mult[M[s]]; mult: 0 a, 1 x2, 2 x3, 3 x11, 4 x22, 5 x44, 6 x88
  constexpr uint8_t N[15] = {1, 1, 3, 3, 2, 11, 22, 44, 88, 44, 3, 23, 5, 3, 2};
  constexpr uint8_t M[15] = {0, 0, 2, 2, 1, 3, 4, 5, 6, 5, 2, 4, 0, 1, 0};
  fe t = a, x2 = a, x3 = a, x11 = a, x22 = a, x44 = a, x88 = a;
#pragma unroll 1
  for (int s = 0; s < 15; ++s) {
#pragma unroll 1
    for (int i = 0; i < N[s]; ++i) fe_sqr(t, t);
    const int m = M[s];
    fe f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      f.d[j] = m == 0 ? a.d[j]
             : m == 1 ? x2.d[j]
             : m == 2 ? x3.d[j]
             : m == 3 ? x11.d[j]
             : m == 4 ? x22.d[j]
             : m == 5 ? x44.d[j]
                      : x88.d[j];
    fe_mul(t, t, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x2.d[j] = s == 0 ? t.d[j] : x2.d[j];
      x3.d[j] = s == 1 ? t.d[j] : x3.d[j];
      x11.d[j] = s == 4 ? t.d[j] : x11.d[j];
      x22.d[j] = s == 5 ? t.d[j] : x22.d[j];
      x44.d[j] = s == 6 ? t.d[j] : x44.d[j];
      x88.d[j] = s == 7 ? t.d[j] : x88.d[j];
    }
  }
  r = t;
}
#endif

// ---- group law (y^2 = x^3 + 7, a = 0) ----

// dbl-2009-l: 2M + 5S
BM_DEV void gej_double(gej& r, const gej& p) {
  if (p.inf || fe_is_zero(p.y)) {
    r.inf = true;
    return;
  }
  fe A, B, C, D, E, F, t;
  fe_sqr(A, p.x);
  fe_sqr(B, p.y);
  fe_sqr(C, B);
  fe_add(t, p.x, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_dbl(D, t);
  fe_dbl(E, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  fe_mul(r.z, p.y, p.z);  // before r.x/r.y overwrite p (r may alias p)
  fe_dbl(r.z, r.z);
  fe_dbl(t, D);
  fe_sub(r.x, F, t);
  fe_sub(t, D, r.x);
  fe_mul(t, E, t);
  fe_dbl(C, C);
  fe_dbl(C, C);
  fe_dbl(C, C);
  fe_sub(r.y, t, C);
  r.inf = false;
}

// r = p + q with q affine (8M + 3S); handles p = inf and p = -q, and p = q by doubling when
// kDouble -- otherwise it returns false there with r unspecified (the comb's hot loop: its caller
// redoes the multiplication with the doubling path, so gej_double's registers never weigh on the
// loop that runs; keeping it inline there pushed the accumulator out to scratch).
template <bool kDouble>
BM_DEV bool gej_add_ge_t(gej& r, const gej& p, const ge& q) {
  // Every path leaves its result in these locals and r is written once at the end: stores to r
  // from several branches became one store through a phi'd address, which kept the comb's
  // accumulator in scratch memory instead of registers.
  fe rx, ry, rz;
  bool rinf = false, ok = true;
  if (p.inf) {
    rx = q.x;
    ry = q.y;
    fe_set(rz, 1);
  } else {
    fe z1z1, u2, s2, h, rr;
    fe_sqr(z1z1, p.z);
    fe_mul(u2, q.x, z1z1);
    fe_mul(s2, q.y, p.z);
    fe_mul(s2, s2, z1z1);
    fe_sub(h, u2, p.x);
    fe_sub(rr, s2, p.y);
    if (fe_is_zero(h)) {
      rx = p.x;
      ry = p.y;
      rz = p.z;
      if (!fe_is_zero(rr)) {
        rinf = true;  // p = -q
      } else if (kDouble) {
        gej d;
        gej_double(d, p);
        rx = d.x;
        ry = d.y;
        rz = d.z;
        rinf = d.inf;
      } else {
        ok = false;  // p = q: the caller takes the doubling pass
      }
    } else {
      fe hh, hhh, v, t;
      fe_sqr(hh, h);
      fe_mul(hhh, h, hh);
      fe_mul(v, p.x, hh);
      fe_mul(rz, p.z, h);
      fe_mul(t, p.y, hhh);
      fe_sqr(rx, rr);
      fe_sub(rx, rx, hhh);
      fe_sub(rx, rx, v);
      fe_sub(rx, rx, v);
      fe_sub(v, v, rx);
      fe_mul(v, rr, v);
      fe_sub(ry, v, t);
    }
  }
  r.x = rx;
  r.y = ry;
  r.z = rz;
  r.inf = rinf;
  return ok;
}

BM_DEV void gej_add_ge(gej& r, const gej& p, const ge& q) { gej_add_ge_t<true>(r, p, q); }

// Jacobian -> affine (p not at infinity)
BM_DEV void gej_to_ge(ge& r, const gej& p) {
  fe zi, zi2;
  fe_inv(zi, p.z);
  fe_sqr(zi2, zi);
  fe_mul(r.x, p.x, zi2);
  fe_mul(zi2, zi2, zi);
  fe_mul(r.y, p.y, zi2);
  fe_normalize(r.x, r.x);
  fe_normalize(r.y, r.y);
}

// Fixed-base combs: table[i << W | v] = v * 2^(W i) * G (affine), ceil(256 / W) windows, the last
// one ragged (256 - W (windows - 1) bits, only 2^that entries stored).  Two widths are built:
//   W = 16: 16 mixed additions per k*G over a 64 MB table (built in ~15 ms);
//   W = 24: 11 additions over a 10.7 GB table (HBM-resident, ~0.4 s to build once per device),
// chosen per search by the host (bmpow_host.hip addr_comb_for) so short searches never pay for the
// big table and long ones run 25 % faster.
constexpr int kCombSmall = 16;
#ifndef AR_WBITS_LARGE
#define AR_WBITS_LARGE 24
#endif
constexpr int kCombLarge = AR_WBITS_LARGE;

template <int W>
struct comb {
  static_assert(W >= 8 && W <= 26, "comb window width");
  static constexpr int kWindows = (256 + W - 1) / W;
  static constexpr int kLastBits = 256 - W * (kWindows - 1);
  static constexpr uint32_t kMask = (1u << W) - 1;
  static constexpr size_t kEntries = ((size_t)(kWindows - 1) << W) + ((size_t)1 << kLastBits);
};

// s (256 bits, s[0] least significant) >>= W
template <int W>
BM_DEV void shr256_window(uint64_t (&s)[4]) {
  s[0] = (s[0] >> W) | (s[1] << (64 - W));
  s[1] = (s[1] >> W) | (s[2] << (64 - W));
  s[2] = (s[2] >> W) | (s[3] << (64 - W));
  s[3] >>= W;
}

// k*G for the 256-bit scalar given as 4 big-endian 64-bit words (k = w0*2^192 + ... + w3),
// i.e. the first 32 bytes of a SHA-512 digest read as a big-endian integer (BN_bin2bn), left in
// Jacobian coordinates (acc.inf for k*G = infinity, i.e. k = 0 mod n).  Windows are peeled off
// the low end of a 256-bit shift register (no runtime-indexed register arrays), and the next
// window's table entry is loaded before the current addition, so the gather's latency hides
// behind ~2,500 VALU instructions.
template <int W, bool kDouble>
BM_DEV bool comb_pass(gej& acc, const ge* __restrict__ table, const uint64_t (&kw)[4]) {
  using C = comb<W>;
  uint64_t s[4] = {kw[3], kw[2], kw[1], kw[0]};
  acc.inf = true;
  bool ok = true;
  uint32_t v = (uint32_t)s[0] & C::kMask;
  ge q = table[v];
#pragma unroll 1
  for (int i = 0; i < C::kWindows; ++i) {
    shr256_window<W>(s);
    const uint32_t vn = (uint32_t)s[0] & C::kMask;
    ge qn;
    if (i + 1 < C::kWindows) qn = table[((size_t)(i + 1) << W) | vn];
    if (v) ok = gej_add_ge_t<kDouble>(acc, acc, q) && ok;
    q = qn;
    v = vn;
  }
  return ok;
}

template <int W>
BM_DEV void scalar_mult_base_jac(gej& acc, const ge* __restrict__ table, const uint64_t (&kw)[4]) {
  // An addition of a point to itself would send the lane through the pass with the doubling
  // path.  For scalars < 2^256 it cannot happen: before window i the sum is (k mod 2^(W i)) G and
  // the entry is v 2^(W i) G with k mod 2^(W i) < v 2^(W i) < n (W i <= 240).  The opposite
  // case (sum + entry = n G, only k = n) gives infinity on the fast pass.
  if (!comb_pass<W, false>(acc, table, kw)) comb_pass<W, true>(acc, table, kw);
}

// k*G in affine coordinates; returns false for k*G = infinity.
template <int W>
BM_DEV bool scalar_mult_base(ge& r, const ge* __restrict__ table, const uint64_t (&kw)[4]) {
  gej acc;
  scalar_mult_base_jac<W>(acc, table, kw);
  if (acc.inf) return false;
  gej_to_ge(r, acc);
  return true;
}

// Two Jacobian points (neither at infinity) to affine with ONE inversion (Montgomery's trick):
// i = (Za Zb)^-1, Za^-1 = i Zb, Zb^-1 = i Za.  The inversion is ~270 multiplications against
// ~180 for a whole comb, so sharing it between the two keys of a try saves ~30 % of the try.
BM_DEV void gej_pair_to_ge(ge& ra, ge& rb, const gej& a, const gej& b) {
  fe zab, i, zia, zib, t;
  fe_mul(zab, a.z, b.z);
  fe_inv(i, zab);
  fe_mul(zia, i, b.z);
  fe_mul(zib, i, a.z);
  fe_sqr(t, zia);
  fe_mul(ra.x, a.x, t);
  fe_mul(t, t, zia);
  fe_mul(ra.y, a.y, t);
  fe_sqr(t, zib);
  fe_mul(rb.x, b.x, t);
  fe_mul(t, t, zib);
  fe_mul(rb.y, b.y, t);
  fe_normalize(ra.x, ra.x);
  fe_normalize(ra.y, ra.y);
  fe_normalize(rb.x, rb.x);
  fe_normalize(rb.y, rb.y);
}

// 4 big-endian 64-bit words of a canonical field element (the 32-byte big-endian serialization)
BM_DEV void fe_to_be64(uint64_t (&w)[4], const fe& a) {
  w[0] = ((uint64_t)a.d[7] << 32) | a.d[6];
  w[1] = ((uint64_t)a.d[5] << 32) | a.d[4];
  w[2] = ((uint64_t)a.d[3] << 32) | a.d[2];
  w[3] = ((uint64_t)a.d[1] << 32) | a.d[0];
}

}  // namespace ec
