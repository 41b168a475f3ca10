// sha512_dev.h -- gfx950 device primitives for the Bitmessage trial function.
//
// trial(n, ih) = BE64(SHA512(SHA512(BE64(n) || ih))[0:8])     (reference:
// src/proofofwork.py:106-107, docs/pow.rst:42-49).  In SHA-512 words no byte swap is
// needed anywhere: block 1 is W0 = n, W1..8 = ih as big-endian u64, W9 = 0x80.., W15 = 576;
// block 2 is W0..7 = H(block 1), W8 = 0x80.., W15 = 512; trial = IV0 + a80(block 2).
//
// All arithmetic is 32-bit VALU on register pairs:
//   ROTR64  -> 2 x v_alignbit_b32          (explicit builtin; hipcc's default lowering of
//                                           (x>>n)|(x<<64-n) emits 64-bit shifts + ORs)
//   XOR3 / Ch / Maj -> 2 x v_bitop3_b32   (gfx950 3-input LUT op, selected by the compiler)
//   ADD64   -> v_lshl_add_u64 (gfx950)    (selected by the compiler for uint64_t +)
#pragma once
#include <stdint.h>

#define BM_DEV __device__ __forceinline__

namespace bm {

// FIPS 180-4 4.2.3 / 5.3.5 constants (compile-time: every round index is a constant).
constexpr uint64_t K(int t) {
  constexpr uint64_t k[80] = {
      0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
      0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
      0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
      0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
      0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
      0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
      0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
      0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
      0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
      0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
      0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
      0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
      0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
      0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
      0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
      0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
      0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
      0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
      0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
      0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};
  return k[t];
}

constexpr uint64_t IV(int i) {
  constexpr uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                              0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                              0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  return iv[i];
}

// ---- 64-bit rotates / shifts on 32-bit halves via v_alignbit_b32 ----
BM_DEV uint32_t lo32(uint64_t x) { return (uint32_t)x; }
BM_DEV uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
BM_DEV uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

template <int N>
BM_DEV uint64_t rotr(uint64_t x) {
  static_assert(N > 0 && N < 64, "rotate");
  const uint32_t l = lo32(x), h = hi32(x);
  if constexpr (N < 32) {
    return mk64(__builtin_amdgcn_alignbit(h, l, N), __builtin_amdgcn_alignbit(l, h, N));
  } else if constexpr (N == 32) {
    return mk64(h, l);
  } else {
    return mk64(__builtin_amdgcn_alignbit(l, h, N - 32), __builtin_amdgcn_alignbit(h, l, N - 32));
  }
}

// SHR64 (sigma0/sigma1's third term) as ONE v_lshrrev_b64: the same half rate as v_alignbit_b32
// (63.6 vs 63.2 lane-ops/clk/CU, tools/ubench_valu.hip), replacing the alignbit + v_lshrrev_b32
// pair LLVM selects for x >> N.  Inline asm because the backend always splits the 64-bit shift.
// kSplit: the builtin form, for the sigma terms of per-object (wave-uniform) words, which LICM must
// be able to hoist out of the nonce loop -- it never hoists the asm.
template <int N, bool kSplit = false>
BM_DEV uint64_t shr(uint64_t x) {
  static_assert(N > 0 && N < 32, "shift");
#ifndef BM_SHR_SPLIT
  if constexpr (!kSplit) {
    uint64_t r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
    return r;
  }
#endif
  const uint32_t l = lo32(x), h = hi32(x);
  return mk64(__builtin_amdgcn_alignbit(h, l, N), h >> N);
}

// ---- 3-input bitwise functions as one v_bitop3_b32 per 32-bit half ----
// Measured on MI355X (tools/ubench_valu.hip): v_bitop3_b32 issues at ~77 lane-ops/clk/CU,
// v_xor_b32 at ~118 and v_bfi_b32 at ~63, so one bitop3 (1/77) beats the xor pair the
// compiler selects for a^b^c (2/118) and the bfi it selects for Ch.  hipcc does not form
// bitop3 for two-op trees by itself, hence the builtin.  LUT bits: S0 = 0xF0, S1 = 0xCC,
// S2 = 0xAA.
template <uint8_t LUT>
BM_DEV uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
  // No constant-folding path: a __builtin_constant_p branch here is resolved only late in the
  // pipeline, so every call dragged a folding body through inlining and scheduling (the
  // SHA-512 compression took ~5 min to compile).  No call site has three constant operands.
  return __builtin_amdgcn_bitop3_b32(a, b, c, LUT);
}

// A 64-bit value rebuilt from two 32-bit halves is ((u64)hi << 32) | lo to LLVM, which
// rewrites the OR as an ADD and then reassociates every following 64-bit add into separate
// lo/hi adds (measured: +35% v_lshl_add_u64 and ~850 extra v_mov per trial).  An empty asm
// with a read-write VGPR-pair operand makes the pair opaque at zero instruction cost.
BM_DEV uint64_t opaque(uint64_t x) {
  if (__builtin_constant_p(x)) return x;
  asm("" : "+v"(x));
  return x;
}

// kHoist: a per-object (wave-uniform) value LICM hoists out of the nonce loop -- no opaque barrier,
// which would pin a register copy of it inside the loop.
template <uint8_t LUT, bool kHoist = false>
BM_DEV uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
  const uint64_t r = mk64(bitop3<LUT>(lo32(a), lo32(b), lo32(c)), bitop3<LUT>(hi32(a), hi32(b), hi32(c)));
  if constexpr (kHoist) return r;
  return opaque(r);
}

// 64-bit add of two nonce-dependent values.  Default: the compiler's v_lshl_add_u64 (one VOP3,
// half rate).  BM_ADD64_VOP2 (A/B variant): v_add_co_u32_e32 +
// v_addc_co_u32_e32, the VOP2 pair with the carry in VCC.
BM_DEV uint64_t add64(uint64_t a, uint64_t b) {
#ifdef BM_ADD64_VOP2
  if (!(__builtin_constant_p(a) && __builtin_constant_p(b))) {
    uint32_t lo, hi;
    asm("v_add_co_u32_e32 %0, vcc, %2, %3\n\tv_addc_co_u32_e32 %1, vcc, %4, %5, vcc"
        : "=&v"(lo), "=v"(hi)
        : "v"(lo32(a)), "v"(lo32(b)), "v"(hi32(a)), "v"(hi32(b))
        : "vcc");
    return opaque(mk64(lo, hi));
  }
#endif
  return a + b;
}

template <bool kHoist = false>
BM_DEV uint64_t xor3(uint64_t a, uint64_t b, uint64_t c) { return bitop3_64<0x96, kHoist>(a, b, c); }

// FIPS 180-4 4.1.3 functions.
BM_DEV uint64_t Sig0(uint64_t a) { return xor3(rotr<28>(a), rotr<34>(a), rotr<39>(a)); }
BM_DEV uint64_t Sig1(uint64_t e) { return xor3(rotr<14>(e), rotr<18>(e), rotr<41>(e)); }
template <bool kSplit = false>
BM_DEV uint64_t sig0(uint64_t w) {
  if (__builtin_constant_p(w)) return (w >> 1 | w << 63) ^ (w >> 8 | w << 56) ^ (w >> 7);
  return xor3<kSplit>(rotr<1>(w), rotr<8>(w), shr<7, kSplit>(w));
}
template <bool kSplit = false>
BM_DEV uint64_t sig1(uint64_t w) {
  if (__builtin_constant_p(w)) return (w >> 19 | w << 45) ^ (w >> 61 | w << 3) ^ (w >> 6);
  return xor3<kSplit>(rotr<19>(w), rotr<61>(w), shr<6, kSplit>(w));
}
BM_DEV uint64_t Ch(uint64_t e, uint64_t f, uint64_t g) { return bitop3_64<0xCA>(e, f, g); }
BM_DEV uint64_t Maj(uint64_t a, uint64_t b, uint64_t c) { return bitop3_64<0xE8>(a, b, c); }

// constexpr twins (host + device) for compile-time folding of IV-only expressions.
constexpr uint64_t crotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
constexpr uint64_t cSig0(uint64_t a) { return crotr(a, 28) ^ crotr(a, 34) ^ crotr(a, 39); }
constexpr uint64_t cSig1(uint64_t e) { return crotr(e, 14) ^ crotr(e, 18) ^ crotr(e, 41); }
constexpr uint64_t csig0(uint64_t w) { return crotr(w, 1) ^ crotr(w, 8) ^ (w >> 7); }
constexpr uint64_t csig1(uint64_t w) { return crotr(w, 19) ^ crotr(w, 61) ^ (w >> 6); }
constexpr uint64_t cCh(uint64_t e, uint64_t f, uint64_t g) { return (e & f) ^ (~e & g); }
constexpr uint64_t cMaj(uint64_t a, uint64_t b, uint64_t c) { return (a & b) ^ (a & c) ^ (b & c); }

// Round 0 from the IV with W0 the only unknown (both blocks start from the IV):
//   T1 = T1C + W0,  a1 = W0 + A1C,  e1 = W0 + E1C
constexpr uint64_t T1C = IV(7) + cSig1(IV(4)) + cCh(IV(4), IV(5), IV(6)) + K(0);
constexpr uint64_t A1C = T1C + cSig0(IV(0)) + cMaj(IV(0), IV(1), IV(2));
constexpr uint64_t E1C = IV(3) + T1C;

constexpr uint64_t PAD = 0x8000000000000000ULL;

// ---------------------------------------------------------------------------------------
// Generic fully-unrolled SHA-512 rounds.  State slot of a at round T is (-T) & 7; every
// index below is a compile-time constant after template expansion, so s[] and w[] live in
// VGPR/SGPR pairs (verified: no scratch in the ISA).
// ---------------------------------------------------------------------------------------
// kTrial1: block 1 of the trial, whose W1..W8 are the object's (wave-uniform) initialHash words: the
// sigma0 of W1..W8 (T = 16..23) and the sigma1 of the uniform W17, W19, W21 (T = 19, 21, 23) take the
// hoistable builtin form.
// kVar0: block 0 of a trial over an initialHash of any other length (trial_var): W1..W15 are all
// per-object (uniform, not compile-time), so the sigma0 of W1..W15 (T = 16..30) and the sigma1 of
// W14, W15, W17, W19, W21 (T = 16, 17, 19, 21, 23) are hoistable.
template <int T, bool kTrial1 = false, bool kVar0 = false>
BM_DEV void round_step(uint64_t (&s)[8], uint64_t (&w)[16]) {
  constexpr int A = (8 - (T & 7)) & 7;
  constexpr int B = (A + 1) & 7, C = (A + 2) & 7, D = (A + 3) & 7;
  constexpr int E = (A + 4) & 7, F = (A + 5) & 7, G = (A + 6) & 7, H = (A + 7) & 7;
  if constexpr (T >= 16) {
    constexpr bool kU0 = (kTrial1 && T <= 23) || (kVar0 && T <= 30);
    constexpr bool kU1 = (kTrial1 && (T == 19 || T == 21 || T == 23)) ||
                         (kVar0 && (T == 16 || T == 17 || T == 19 || T == 21 || T == 23));
    // grouped so the terms that do not depend on the nonce (per-object or compile-time)
    // are summed first and hoisted out of the nonce loop by LICM
    w[T & 15] = (w[(T - 7) & 15] + sig0<kU0>(w[(T - 15) & 15]) + w[(T - 16) & 15]) + sig1<kU1>(w[(T - 2) & 15]);
  }
#ifdef BM_GROUP_BITOP3
  // A/B variant: the round's eight 3-input ops (Sigma1 / Sigma0 XOR3, Ch, Maj on both halves) issue
  // back to back, so waves sharing a SIMD meet at them together more often (they co-issue only
  // with each other); rotates and adds stay the compiler's.
  const uint64_t e = s[E], a = s[A];
  const uint64_t r14 = rotr<14>(e), r18 = rotr<18>(e), r41 = rotr<41>(e);
  const uint64_t r28 = rotr<28>(a), r34 = rotr<34>(a), r39 = rotr<39>(a);
  uint32_t s1l, s1h, s0l, s0h, chl, chh, mjl, mjh;
  asm("v_bitop3_b32 %0, %8, %9, %10 bitop3:0x96\n\t"
      "v_bitop3_b32 %1, %11, %12, %13 bitop3:0x96\n\t"
      "v_bitop3_b32 %2, %14, %15, %16 bitop3:0x96\n\t"
      "v_bitop3_b32 %3, %17, %18, %19 bitop3:0x96\n\t"
      "v_bitop3_b32 %4, %20, %21, %22 bitop3:0xca\n\t"
      "v_bitop3_b32 %5, %23, %24, %25 bitop3:0xca\n\t"
      "v_bitop3_b32 %6, %26, %27, %28 bitop3:0xe8\n\t"
      "v_bitop3_b32 %7, %29, %30, %31 bitop3:0xe8"
      : "=&v"(s1l), "=&v"(s1h), "=&v"(s0l), "=&v"(s0h), "=&v"(chl), "=&v"(chh), "=&v"(mjl), "=&v"(mjh)
      : "v"(lo32(r14)), "v"(lo32(r18)), "v"(lo32(r41)), "v"(hi32(r14)), "v"(hi32(r18)), "v"(hi32(r41)),
        "v"(lo32(r28)), "v"(lo32(r34)), "v"(lo32(r39)), "v"(hi32(r28)), "v"(hi32(r34)), "v"(hi32(r39)),
        "v"(lo32(e)), "v"(lo32(s[F])), "v"(lo32(s[G])), "v"(hi32(e)), "v"(hi32(s[F])), "v"(hi32(s[G])),
        "v"(lo32(a)), "v"(lo32(s[B])), "v"(lo32(s[C])), "v"(hi32(a)), "v"(hi32(s[B])), "v"(hi32(s[C])));
  const uint64_t t1 = add64(add64(add64(s[H], opaque(mk64(s1l, s1h))), opaque(mk64(chl, chh))), K(T) + w[T & 15]);
  s[D] = add64(s[D], t1);
  s[H] = add64(add64(t1, opaque(mk64(s0l, s0h))), opaque(mk64(mjl, mjh)));
#else
  const uint64_t t1 = add64(add64(add64(s[H], Sig1(s[E])), Ch(s[E], s[F], s[G])), K(T) + w[T & 15]);
  s[D] = add64(s[D], t1);
  s[H] = add64(add64(t1, Sig0(s[A])), Maj(s[A], s[B], s[C]));
#endif
}

template <int T, int END, bool kTrial1 = false, bool kVar0 = false>
BM_DEV void rounds(uint64_t (&s)[8], uint64_t (&w)[16]) {
  if constexpr (T < END) {
    round_step<T, kTrial1, kVar0>(s, w);
    rounds<T + 1, END, kTrial1, kVar0>(s, w);
  }
}

#ifdef BM_HETERO
// A/B variant (BM_HETERO): the same dataflow in another instruction order, for
// the odd waves of each workgroup, so the waves sharing a SIMD run different streams.  Rounds 16..79
// go in groups of 8: the group's eight schedule words first (sigma0 / sigma1: rotates and shifts),
// then its eight rounds (Sigma, Ch, Maj: the v_bitop3_b32-rich part), with scheduling barriers
// between the phases so the compiler keeps them apart.
template <int T, int END, bool kTrial1>
BM_DEV void sched_words(uint64_t (&w)[16]) {
  if constexpr (T < END) {
    constexpr bool kU0 = kTrial1 && T <= 23;
    constexpr bool kU1 = kTrial1 && (T == 19 || T == 21 || T == 23);
    w[T & 15] = (w[(T - 7) & 15] + sig0<kU0>(w[(T - 15) & 15]) + w[(T - 16) & 15]) + sig1<kU1>(w[(T - 2) & 15]);
    sched_words<T + 1, END, kTrial1>(w);
  }
}
template <int T, int END>
BM_DEV void rounds_only(uint64_t (&s)[8], const uint64_t (&w)[16]) {
  if constexpr (T < END) {
    constexpr int A = (8 - (T & 7)) & 7;
    constexpr int B = (A + 1) & 7, C = (A + 2) & 7, D = (A + 3) & 7;
    constexpr int E = (A + 4) & 7, F = (A + 5) & 7, G = (A + 6) & 7, H = (A + 7) & 7;
    const uint64_t t1 = add64(add64(add64(s[H], Sig1(s[E])), Ch(s[E], s[F], s[G])), K(T) + w[T & 15]);
    s[D] = add64(s[D], t1);
    s[H] = add64(add64(t1, Sig0(s[A])), Maj(s[A], s[B], s[C]));
    rounds_only<T + 1, END>(s, w);
  }
}
template <int T, bool kTrial1>
BM_DEV void rounds_grouped(uint64_t (&s)[8], uint64_t (&w)[16]) {
  if constexpr (T < 80) {
    sched_words<T, T + 8, kTrial1>(w);
    __builtin_amdgcn_sched_barrier(0);
    rounds_only<T, T + 8>(s, w);
    __builtin_amdgcn_sched_barrier(0);
    rounds_grouped<T + 8, kTrial1>(s, w);
  }
}
#endif

// Rounds of a block whose whole message schedule is per-object: kw[t] = K[t] + W[t] precomputed on
// the host (the later blocks of a long initialHash's first hash, bmsched::pack_var), read with
// uniform (scalar) loads, so a round is its state update alone.
template <int T, int END>
BM_DEV void rounds_kw(uint64_t (&s)[8], const uint64_t* __restrict__ kw) {
  if constexpr (T < END) {
    constexpr int A = (8 - (T & 7)) & 7;
    constexpr int B = (A + 1) & 7, C = (A + 2) & 7, D = (A + 3) & 7;
    constexpr int E = (A + 4) & 7, F = (A + 5) & 7, G = (A + 6) & 7, H = (A + 7) & 7;
    const uint64_t t1 = add64(add64(add64(s[H], Sig1(s[E])), Ch(s[E], s[F], s[G])), kw[T]);
    s[D] = add64(s[D], t1);
    s[H] = add64(add64(t1, Sig0(s[A])), Maj(s[A], s[B], s[C]));
    rounds_kw<T + 1, END>(s, kw);
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
  rounds<1, 80, true>(s, w);
#ifdef BM_TRIAL_MID
  BM_TRIAL_MID();  // A/B hook of the search kernel (bmpow_kernels.hip), nothing elsewhere
#endif
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

// trial_of with a test between its two compressions: when stop() (wave-uniform) holds, the second is
// skipped and *cut is set (the single-object kernel's mid-trial bound check, bmpow_kernels.hip sweep).
// Kept apart from trial_of: passing the state between two halves through an array made the compiler
// emit ~105 more VALU per trial in every caller (PMC, profiles/r04/eng6/).
template <class Stop>
BM_DEV uint64_t trial_of_cut(const uint64_t (&ihw)[8], uint64_t nonce, Stop&& stop, bool& cut) {
  uint64_t w[16];
  w[0] = nonce;
#pragma unroll
  for (int i = 0; i < 8; ++i) w[1 + i] = ihw[i];
  w[9] = PAD;
#pragma unroll
  for (int i = 10; i < 15; ++i) w[i] = 0;
  w[15] = 72 * 8;
  uint64_t s[8] = {IV(0), IV(1), IV(2), nonce + E1C, IV(4), IV(5), IV(6), nonce + A1C};
  rounds<1, 80, true>(s, w);
  cut = stop();
  if (cut) return ~0ULL;
  uint64_t w2[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w2[i] = s[i] + IV(i);
  w2[8] = PAD;
#pragma unroll
  for (int i = 9; i < 15; ++i) w2[i] = 0;
  w2[15] = 64 * 8;
  uint64_t s2[8] = {IV(0), IV(1), IV(2), w2[0] + E1C, IV(4), IV(5), IV(6), w2[0] + A1C};
#ifdef BM_CUT2  // A/B variant: a second test halfway through the second compression
  rounds<1, 40>(s2, w2);
  cut = stop();
  if (cut) return ~0ULL;
  rounds<40, 80>(s2, w2);
#else
  rounds<1, 80>(s2, w2);
#endif
  return s2[0] + IV(0);
}

#ifdef BM_HETERO
// trial_of with rounds 16..79 of both blocks in rounds_grouped's order (the A/B variant above).
BM_DEV uint64_t trial_of_b(const uint64_t (&ihw)[8], uint64_t nonce) {
  uint64_t w[16];
  w[0] = nonce;
#pragma unroll
  for (int i = 0; i < 8; ++i) w[1 + i] = ihw[i];
  w[9] = PAD;
#pragma unroll
  for (int i = 10; i < 15; ++i) w[i] = 0;
  w[15] = 72 * 8;
  uint64_t s[8] = {IV(0), IV(1), IV(2), nonce + E1C, IV(4), IV(5), IV(6), nonce + A1C};
  rounds<1, 16, true>(s, w);
  rounds_grouped<16, true>(s, w);
  uint64_t w2[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w2[i] = s[i] + IV(i);
  w2[8] = PAD;
#pragma unroll
  for (int i = 9; i < 15; ++i) w2[i] = 0;
  w2[15] = 64 * 8;
  uint64_t s2[8] = {IV(0), IV(1), IV(2), w2[0] + E1C, IV(4), IV(5), IV(6), w2[0] + A1C};
  rounds<1, 16>(s2, w2);
  rounds_grouped<16, false>(s2, w2);
  return s2[0] + IV(0);
}
#endif

// trial(n, ih) for an initialHash of any length L != 64 (the reference hashes pack('>Q', n) + ih as
// given, src/proofofwork.py:104-107).  The first hash's message BE64(n) || ih || padding is
// nblk = ceil((8 + L + 17) / 128) blocks (bmsched::pack_var lays out the per-object words):
//   mw[1..15]  block 0's words after the nonce (ih bytes, the 0x80 pad, the bit length when it fits);
//   kw[80 (j-1) .. 80 j)  K[t] + W[t] of block j = 1 .. nblk-1 (those blocks hold no nonce bit).
// Block 0 starts from the IV with W0 = n, so round 0 folds as in trial_of; the second hash is the
// one-block digest hash of trial_of.
BM_DEV uint64_t trial_var(const uint64_t (&mw)[16], const uint64_t* __restrict__ kw, uint32_t nblk,
                          uint64_t nonce) {
  uint64_t w[16];
  w[0] = nonce;
#pragma unroll
  for (int i = 1; i < 16; ++i) w[i] = mw[i];
  uint64_t s[8] = {IV(0), IV(1), IV(2), nonce + E1C, IV(4), IV(5), IV(6), nonce + A1C};
  rounds<1, 80, false, true>(s, w);
  uint64_t h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = s[i] + IV(i);
  for (uint32_t j = 1; j < nblk; ++j) {
    uint64_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = h[i];
    rounds_kw<0, 80>(t, kw + (size_t)80 * (j - 1));
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = opaque(h[i] + t[i]);
  }
  uint64_t w2[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) w2[i] = h[i];
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
