// ripemd160_dev.h -- gfx950 RIPEMD-160 compression for the address search.
//
// The reference hashes sha512(pubSigningKey || pubEncryptionKey) with RIPEMD-160
// (src/class_addressGenerator.py:143,266 via src/fallback/__init__.py RIPEMD160Hash).  Fully
// unrolled over the 80 steps of both lines (compile-time message selection and rotations, so
// x[] stays in registers); the five boolean functions are one v_bitop3_b32 each
// (LUTs f1 0x96, f2 0xCA, f3 0x59, f4 0xE4, f5 0x2D over S0 = x, S1 = y, S2 = z); rotates are
// v_alignbit_b32.
#pragma once
#include <stdint.h>

#include "sha512_dev.h"  // bm::bitop3

namespace rmd {

constexpr int RL(int j) {
  constexpr int r[80] = {0, 1, 2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 7,  4,  13, 1,
                         10, 6, 15, 3,  12, 0,  9,  5,  2,  14, 11, 8,  3,  10, 14, 4,  9,  15, 8,  1,
                         2,  7, 0,  6,  13, 11, 5,  12, 1,  9,  11, 10, 0,  8,  12, 4,  13, 3,  7,  15,
                         14, 5, 6,  2,  4,  0,  5,  9,  7,  12, 2,  10, 14, 1,  3,  8,  11, 6,  15, 13};
  return r[j];
}
constexpr int RR(int j) {
  constexpr int r[80] = {5,  14, 7,  0,  9, 2,  11, 4,  13, 6,  15, 8,  1,  10, 3,  12, 6,  11, 3,  7,
                         0,  13, 5,  10, 14, 15, 8,  12, 4,  9,  1,  2,  15, 5,  1,  3,  7,  14, 6,  9,
                         11, 8,  12, 2,  10, 0,  4,  13, 8,  6,  4,  1,  3,  11, 15, 0,  5,  12, 2,  13,
                         9,  7,  10, 14, 12, 15, 10, 4,  1,  5,  8,  7,  6,  2,  13, 14, 0,  3,  9,  11};
  return r[j];
}
constexpr int SL(int j) {
  constexpr int s[80] = {11, 14, 15, 12, 5,  8,  7,  9,  11, 13, 14, 15, 6,  7,  9,  8,  7,  6,  8,  13,
                         11, 9,  7,  15, 7,  12, 15, 9,  11, 7,  13, 12, 11, 13, 6,  7,  14, 9,  13, 15,
                         14, 8,  13, 6,  5,  12, 7,  5,  11, 12, 14, 15, 14, 15, 9,  8,  9,  14, 5,  6,
                         8,  6,  5,  12, 9,  15, 5,  11, 6,  8,  13, 12, 5,  12, 13, 14, 11, 8,  5,  6};
  return s[j];
}
constexpr int SR(int j) {
  constexpr int s[80] = {8,  9,  9,  11, 13, 15, 15, 5,  7,  7,  8,  11, 14, 14, 12, 6,  9,  13, 15, 7,
                         12, 8,  9,  11, 7,  7,  12, 7,  6,  15, 13, 11, 9,  7,  15, 11, 8,  6,  6,  14,
                         12, 13, 5,  14, 13, 13, 7,  5,  15, 5,  8,  11, 14, 14, 6,  14, 6,  9,  12, 9,
                         12, 5,  15, 8,  8,  5,  12, 9,  12, 5,  14, 6,  8,  13, 6,  5,  15, 13, 11, 11};
  return s[j];
}
constexpr uint32_t KL(int rnd) {
  constexpr uint32_t k[5] = {0x00000000u, 0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xA953FD4Eu};
  return k[rnd];
}
constexpr uint32_t KR(int rnd) {
  constexpr uint32_t k[5] = {0x50A28BE6u, 0x5C4DD124u, 0x6D703EF3u, 0x7A6D76E9u, 0x00000000u};
  return k[rnd];
}
constexpr uint8_t LUT(int rnd) {
  constexpr uint8_t l[5] = {0x96, 0xCA, 0x59, 0xE4, 0x2D};
  return l[rnd];
}

template <int S>
BM_DEV uint32_t rol(uint32_t x) {
  return __builtin_amdgcn_alignbit(x, x, 32 - S);
}

template <int J>
BM_DEV void steps(uint32_t (&l)[5], uint32_t (&r)[5], const uint32_t (&x)[16]) {
  if constexpr (J < 80) {
    constexpr int rnd = J / 16;
    // left line: T = rol(A + f(B,C,D) + X + K, s) + E; A=E, E=D, D=rol(C,10), C=B, B=T
    uint32_t t = rol<SL(J)>(l[0] + bm::bitop3<LUT(rnd)>(l[1], l[2], l[3]) + x[RL(J)] + KL(rnd)) + l[4];
    l[0] = l[4];
    l[4] = l[3];
    l[3] = rol<10>(l[2]);
    l[2] = l[1];
    l[1] = t;
    // right line uses the functions in reverse order
    t = rol<SR(J)>(r[0] + bm::bitop3<LUT(4 - rnd)>(r[1], r[2], r[3]) + x[RR(J)] + KR(rnd)) + r[4];
    r[0] = r[4];
    r[4] = r[3];
    r[3] = rol<10>(r[2]);
    r[2] = r[1];
    r[1] = t;
    steps<J + 1>(l, r, x);
  }
}

// One compression of a 64-byte block given as 16 little-endian words.
BM_DEV void compress(uint32_t (&h)[5], const uint32_t (&x)[16]) {
  uint32_t l[5] = {h[0], h[1], h[2], h[3], h[4]};
  uint32_t r[5] = {h[0], h[1], h[2], h[3], h[4]};
  steps<0>(l, r, x);
  const uint32_t t = h[1] + l[2] + r[3];
  h[1] = h[2] + l[3] + r[4];
  h[2] = h[3] + l[4] + r[0];
  h[3] = h[4] + l[0] + r[1];
  h[4] = h[0] + l[1] + r[2];
  h[0] = t;
}

BM_DEV void init(uint32_t (&h)[5]) {
  h[0] = 0x67452301u;
  h[1] = 0xEFCDAB89u;
  h[2] = 0x98BADCFEu;
  h[3] = 0x10325476u;
  h[4] = 0xC3D2E1F0u;
}

// RIPEMD-160 of a 64-byte message given as 8 big-endian 64-bit words (a SHA-512 digest):
// block 1 is the digest (bytes read little-endian per 32-bit word), block 2 the padding.
BM_DEV void of_sha512_digest(uint32_t (&h)[5], const uint64_t (&hw)[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[2 * i] = __builtin_bswap32((uint32_t)(hw[i] >> 32));
    x[2 * i + 1] = __builtin_bswap32((uint32_t)hw[i]);
  }
  init(h);
#pragma unroll 1
  for (int b = 0; b < 2; ++b) {  // one compression body for both blocks
    compress(h, x);
    x[0] = 0x80u;
#pragma unroll
    for (int i = 1; i < 16; ++i) x[i] = 0;
    x[14] = 512;  // bit length, little-endian 64-bit
  }
}

}  // namespace rmd
