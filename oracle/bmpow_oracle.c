/*
 * bmpow_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's proof-of-work algorithm, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * pybitmessage_amd/ links, loads or calls this file.
 *
 *   trial(n, ih)  = BE64( SHA512( SHA512( BE64(n) || ih ) )[0:8] )
 *                   reference: src/proofofwork.py:106-107, docs/pow.rst:42-49
 *   first nonce   = min{ n >= start : trial(n, ih) <= target }
 *                   reference: _doSafePoW, src/proofofwork.py:100-111 (start = 1, `<=`)
 *
 * SHA-512 is restated from FIPS 180-4 section 6.4 (the reference delegates it to
 * OpenSSL libcrypto via hashlib / SHA512_* -- SURVEY.md 8(c)); this restatement is
 * pinned against hashlib and the golden vectors in tests/golden/.
 *
 * The multi-threaded search (bmo_search_mt) is the CPU baseline "port" of the
 * reference's _doCPoW mechanism (src/bitmsghash/bitmsghash.cpp:39-165: N pthreads over
 * the nonce space) but with the exact _doSafePoW answer: threads pull ascending
 * fixed-size chunks from an atomic counter and stop pulling chunks above the best hit.
 */
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

static const uint64_t K512[80] = {
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

/* the table itself, for the scheduler simulator's CPU stand-in (tests/native/sched_sim.cpp) */
const uint64_t *bmo_k512(void) { return K512; }

static const uint64_t IV512[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static inline uint64_t ror64(uint64_t x, unsigned n) { return (x >> n) | (x << (64 - n)); }

static uint64_t load_be64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return v;
}

static void store_be64(uint8_t *p, uint64_t v) {
    for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)v; v >>= 8; }
}

/* FIPS 180-4 6.4.2: one compression of a 16-word block into state h[8]. */
static void compress(uint64_t h[8], const uint64_t blk[16]) {
    uint64_t w[80];
    for (int t = 0; t < 16; t++) w[t] = blk[t];
    for (int t = 16; t < 80; t++) {
        uint64_t s0 = ror64(w[t - 15], 1) ^ ror64(w[t - 15], 8) ^ (w[t - 15] >> 7);
        uint64_t s1 = ror64(w[t - 2], 19) ^ ror64(w[t - 2], 61) ^ (w[t - 2] >> 6);
        w[t] = s1 + w[t - 7] + s0 + w[t - 16];
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 80; t++) {
        uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
        uint64_t ch = (e & f) ^ (~e & g);
        uint64_t t1 = hh + S1 + ch + K512[t] + w[t];
        uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
        uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint64_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* General SHA-512 (FIPS 180-4 5.1.2 padding), any length < 2^61 bytes. */
void bmo_sha512(const uint8_t *msg, size_t len, uint8_t out[64]) {
    uint64_t h[8], blk[16];
    memcpy(h, IV512, sizeof h);
    size_t off = 0;
    for (; off + 128 <= len; off += 128) {
        for (int i = 0; i < 16; i++) blk[i] = load_be64(msg + off + 8 * i);
        compress(h, blk);
    }
    uint8_t tail[256];
    size_t rem = len - off;
    memset(tail, 0, sizeof tail);
    memcpy(tail, msg + off, rem);
    tail[rem] = 0x80;
    size_t tlen = (rem + 1 + 16 <= 128) ? 128 : 256;
    store_be64(tail + tlen - 8, (uint64_t)len << 3);
    store_be64(tail + tlen - 16, (uint64_t)(len >> 61));
    for (size_t b = 0; b < tlen; b += 128) {
        for (int i = 0; i < 16; i++) blk[i] = load_be64(tail + b + 8 * i);
        compress(h, blk);
    }
    for (int i = 0; i < 8; i++) store_be64(out + 8 * i, h[i]);
}

/* trial(n, ih): reference src/proofofwork.py:106-107.  The 72-byte first message is one
 * padded block (W9 = 0x80.., W15 = 576 bits); the 64-byte digest is one block (W15 = 512). */
uint64_t bmo_trial(const uint8_t ih[64], uint64_t nonce) {
    uint64_t h[8], blk[16];
    memcpy(h, IV512, sizeof h);
    blk[0] = nonce;
    for (int i = 0; i < 8; i++) blk[1 + i] = load_be64(ih + 8 * i);
    blk[9] = 0x8000000000000000ULL;
    for (int i = 10; i < 15; i++) blk[i] = 0;
    blk[15] = 72 * 8;
    compress(h, blk);
    for (int i = 0; i < 8; i++) blk[i] = h[i];
    blk[8] = 0x8000000000000000ULL;
    for (int i = 9; i < 15; i++) blk[i] = 0;
    blk[15] = 64 * 8;
    memcpy(h, IV512, sizeof h);
    compress(h, blk);
    return h[0];
}

/* trial(n, ih) for an initialHash of any length: the reference hashes pack('>Q', n) + ih as given
 * (src/proofofwork.py:104-107), so the first hash is the general SHA-512 of 8 + len bytes. */
uint64_t bmo_trial_len(const uint8_t *ih, size_t len, uint64_t nonce) {
    uint8_t stackbuf[8 + 256], *msg = stackbuf, h1[64], h2[64];
    if (len > 256) {
        msg = (uint8_t *)malloc(8 + len);
        if (!msg) return 0;
    }
    store_be64(msg, nonce);
    if (len) memcpy(msg + 8, ih, len);
    bmo_sha512(msg, 8 + len, h1);
    bmo_sha512(h1, 64, h2);
    if (msg != stackbuf) free(msg);
    return load_be64(h2);
}

/* _doSafePoW over an initialHash of any length, with a budget (as bmo_search). */
int bmo_search_len(const uint8_t *ih, size_t len, uint64_t target, uint64_t start, uint64_t max_trials,
                   uint64_t *nonce_out, uint64_t *trial_out) {
    for (uint64_t i = 0; i < max_trials; i++) {
        uint64_t n = start + i;
        uint64_t tv = bmo_trial_len(ih, len, n);
        if (tv <= target) { *nonce_out = n; *trial_out = tv; return 1; }
        if (n == UINT64_MAX) break;
    }
    return 0;
}

void bmo_trials(const uint8_t ih[64], const uint64_t *nonces, size_t n, uint64_t *out) {
    for (size_t i = 0; i < n; i++) out[i] = bmo_trial(ih, nonces[i]);
}

/* Sequential scan, _doSafePoW restated (src/proofofwork.py:100-111) with a trial budget:
 * tests start, start+1, ... start+max_trials-1 (never past 2^64-1).
 * returns 1 and the first hit, or 0 when the budget ran out. */
int bmo_search(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials,
               uint64_t *nonce_out, uint64_t *trial_out) {
    for (uint64_t i = 0; i < max_trials; i++) {
        uint64_t n = start + i;
        uint64_t tv = bmo_trial(ih, n);
        if (tv <= target) { *nonce_out = n; *trial_out = tv; return 1; }
        if (n == UINT64_MAX) break;
    }
    return 0;
}

/* Minimum trial value over [start, start+count) (never past 2^64-1) and the FIRST nonce that
 * reaches it -- the checker for the device probe bmpow_min_trial.  Minimality of a search
 * answer n follows from min over [1, n) > target (no earlier nonce satisfies _doSafePoW's
 * `trialValue <= target`, src/proofofwork.py:104).  count == 0: *min_out = UINT64_MAX and
 * *argmin_out = start, returns 0; else returns 1. */
int bmo_min_trial(const uint8_t ih[64], uint64_t start, uint64_t count, uint64_t *min_out,
                  uint64_t *argmin_out) {
    uint64_t best = UINT64_MAX, arg = start;
    int any = 0;
    for (uint64_t i = 0; i < count; i++) {
        uint64_t n = start + i;
        uint64_t tv = bmo_trial(ih, n);
        if (!any || tv < best) { best = tv; arg = n; any = 1; }
        if (n == UINT64_MAX) break;
    }
    *min_out = best;
    *argmin_out = arg;
    return any;
}

/* ---- multi-threaded exact search (CPU baseline port) ---- */
#define MT_CHUNK 4096u

typedef struct {
    const uint8_t *ih;
    uint64_t target, start, max_trials;
    uint64_t next_chunk;  /* atomic */
    uint64_t best;        /* atomic: min hit nonce offset (UINT64_MAX = none) */
    uint64_t done;        /* atomic: trials performed */
} mt_ctx;

static void *mt_worker(void *arg) {
    mt_ctx *c = (mt_ctx *)arg;
    uint64_t local_done = 0;
    for (;;) {
        uint64_t ck = __atomic_fetch_add(&c->next_chunk, 1, __ATOMIC_RELAXED);
        uint64_t off = ck * MT_CHUNK;
        if (off >= c->max_trials) break;
        if (off > __atomic_load_n(&c->best, __ATOMIC_RELAXED)) break;
        uint64_t cnt = c->max_trials - off < MT_CHUNK ? c->max_trials - off : MT_CHUNK;
        for (uint64_t j = 0; j < cnt; j++) {
            uint64_t tv = bmo_trial(c->ih, c->start + off + j);
            local_done++;
            if (tv <= c->target) {
                uint64_t o = off + j, cur = __atomic_load_n(&c->best, __ATOMIC_RELAXED);
                while (o < cur && !__atomic_compare_exchange_n(&c->best, &cur, o, 0,
                                                               __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
                break;
            }
        }
    }
    __atomic_fetch_add(&c->done, local_done, __ATOMIC_RELAXED);
    return NULL;
}

/* Exact first hit in [start, start+max_trials) on nthreads threads.  *performed gets the
 * number of trials actually hashed (for rate reporting).  returns 1 found / 0 budget out. */
int bmo_search_mt(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials,
                  int nthreads, uint64_t *nonce_out, uint64_t *trial_out, uint64_t *performed) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    /* never run past nonce 2^64-1 (the condition is false when start == 0) */
    if (max_trials && max_trials - 1 > UINT64_MAX - start) max_trials = UINT64_MAX - start + 1;
    mt_ctx c = {ih, target, start, max_trials, 0, UINT64_MAX, 0};
    pthread_t th[1024];
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, mt_worker, &c);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    if (performed) *performed = c.done;
    if (c.best == UINT64_MAX) return 0;
    *nonce_out = start + c.best;
    *trial_out = bmo_trial(ih, *nonce_out);
    return 1;
}
