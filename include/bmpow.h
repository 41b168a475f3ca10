/*
 * bmpow.h -- C ABI of libbmpow_hip.so, the MI355X proof-of-work engine for PyBitmessage.
 *
 * Drop-in boundary for the reference's native PoW.  Plain pointers and
 * sizes only; loaded from Python with ctypes.CDLL exactly like the reference loads
 * bitmsghash.so (src/proofofwork.py:371-388).
 *
 * Semantics of every search entry point (the _doSafePoW contract,
 * src/proofofwork.py:100-111):
 *     trial(n, ih) = BE64(SHA512(SHA512(BE64(n) || ih))[0:8])
 *     answer       = min { n >= start : trial(n, ih) <= target }
 * Searches are BOUNDED (a trial budget per call) so the caller can poll its shutdown flag
 * between calls -- the pattern of dev/powinterrupttest.py:22-37 -- and bmpow_abort() stops
 * an in-flight call from another thread or a signal handler.
 *
 * Return codes: >= 0 success (meaning per function), < 0 error (BMPOW_E_*);
 * bmpow_last_error() describes the last error of the calling thread.
 *
 * Thread safety: all entry points may be called from any thread; they are serialised by an
 * internal first-come first-served mutex, the GIL is not needed.  A 64-byte bmpow_search holds a
 * second mutex of its own for its whole call (one such search at a time) and gives the first up while
 * it waits for its windows, so a batch session or service steps between them.
 */
#ifndef BMPOW_H
#define BMPOW_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__) || defined(__clang__)
#define BMPOW_API __attribute__((visibility("default")))
#else
#define BMPOW_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define BMPOW_ABI_VERSION 1

#define BMPOW_NOT_FOUND 0      /* budget exhausted, no hit: resume at start + trials */
#define BMPOW_FOUND 1          /* *nonce_out / *trial_out hold the exact first hit */
#define BMPOW_E_NODEV (-1)     /* no usable gfx950 device / HIP runtime failure at init */
#define BMPOW_E_HIP (-2)       /* HIP runtime error during a call */
#define BMPOW_E_ARG (-3)       /* invalid argument */
#define BMPOW_E_ABORTED (-4)   /* bmpow_abort() was called; nothing returned is final */
#define BMPOW_E_STATE (-5)     /* library not initialised / handle misuse */

/* Object state in bmpow_batch_results()/bmpow_search_batch() `done` arrays. */
#define BMPOW_PENDING 0
#define BMPOW_DONE_FOUND 1
#define BMPOW_DONE_EXHAUSTED 2 /* reached nonce 2^64-1 without a hit */
#define BMPOW_PARKED 3         /* in the table but not scheduled (bmpow_batch_set_pending) */
#define BMPOW_FREE 4           /* released slot (bmpow_batch_take_done), reused by bmpow_batch_add */
#define BMPOW_DONE_BADHASH 5   /* service with BMPOW_SERVICE_VERIFY: the device's answer failed the host re-check */

/* ---- lifecycle (replaces proofofwork.init / bmpow global, src/proofofwork.py:336-394) ---- */

/* Initialise the HIP runtime and select every visible gfx950 device (or those named by the
 * BMPOW_DEVICES env var, e.g. "0,1").  Idempotent.  Returns the number of devices in use
 * (> 0) or BMPOW_E_NODEV. */
BMPOW_API int bmpow_init(void);

/* Number of gfx950 devices visible to the process (>= 0), without selecting them. */
BMPOW_API int bmpow_device_count(void);

/* Use exactly these device ordinals for subsequent searches (n >= 1).  A device may be
 * listed more than once: each entry is a separate nonce shard with its own stream.
 * n == 0 selects every visible device; ids == NULL with n >= 1 the first n visible devices.
 * Returns the number of shards or < 0. */
BMPOW_API int bmpow_set_devices(const int *ids, int n);

/* SURVEY 8(b)'s `int bmpow_set_devices(int ndev)` form: the first ndev visible gfx950 devices
 * (1/2/4/8-GPU runs).  Same as bmpow_set_devices(NULL, ndev).  Returns the shard count or < 0. */
BMPOW_API int bmpow_set_device_count(int ndev);

/* Copy the active shard -> device map into ids[0..cap); returns the shard count. */
BMPOW_API int bmpow_get_devices(int *ids, int cap);

/* PCI bus id ("0000:75:00.0") of device ordinal `device` into out[0..len) (NUL-terminated); 0 or < 0.
 * Lets a multi-rank run show which physical GPU each rank drove (bench.py's per_rank). */
BMPOW_API int bmpow_device_pci_bus_id(int device, char *out, int len);

/* Per-shard search throughput the step planner weights its slices by (trials per ms, an
 * exponential average over launches of >= 2^24 trials; 0 = no sample yet) into rates[0..cap);
 * returns the shard count.  A shard's share of a multi-shard step is its rate over the mean,
 * clamped to [1/2, 2], once every shard has a sample (equal shares before). */
BMPOW_API int bmpow_get_shard_rates(double *rates, int cap);

/* Release all device memory and streams (bmpow_init may be called again). */
BMPOW_API void bmpow_shutdown(void);

/* Process exit: stop every live service's thread, then release everything bmpow_shutdown does plus the
 * streams the library keeps for the life of the process (run()'s and the rehearsal's CU-masked ones),
 * before the HIP runtime's own exit handlers run.  The library registers it with atexit() at its first
 * initialisation (after the runtime's handlers, so it runs before them); pybitmessage_amd._lib also runs it
 * from Python's atexit.  Idempotent; afterwards every initialising call fails with BMPOW_E_STATE.  A call
 * still running in another thread for 5 s leaves the library as it is. */
BMPOW_API void bmpow_atexit(void);

BMPOW_API const char *bmpow_last_error(void);
BMPOW_API const char *bmpow_version(void);

/* ---- interrupt (replaces the dead OpenCL shutdown check, src/openclpow.py:10,99) ---- */

/* Async-signal-safe.  In-flight and later searches return BMPOW_E_ABORTED at their next
 * step boundary (<= one launch, ~tens of ms) until bmpow_clear_abort(). */
BMPOW_API void bmpow_abort(void);
BMPOW_API void bmpow_clear_abort(void);

/* ---- the hot path ---- */

/* initialHash length.  Every caller in the reference passes a 64-byte sha512 digest
 * (src/class_singleWorker.py:233, src/api.py:1300), the layout the search kernel is specialised for;
 * the reference's _doSafePoW hashes pack('>Q', nonce) + initialHash as given, at any length
 * (src/proofofwork.py:104-107), so the *_len / *_var entry points take any length up to
 * BMPOW_MAX_IH_LEN bytes (a separate kernel, bm_search_var_kernel) with the same semantics. */
#ifndef BMPOW_MAX_IH_LEN
#define BMPOW_MAX_IH_LEN (1u << 20)
#endif

/* trial(nonces[i], ih) for i < n, computed on the first shard's device.
 * Parity probe for the trial function (reference src/proofofwork.py:106-107). */
BMPOW_API int bmpow_trials(const uint8_t ih[64], const uint64_t *nonces, size_t n, uint64_t *trials_out);
/* The same for an initialHash of ih_len bytes (any length <= BMPOW_MAX_IH_LEN). */
BMPOW_API int bmpow_trials_len(const uint8_t *ih, size_t ih_len, const uint64_t *nonces, size_t n,
                               uint64_t *trials_out);

/* Bounded single-object search of [start, start + max_trials) (never past 2^64-1), nonce
 * space sharded over the active devices: each window is cut into one interleaved piece per physical
 * device (shards sharing a device never split a window; bmpow_set_run_split), the pieces sharing the
 * running minimum through a host-pinned cross-device bound.  Replaces BitmessagePOW
 * (src/bitmsghash/bitmsghash.cpp:127-165) and do_opencl_pow (src/openclpow.py:77-111).
 * Returns BMPOW_FOUND with the exact first hit, BMPOW_NOT_FOUND, or < 0. */
BMPOW_API int bmpow_search(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials,
                 uint64_t *nonce_out, uint64_t *trial_out);
/* The same for an initialHash of ih_len bytes: _doSafePoW's answer for pack('>Q', n) + ih as given
 * (src/proofofwork.py:100-111) -- run(target, initialHash) for any initialHash. */
BMPOW_API int bmpow_search_len(const uint8_t *ih, size_t ih_len, uint64_t target, uint64_t start,
                               uint64_t max_trials, uint64_t *nonce_out, uint64_t *trial_out);

/* Bounded batch search: n objects (ihs: n x 64 bytes, targets: n), each resuming at
 * next_start[i] (in/out).  Spends about `budget` trials in total, then returns the number
 * of objects still pending (>= 0) or < 0.  For objects with done[i] = BMPOW_DONE_FOUND,
 * nonce_out[i]/trial_out[i] are final.  Objects already marked done on entry are skipped,
 * so calling it in a loop until it returns 0 solves the whole batch (run_batch). */
BMPOW_API int bmpow_search_batch(size_t n, const uint8_t *ihs, const uint64_t *targets, uint64_t *next_start,
                       uint64_t budget, uint64_t *nonce_out, uint64_t *trial_out, uint8_t *done);

/* Min-trial probe: *min_out = min{ trial(m, ih) : start <= m < start + count } (never past
 * 2^64-1) and *argmin_out = the first m reaching it; count == 0 gives UINT64_MAX and start.
 * It hashes every nonce of the range (no target, no early exit) and reduces, a code path apart
 * from the search's hit logic, so it proves a search answer n minimal at any size: n is the
 * _doSafePoW answer (src/proofofwork.py:100-111) iff trial(n) <= target and the min over
 * [1, n) is > target.  No reference counterpart (test and bench instrument).  0 or < 0. */
BMPOW_API int bmpow_min_trial(const uint8_t ih[64], uint64_t start, uint64_t count, uint64_t *min_out,
                              uint64_t *argmin_out);

/* The same for n objects (ihs: n x 64 bytes) with their own ranges, in one pass over the devices. */
BMPOW_API int bmpow_min_trial_batch(size_t n, const uint8_t *ihs, const uint64_t *start, const uint64_t *count,
                                    uint64_t *min_out, uint64_t *argmin_out);
/* The same for initialHashes of any length: object i is ihs[ih_off[i] .. ih_off[i+1]) (n + 1
 * ascending offsets). */
BMPOW_API int bmpow_min_trial_var(size_t n, const uint8_t *ihs, const uint64_t *ih_off, const uint64_t *start,
                                  const uint64_t *count, uint64_t *min_out, uint64_t *argmin_out);

/* ---- device-resident batch session (the object table stays in HBM across steps) ---- */
typedef struct bmpow_batch bmpow_batch;

/* Upload n objects; start may be NULL (every object starts at nonce 1). NULL on error. */
BMPOW_API bmpow_batch *bmpow_batch_create(size_t n, const uint8_t *ihs, const uint64_t *targets,
                                const uint64_t *start);

/* One bounded step of ~budget trials over the pending objects (0 = library default).
 * Returns the number of objects still pending (>= 0) or < 0. */
BMPOW_API int bmpow_batch_step(bmpow_batch *b, uint64_t budget);

/* Copy out per-object state; any pointer may be NULL. Returns the pending count. */
BMPOW_API int bmpow_batch_results(const bmpow_batch *b, uint64_t *nonce_out, uint64_t *trial_out,
                        uint8_t *done, uint64_t *next_start);

/* Restart every object at nonce `start` (NULL = 1) without re-uploading the object table
 * (used by bench.py to time repeated full solves with inputs already resident in HBM). */
BMPOW_API int bmpow_batch_reset(bmpow_batch *b, const uint64_t *start);

/* Park (pending = 0) or schedule (pending = 1) objects [first, first + count) of a session:
 * parked objects stay resident but bmpow_batch_step skips them; finished objects are not
 * affected.  Lets a caller feed a resident table in pieces (bench.py hands out pieces of one
 * global batch to the ranks on demand).  Returns the pending count or < 0. */
BMPOW_API int bmpow_batch_set_pending(bmpow_batch *b, size_t first, size_t count, int pending);

/* Append n objects to a live session (between steps; start may be NULL = nonce 1): they join the
 * next bmpow_batch_step.  Slots released by bmpow_batch_take_done are reused first, then the
 * table grows; slot_out[i] (may be NULL) receives object i's slot.  Only the new objects cross
 * PCIe.  Returns the pending count or < 0.  (The continuous-batching feed of worker.PowService:
 * producers join at any step boundary without a re-upload of the table.) */
BMPOW_API int bmpow_batch_add(bmpow_batch *b, size_t n, const uint8_t *ihs, const uint64_t *targets,
                              const uint64_t *start, uint32_t *slot_out);
/* bmpow_batch_add for initialHashes of any length (object i = ihs[ih_off[i] .. ih_off[i+1])). */
BMPOW_API int bmpow_batch_add_var(bmpow_batch *b, size_t n, const uint8_t *ihs, const uint64_t *ih_off,
                                  const uint64_t *targets, const uint64_t *start, uint32_t *slot_out);

/* Pop up to `cap` objects finished (FOUND or EXHAUSTED) since the last call, in the order the
 * steps finished them: slot, nonce, trial, done state (any output but slot_out may be NULL).
 * Their slots become BMPOW_FREE, for reuse by bmpow_batch_add.  Cost O(returned), so a caller
 * never scans the whole table per step.  Returns the count (>= 0) or < 0. */
BMPOW_API int bmpow_batch_take_done(bmpow_batch *b, size_t cap, uint32_t *slot_out, uint64_t *nonce_out,
                                    uint64_t *trial_out, uint8_t *done_out);

BMPOW_API void bmpow_batch_destroy(bmpow_batch *b);

/* ---- continuous-batching service: a library thread steps one resident session while producers
 *      submit and a consumer polls (worker.PowService; replaces concurrent blocking run() calls of
 *      the worker and API threads, src/class_singleWorker.py:236,1276, src/api.py:1304,1350) ---- */
typedef struct bmpow_service bmpow_service;

/* Start the service thread.  step_budget: trials per step (0 = library default).  flags:
 * BMPOW_SERVICE_VERIFY re-hashes every found nonce on the host (OpenSSL SHA-512) inside
 * bmpow_service_poll, on the polling thread, and reports a mismatch or a trial above the target as
 * BMPOW_DONE_BADHASH -- the check _doGPUPoW makes with hashlib (src/proofofwork.py:176-190).
 * NULL on error. */
#define BMPOW_SERVICE_VERIFY 1u
BMPOW_API bmpow_service *bmpow_service_create(uint64_t step_budget, uint32_t flags);

/* Queue n objects (ihs: n x 64 bytes, targets: n; every search starts at nonce 1); they join the
 * session at the next step.  tickets_out[i] (may be NULL) = object i's ticket (ascending over the
 * service's life).  Returns 0 or < 0. */
BMPOW_API int bmpow_service_submit(bmpow_service *s, size_t n, const uint8_t *ihs, const uint64_t *targets,
                                   uint64_t *tickets_out);
/* bmpow_service_submit for initialHashes of any length (object i = ihs[ih_off[i] .. ih_off[i+1])). */
BMPOW_API int bmpow_service_submit_var(bmpow_service *s, size_t n, const uint8_t *ihs, const uint64_t *ih_off,
                                       const uint64_t *targets, uint64_t *tickets_out);

/* Pop up to cap finished objects (ticket, nonce, trial, BMPOW_DONE_FOUND or BMPOW_DONE_EXHAUSTED),
 * waiting up to timeout_ms (< 0: forever) for the first.  Returns the count (0 on timeout), or the
 * error a step hit (< 0, bmpow_last_error() in this thread) once everything before it was popped;
 * the service then steps nothing until bmpow_service_cancel. */
BMPOW_API int bmpow_service_poll(bmpow_service *s, size_t cap, int timeout_ms, uint64_t *tickets, uint64_t *nonce_out,
                                 uint64_t *trial_out, uint8_t *done_out);

/* Drop every queued, live and unpolled object (and a pending error); the service keeps running. */
BMPOW_API int bmpow_service_cancel(bmpow_service *s);

/* Objects submitted and not yet popped by bmpow_service_poll. */
BMPOW_API int bmpow_service_outstanding(bmpow_service *s);

/* Stop stepping (after the current step) and wake every bmpow_service_poll: they return what is
 * already finished, then 0 at once.  Submits fail with BMPOW_E_STATE.  The handle stays valid. */
BMPOW_API void bmpow_service_stop(bmpow_service *s);

/* Stop (as above) and free the session; no other call on s may be in progress. */
BMPOW_API void bmpow_service_destroy(bmpow_service *s);

/* ---- receive-side verification (replaces protocol.isProofOfWorkSufficient,
 *      src/protocol.py:258-286, called once per received object from
 *      src/network/bmobject.py:71-76) ----
 *
 * Objects are finished objects as they travel: nonce (8 bytes, big-endian) || payload, passed
 * as one concatenated buffer `objs` with byte offsets[0..n] (object i = objs[offsets[i] ..
 * offsets[i+1])).  POW(i) = BE64(SHA512(SHA512(obj[0:8] || SHA512(obj[8:])))[0:8])
 * (protocol.py:280-282), computed one object per GPU lane, objects spread over the active
 * devices. */

/* POW values of n objects (each >= 8 bytes).  Returns 0 or < 0. */
BMPOW_API int bmpow_pow_values(size_t n, const uint8_t *objs, const uint64_t *offsets, uint64_t *pow_out);

/* isProofOfWorkSufficient for n objects: ntpb[i]/extra[i] (NULL = 0; raised to the network
 * defaults 1000/1000 as protocol.py:272-275 does), recv_time[i] (NULL or 0 = now, :277);
 * TTL = expiresTime (obj[8:16]) - recv_time, at least 300 s; ok_out[i] = 1 when
 * POW <= 2^64 / (ntpb * (len + extra + TTL * (len + extra) / 2^16)) in the reference's IEEE
 * double arithmetic, 0 when not, 2 when the object is shorter than 16 bytes (the reference
 * raises struct.error there).  Returns 0 or < 0. */
BMPOW_API int bmpow_verify_batch(size_t n, const uint8_t *objs, const uint64_t *offsets, const uint64_t *ntpb,
                                 const uint64_t *extra, const int64_t *recv_time, uint8_t *ok_out);

/* The verdict arithmetic alone, on the host (no device): 1 when `pow` is sufficient for an
 * object of `len` bytes (nonce included) with expiresTime `expires`, received at `recv_time`
 * (0 = now), else 0 -- the comparison bmpow_verify_batch applies (protocol.py:272-286). */
BMPOW_API int bmpow_pow_sufficient(uint64_t pow, uint64_t len, uint64_t ntpb, uint64_t extra, int64_t recv_time,
                                   uint64_t expires);

/* The same check with the objects where they lie: objs[i] points at object i (lens[i] bytes),
 * so a caller holding separate buffers (one per received object) needs no concatenation. */
BMPOW_API int bmpow_verify_batch_ptrs(size_t n, const uint8_t *const *objs, const uint64_t *lens,
                                      const uint64_t *ntpb, const uint64_t *extra, const int64_t *recv_time,
                                      uint8_t *ok_out);

/* Device-resident verification session: pad, sort and upload the objects once, then hash
 * them repeatedly (bench.py times bmpow_vbatch_run with the payloads resident in HBM). */
typedef struct bmpow_vbatch bmpow_vbatch;
BMPOW_API bmpow_vbatch *bmpow_vbatch_create(size_t n, const uint8_t *objs, const uint64_t *offsets);
/* One pass over every object; pow_out (n, input order) may be NULL.  Returns 0 or < 0. */
BMPOW_API int bmpow_vbatch_run(bmpow_vbatch *vb, uint64_t *pow_out);
BMPOW_API void bmpow_vbatch_destroy(bmpow_vbatch *vb);

/* ---- RIPE-prefix address search (replaces the key-generation loops of
 *      src/class_addressGenerator.py:130-148 (random) and :238-271 (deterministic)) ----
 *
 * Try k derives two secp256k1 private keys, multiplies them by G (src/highlevelcrypto.py:111-140,
 * pointMult) and computes ripe = RIPEMD160(SHA512(pubSigning || pubEncryption)) over the
 * 65-byte uncompressed keys; the search returns the first k whose ripe starts with null_bytes
 * zero bytes (numberOfNullBytesDemandedOnFrontOfRipeHash). */
typedef struct bmpow_address {
    uint64_t k;                   /* the try index found */
    uint8_t ripe[20];
    uint8_t priv_signing[32];
    uint8_t priv_encryption[32];
    uint8_t pub_signing[65];      /* 04 || X || Y */
    uint8_t pub_encryption[65];
} bmpow_address;

/* pointMult for n private keys (n x 32 bytes, big-endian) -> n x 65-byte keys; a zero key gives
 * 65 zero bytes.  Returns 0 or < 0. */
BMPOW_API int bmpow_pubkeys(size_t n, const uint8_t *privkeys, uint8_t *pubkeys_out);

/* Field-arithmetic probe for the tests (no reference counterpart): out[i] = op(a[i], b[i]) mod
 * p = 2^256 - 2^32 - 977 on the device, operands as 8 little-endian 32-bit limbs each (any value
 * below 2^256, reduced or not).  op: 0 a+b, 1 a-b, 2 a*b, 3 a^2, 4 canonical form of a, 5 a^-1
 * (0 for a = 0 mod p), 6 (a = 0 mod p) in limb 0.  Results of 0..3 are weakly reduced (< 2^256,
 * congruent), of 4..5 canonical (< p).  Returns 0 or < 0. */
BMPOW_API int bmpow_fe_probe(int op, size_t n, const uint32_t *a, const uint32_t *b, uint32_t *out);

/* Deterministic addresses (createDeterministicAddresses / getDeterministicAddress / chans):
 * privSigning = SHA512(passphrase || varint(2k))[:32], privEncryption = SHA512(passphrase ||
 * varint(2k+1))[:32], k in [start, start + max_tries).  Returns BMPOW_FOUND (out filled) with
 * the first k, BMPOW_NOT_FOUND, or < 0.  The reference continues the next address at k + 1. */
BMPOW_API int bmpow_address_search(const uint8_t *passphrase, size_t len, uint64_t start, uint64_t max_tries,
                                   int null_bytes, bmpow_address *out);

/* Random addresses (createRandomAddress): the given signing key is kept; the encryption key of
 * try k is SHA512(seed || varint(k))[:32] (the caller draws `seed` from a CSPRNG, as the
 * reference draws each key from OpenSSL.rand).  Same return convention. */
BMPOW_API int bmpow_address_search_random(const uint8_t priv_signing[32], const uint8_t *seed, size_t seed_len,
                                          uint64_t start, uint64_t max_tries, int null_bytes, bmpow_address *out);

/* Fixed-base comb used by the address search: 16-bit windows (64 MB table, 16 additions per k*G)
 * or 24-bit windows (10.7 GB table per device, 11 additions, ~25 % more tries/s, ~0.4 s to build
 * once).  wbits = 0 (default): automatic -- the 24-bit comb when it is already built or a search
 * is expected to need >= 2^32 tries; 16 or 24 force one.  Returns the previous setting or < 0. */
BMPOW_API int bmpow_addr_set_comb(int wbits);
/* Window width (16 or 24) the last address search ran with; 0 before the first. */
BMPOW_API int bmpow_addr_last_comb(void);

/* ---- instrumentation (bench.py's roofline leg) ---- */
typedef struct bmpow_stats {
    uint64_t launches;        /* search-kernel launches (summed over shards) */
    uint64_t trials;          /* trials actually hashed by search kernels (device-counted) */
    double kernel_ms;         /* sum over launches of search-kernel time, HIP events on the
                                 launching stream */
    double max_shard_kernel_ms; /* max over shards of their summed kernel time */
    uint64_t steps;           /* host scheduler steps */
    /* receive-side verification (bmpow_pow_values / bmpow_verify_batch / bmpow_vbatch_run) */
    uint64_t verify_launches; /* bv_pow_kernel launches (summed over shards) */
    uint64_t verify_objects;  /* objects hashed */
    uint64_t verify_blocks;   /* 128-B SHA-512 blocks of payload hashed (padding included) */
    double verify_kernel_ms;  /* max over shards per run, summed over runs (HIP events) */
    /* RIPE-prefix address search (bmpow_address_search*) */
    uint64_t addr_launches;   /* search steps */
    uint64_t addr_tries;      /* tries launched (each: 2 SHA-512, 2 k*G, SHA-512, RIPEMD-160) */
    double addr_kernel_ms;    /* max over shards per step, summed (HIP events) */
    /* min-trial probe (bmpow_min_trial*) */
    uint64_t probe_trials;    /* nonces hashed by the probe */
    double probe_kernel_ms;   /* sum over launches of probe-kernel time (HIP events) */
    /* host-side wall time of bmpow_verify_batch* (steady clock), summed over calls */
    double verify_host_build_ms;    /* sort, layout, padding into pinned staging, PCIe upload issued */
    double verify_host_run_ms;      /* kernel + results back (waits for the uploads) */
    double verify_host_verdict_ms;  /* IEEE-double verdicts */
    /* run()'s single-object kernel: nonces whose trial stopped after the first of its two SHA-512
       compressions, the call's answer having been published below them meanwhile (not in trials) */
    uint64_t cut_trials;
    /* run()'s single-object path: wall time the calling thread spent waiting for its launches,
       spinning on the result word (a short call's last window) and sleeping between polls */
    double one_wait_spin_ms;
    double one_wait_sleep_ms;
    /* the engine's (batch) trials hashed past the objects' answers, by where, priced once an object's
       answer is final.  Estimates from each item's block queue: every workgroup ends on one unit it
       takes and does not hash, so of the units handed out the first (taken - workgroups) count as
       hashed (within one block per workgroup of the device's count) */
    uint64_t past_window;     /* unsplit windows holding the answer: nonces above it */
    uint64_t past_later;      /* unsplit windows starting above the answer (the lookahead queued behind) */
    uint64_t past_split;      /* pieces of windows split over device groups: nonces above the answer */
    uint64_t engine_hashed_est; /* every priced item's estimated hashed nonces (compare with trials) */
    /* streams the library keeps for the life of the process (current counts, not reset): CU-masked
       streams of the forced-split rehearsal (bmpow_set_run_split) and run()'s priority streams */
    uint64_t masked_streams;
    uint64_t run_streams;
} bmpow_stats;

BMPOW_API int bmpow_get_stats(bmpow_stats *out);
BMPOW_API void bmpow_reset_stats(void);

/* Per-shard search work since the last bmpow_reset_stats: trials hashed and summed search-kernel
 * time (HIP events) of each shard's launches, into trials[0..cap) / kernel_ms[0..cap) (either may be
 * NULL).  Returns the shard count. */
BMPOW_API int bmpow_get_shard_stats(uint64_t *trials, double *kernel_ms, int cap);

/* The per-shard stepper threads (one per shard, bmsched::Engine): CPU seconds each has used so far
 * (CLOCK_THREAD_CPUTIME_ID) and its scheduling policy (sched_getscheduler: SCHED_IDLE by default, as
 * the reference's PoW threads, src/bitmsghash/bitmsghash.cpp:149; BMPOW_THREAD_POLICY=batch|normal
 * overrides).  Either output may be NULL.  Returns the shard count (0 before bmpow_init). */
BMPOW_API int bmpow_get_thread_info(double *cpu_s, int *policy, int cap);

/* A/B and test knob: shard `shard`'s stepper sleeps `ms` before each launch (a slow device); 0 turns
 * it off.  Returns 0 or < 0. */
BMPOW_API int bmpow_set_shard_throttle(int shard, double ms);

/* run()'s pieces (bmpow_search / bmpow_search_len): 0 (default) = one piece per physical device, the
 * first shard of each; 1 = one piece per shard even where shards share a device -- a test and
 * rehearsal knob (pieces on one device compete for its SIMDs).  < 0 only queries.  Returns the
 * previous setting. */
BMPOW_API int bmpow_set_run_split(int per_shard);
/* The batch engine's device groups: 0 (default) = the shards of one physical device form one group,
 * which never holds an object on two of its shards at once and never splits a window among them (a
 * split window has one piece per device); 1 = every shard its own group, as if each were a separate
 * GPU -- the test and rehearsal knob for the multi-device split on one GPU (its pieces then compete for
 * the device's SIMDs).  Drains the engine.  < 0 only queries.  Returns the previous setting. */
BMPOW_API int bmpow_set_engine_split(int per_shard);
/* The shards carrying run()'s pieces into shards[0..cap) (may be NULL); returns their count or < 0. */
BMPOW_API int bmpow_get_run_pieces(int *shards, int cap);

/* Per-shard trial budget of one step (one kernel launch), default 2^29 (~80 ms on one MI355X: the
 * interrupt granularity of a batch); set 0 to restore the default.  At least one chunk (8,192). */
BMPOW_API uint64_t bmpow_get_step_trials(void);
BMPOW_API void bmpow_set_step_trials(uint64_t trials_per_shard);

/* ---- compatibility shim ---- */

/* Same signature as the reference's export (src/bitmsghash/bitmsghash.cpp:127), so an
 * unmodified _doCPoW (src/proofofwork.py:157-170) can load this library.  Blocks until
 * found; returns the EXACT first nonce >= 1 with trial <= target (the _doSafePoW answer,
 * not the racy strict-< answer of the reference C code).  Returns 0 on error/abort. */
BMPOW_API unsigned long long BitmessagePOW(unsigned char *starthash, unsigned long long target);

#ifdef __cplusplus
}
#endif

#endif /* BMPOW_H */
