// bmpow_layout.h -- the data layout shared by the gfx950 kernels and the host scheduler: plain
// structs and sizes only, no HIP, so the host-only scheduler unit (bmpow_sched.cpp) and its
// sanitizer tests (tests/native/) build without a device toolchain.
#pragma once
#include <stdint.h>

// One workgroup = BM_BLOCK lanes x iters nonces = one CHUNK of a work item.  Full steps use
// BM_ITERS iterations per workgroup; small steps (a single easy object) use BM_ITERS_SMALL so a
// "round" of resident workgroups is short and the answer is reached sooner.  BM_CHUNK (the full
// chunk) is a multiple of every chunk size, so windows rounded to it fit either.
#ifndef BM_ITERS
#define BM_ITERS 32
#endif
#define BM_ITERS_SMALL 4
#ifndef BM_BLOCK
#define BM_BLOCK 256  // lanes per search workgroup (A/B builds may override it)
#endif
#define BM_CHUNK ((uint64_t)BM_BLOCK * BM_ITERS)

// Per-object record, device resident for the life of a batch (128 B, one per object).
//   ihlen == 64 (every caller in the reference: sha512(payload).digest()): w[] holds the
//     initialHash, searched by bm_search_kernel;
//   any other length: w[] is unused and the object's message words live in the batch's var pool
//     from word vword on (16 words of block 0, then 80 K+W words per further block, nblk blocks in
//     the first hash; bmsched::pack_var), searched by bm_search_var_kernel.
constexpr uint32_t BM_IH_MAIN = 64;
struct bm_obj {
  uint64_t w[8];     // initialHash as 8 big-endian words = W1..W8 of SHA-512 block 1 (ihlen == 64)
  uint64_t target;   // accept trial <= target
  uint32_t ihlen;    // initialHash length in bytes
  uint32_t nblk;     // var form: blocks of the first hash's message
  uint64_t vword;    // var form: first word of this object in the var pool
  uint64_t pad[5];
};
static_assert(sizeof(bm_obj) == 128, "bm_obj is 128 B");

// Words an initialHash of len bytes (!= 64) takes in the var pool.
inline uint64_t bm_var_blocks(uint64_t len) { return (8 + len + 17 + 127) / 128; }
inline uint64_t bm_var_words(uint64_t len) { return 16 + 80 * (bm_var_blocks(len) - 1); }
#ifndef BMPOW_MAX_IH_LEN  // (also in include/bmpow.h)
#define BMPOW_MAX_IH_LEN (1u << 20)  // longest initialHash the library accepts (1 MiB)
#endif

// Work item = one object's nonce window [start, start + count) inside one launch (48 B), cut into
// blocks of BM_BLOCK nonces (one per lane).  The item's workgroups take its blocks IN ORDER from a
// per-item counter (the block queue, bmpow_kernels.h: the k-th block taken is bm_block_of(item, k)),
// so the hashed set is a prefix of the item's blocks plus those in flight, and a workgroup stops at
// its next block above the running minimum.  The order is that of the item's COLUMNS: the window's
// blocks are dealt round-robin to gn columns (column c: blocks c, c + gn, c + 2 gn, ...), this item
// owns columns [g0, g0 + nwg) and runs nwg workgroups, and its k-th block is row k / nwg of column
// g0 + k % nwg.
//   * a window on one shard: one item, g0 = 0, gn = nwg (capped at the shard's resident workgroups),
//     so the k-th block is simply block k;
//   * a window split over the S shards (fewer pending objects than shards): one item per shard, all
//     covering the whole window, interleaved: shard s runs columns [g0_s, g0_s + nwg_s) of gn = sum
//     nwg_s -- so every device sweeps the same rows -- and the shards share the window's running
//     minimum through the cross-shard bound (xslot, below).
// The min-trial probe (no early exit) runs the same items as static columns: workgroup c of the item
// hashes column g0 + c top to bottom.
struct bm_item {
  uint64_t start;       // first nonce of the window
  uint64_t count;       // nonces in the window (> 0; start + count - 1 <= 2^64 - 1)
  uint32_t obj;         // object index (into bm_obj[] and best[])
  uint32_t chunk_base;  // first workgroup of this item in its launch
  uint32_t g0;          // first column of this item
  uint32_t gn;          // columns of the window (over every item of the window)
  uint32_t nwg;         // workgroups (columns) of this item
  uint32_t xslot;       // cross-shard bound slot of a split window, or BM_NO_XSLOT
  uint64_t pad;
};
static_assert(sizeof(bm_item) == 48, "bm_item is 48 B");
#define BM_NO_XSLOT 0xffffffffu
// Cross-shard bound table: host-pinned, coherent, mapped into every device; row s (BM_XSLOTS words)
// belongs to shard s, which stores its hits there (any hit of the window is a valid bound); every
// shard's kernel reads all rows' slot of the window.  Split windows number fewer than the shards.
#define BM_XSLOTS 64
#define BM_MAX_SHARDS 64

// ---- the single-object path of run() (bmpow_search_len, any number of devices; bm_search1_kernel) ----
// One launch per window of the object (per piece: one interleaved piece of each window per device), the
// object's words in the kernel arguments, the next window queued behind; the launch's last workgroup
// writes its result into host-mapped memory, so a call costs one kernel launch per window and piece and
// no copy or resolve kernel.
// Per call (a ring of BM_ONE_CALLS, slot c % BM_ONE_CALLS; every launch of call c puts slot
// (c + 2) % BM_ONE_CALLS back to "no hit", which no launch in flight uses): the running minimum and
// a log of the hits with their trial values (so the result needs no re-hash).
#define BM_ONE_CALLS 4
#define BM_ONE_LOG 32
struct bm_one_call {
  unsigned long long best;  // running minimum hit nonce (valid where found)
  uint32_t found, nhits;
  unsigned long long hit_nonce[BM_ONE_LOG], hit_trial[BM_ONE_LOG];
};
// Per launch (a ring of BM_ONE_RING per piece; reset by the launch's last wave once it has used them).
#define BM_ONE_RING 256
// acc packs, per launch, the sums of every workgroup's one atomic as it finishes: trials hashed
// (bits 31..63; a piece hashes at most ~2^32 nonces of a window, bmpow_host.hip search_one), lanes
// whose block skipped its second compression (bits 12..30: at most one block per wave, so at most
// 2,047 x 256 = 524,032 < 2^19 with BM_ONE_MAX_WG column workgroups), workgroups done (bits 0..11,
// the relay included).
#define BM_ONE_MAX_WINDOW (1ULL << 32)
#define BM_ONE_MAX_WG 2047u
struct bm_one_ctr {
  unsigned long long queue;  // the block queue
  unsigned long long acc;    // trials << 31 | cut << 12 | workgroups done
  unsigned long long t0;     // s_memrealtime at workgroup 0's start (0 = unset)
  unsigned long long pad;
};
// The launch's result, host-mapped; seq is written last (release), the host polls it.
struct bm_one_out {
  uint64_t nonce, trial, trials, t0, t1;  // t0, t1: s_memrealtime (100 MHz) at workgroup 0's start, last exit
  uint32_t found;
  uint32_t cut;  // lanes that hashed only the first compression of their trial (bm_one_ctr.acc)
  uint64_t seq;
};
// The kernel's arguments (by value).  A run() on several physical devices cuts each window into P
// interleaved pieces, one per device (piece p = columns [g0, g0 + nwg) of the window's gn, as a split
// bm_item); the pieces share the call's running minimum through the cross-device bound: a hit is
// stored into slot xslot of every row of the host-pinned table xb (bm_publish), and each launch's
// workgroup 0 relays its own row into the device's running minimum (the grid is then nwg + 1).
struct bm_one_args {
  uint64_t w[8];  // the initialHash as big-endian words (W1..W8 of block 1)
  uint64_t target, start, count;
  bm_one_call* call;   // this call's state
  bm_one_call* reset;  // the state of the call two ahead: put back to "no hit"
  bm_one_ctr* ctr;
  bm_one_out* out;     // the device's address of the host-mapped result
  uint64_t seq;
  uint32_t nwg;        // column workgroups of this piece
  uint32_t g0, gn;     // split run: this piece's first column and the window's columns (else 0, nwg)
  uint32_t xslot, xrow, xrows;  // split run: the call's slot, this piece's row, the rows (pieces)
  // split run: the cross-device bound table as this device maps it, else null (last, so the one-device
  // kernel reads its fields at the offsets it always did: its code is unchanged)
  unsigned long long* xb;
};

struct bm_result {
  uint64_t nonce;  // the object's minimum hit so far (meaningful only when found)
  uint64_t trial;
  uint32_t found;  // 1: the object has a hit (nonce 2^64-1 included); 0: none yet
  uint32_t pad;
};

// One workgroup's minimum of the min-trial probe: the lowest trial value over its chunk and the
// first nonce reaching it.
struct bm_minpart {
  uint64_t trial;
  uint64_t nonce;
};

// Receive-side verification (bv_*): one finished object (nonce || payload) per lane.  The
// payload is stored SHA-512-padded in a pool of 128-B blocks; objects are sorted by block
// count (descending) on the host so the lanes of a wave loop the same number of times.
#define BV_BLOCK 64
#define BV_BINNED_WG 1024  // bv_pow_binned_kernel: 16 waves per CU, 4 per SIMD
struct bv_obj {
  uint32_t blk;    // first 128-B block of the padded payload in the pool
  uint32_t nblk;   // padded blocks (>= 1)
  uint64_t nonce;  // BE64(object[0:8])
};

