// bmpow_sched.cpp -- host-only scheduler logic of libbmpow_hip.so (see bmpow_sched.h).  No HIP:
// compiled into the library by hipcc and, for tests/native/, by g++ under the sanitizers.
#include "bmpow_sched.h"

#include <openssl/sha.h>

#include <emmintrin.h>
#include <unistd.h>

#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>
#include <sys/syscall.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <thread>

namespace bmsched {

uint64_t load_be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int j = 0; j < 8; ++j) v = (v << 8) | p[j];
  return v;
}

uint64_t host_trial(const uint8_t ih[64], uint64_t nonce) {
  uint8_t msg[72], h1[64], h2[64];
  for (int i = 0; i < 8; ++i) msg[i] = (uint8_t)(nonce >> (56 - 8 * i));
  memcpy(msg + 8, ih, 64);
  SHA512(msg, sizeof msg, h1);
  SHA512(h1, sizeof h1, h2);
  return load_be64(h2);
}

uint64_t host_trial_len(const uint8_t* ih, size_t len, uint64_t nonce) {
  if (len == 64) return host_trial(ih, nonce);
  std::vector<uint8_t> msg(8 + len);
  for (int i = 0; i < 8; ++i) msg[i] = (uint8_t)(nonce >> (56 - 8 * i));
  if (len) memcpy(msg.data() + 8, ih, len);
  uint8_t h1[64], h2[64];
  SHA512(msg.data(), msg.size(), h1);
  SHA512(h1, sizeof h1, h2);
  return load_be64(h2);
}

void pack_obj(const uint8_t* ih, uint64_t target, bm_obj* o) {
  std::memset(o, 0, sizeof(*o));
  for (int i = 0; i < 8; ++i) o->w[i] = load_be64(ih + 8 * i);
  o->target = target;
  o->ihlen = BM_IH_MAIN;
  o->nblk = 1;
}

namespace {

// FIPS 180-4 4.2.3 (the K+W words of pack_var's later blocks are summed on the host)
constexpr uint64_t kK512[80] = {
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

inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

}  // namespace

void pack_var(const uint8_t* ih, size_t len, uint64_t target, bm_obj* o, std::vector<uint64_t>& pool) {
  if (len == BM_IH_MAIN) {
    pack_obj(ih, target, o);
    return;
  }
  std::memset(o, 0, sizeof(*o));
  o->target = target;
  o->ihlen = (uint32_t)len;
  // BE64(nonce) || ih || 0x80 || zeros || BE128(bit length), the nonce bytes left zero (the kernel's W0)
  const uint64_t m = 8 + (uint64_t)len, nblk = bm_var_blocks(len);
  std::vector<uint8_t> buf(nblk * 128, 0);
  if (len) memcpy(buf.data() + 8, ih, len);
  buf[m] = 0x80;
  for (int i = 0; i < 8; ++i) buf[nblk * 128 - 1 - i] = (uint8_t)((m * 8) >> (8 * i));
  buf[nblk * 128 - 9] = (uint8_t)(m >> 61);
  o->nblk = (uint32_t)nblk;
  o->vword = pool.size();
  for (int i = 0; i < 16; ++i) pool.push_back(load_be64(buf.data() + 8 * i));
  uint64_t w[80];
  for (uint64_t j = 1; j < nblk; ++j) {
    for (int t = 0; t < 16; ++t) w[t] = load_be64(buf.data() + 128 * j + 8 * t);
    for (int t = 16; t < 80; ++t) {
      const uint64_t s0 = ror(w[t - 15], 1) ^ ror(w[t - 15], 8) ^ (w[t - 15] >> 7);
      const uint64_t s1 = ror(w[t - 2], 19) ^ ror(w[t - 2], 61) ^ (w[t - 2] >> 6);
      w[t] = s1 + w[t - 7] + s0 + w[t - 16];
    }
    for (int t = 0; t < 80; ++t) pool.push_back(kK512[t] + w[t]);
  }
}

// ---------------------------------------------------------------------------------------
// sessions
// ---------------------------------------------------------------------------------------
namespace {

// The frontier of slot k starts over at nonce st: a new generation (launches planned for the slot
// before are stale), no hit, no window.
void restart_slot(BatchState& b, size_t k, uint64_t st) {
  b.gen[k]++;
  b.next[k] = st;
  b.lim[k] = kU64Max;
  b.nonce[k] = b.trial[k] = 0;
  b.hit[k] = 0;
  b.top[k] = 0;
  b.holder[k] = kNoHolder;
  b.nfly[k] = 0;
  b.fly1[k] = b.fly2[k] = 0;
  b.xs[k] = 0;
  b.open[k].clear();
  b.wseq[k] = 0;
  b.wrec[k].clear();
}

void grow_slots(BatchState& b, size_t n) {
  b.objs.resize(n);
  b.next.resize(n);
  b.nonce.resize(n);
  b.trial.resize(n);
  b.done.resize(n, BMPOW_FREE);
  if (b.gen.size() < n) b.gen.resize(n, 0);  // never shrinks: a slot's generations only count up
  b.lim.resize(n, kU64Max);
  b.hit.resize(n, 0);
  b.top.resize(n, 0);
  b.holder.resize(n, kNoHolder);
  b.nfly.resize(n, 0);
  b.fly1.resize(n, 0);
  b.fly2.resize(n, 0);
  b.xs.resize(n, 0);
  b.open.resize(n);
  b.wseq.resize(n, 0);
  b.wrec.resize(n);
}

}  // namespace

void init(BatchState& b, size_t n, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
          const uint64_t* ih_off) {
  const uint64_t epoch = b.vpool_epoch + 1;
  // generations carry over: launches still in flight for the previous contents stay stale
  std::vector<uint32_t> gen;
  gen.swap(b.gen);
  b = BatchState();
  b.vpool_epoch = epoch;
  b.n = n;
  b.gen.swap(gen);
  grow_slots(b, n);
  for (size_t i = 0; i < n; ++i) {
    pack_var(ih_ptr(ihs, ih_off, i), ih_len(ih_off, i), targets[i], &b.objs[i], b.vpool);
    if (b.objs[i].ihlen != BM_IH_MAIN) {
      b.nvar_slots++;
      b.vlive += bm_var_words(b.objs[i].ihlen);
    }
    b.done[i] = BMPOW_PENDING;
    restart_slot(b, i, start ? start[i] : 1);
  }
  b.pending = n;
  b.cap = n;
}

namespace {

void mark_finished(BatchState& b, uint32_t slot) {
  if (b.finished_head > 4096 && b.finished_head * 2 > b.finished.size()) {  // drop the consumed prefix
    b.finished.erase(b.finished.begin(), b.finished.begin() + (ptrdiff_t)b.finished_head);
    b.finished_head = 0;
  }
  b.finished.push_back(slot);
}

}  // namespace

namespace {

// Repack vpool to the words of the slots that still hold a var-form object (see add()).
void compact_vpool(BatchState& b) {
  std::vector<uint64_t> pool;
  pool.reserve(b.vlive);
  for (size_t k = 0; k < b.n; ++k) {
    bm_obj& o = b.objs[k];
    if (b.done[k] == BMPOW_FREE || o.ihlen == BM_IH_MAIN) continue;
    const uint64_t w = bm_var_words(o.ihlen);
    const uint64_t at = pool.size();
    pool.insert(pool.end(), b.vpool.begin() + (ptrdiff_t)o.vword, b.vpool.begin() + (ptrdiff_t)(o.vword + w));
    if (o.vword != at) b.vmoved.push_back((uint32_t)k);
    o.vword = at;
  }
  b.vpool.swap(pool);
  b.vpool_epoch++;
}

}  // namespace

bool add(BatchState& b, size_t m, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
         std::vector<uint32_t>& slots, const uint64_t* ih_off) {
  if (b.nvar_slots == 0 && !b.vpool.empty()) {  // nothing refers to the old words any more
    b.vpool.clear();
    b.vpool_epoch++;
  } else if (b.vpool.size() > 2 * b.vlive && b.vpool.size() - b.vlive > ((size_t)1 << 16)) {
    compact_vpool(b);
  }
  slots.resize(m);
  const size_t n0 = b.n;
  for (size_t i = 0; i < m; ++i) {
    if (!b.free_slots.empty()) {
      slots[i] = b.free_slots.back();
      b.free_slots.pop_back();
    } else {
      slots[i] = (uint32_t)b.n++;
    }
  }
  if (b.n > n0) grow_slots(b, b.n);
  for (size_t i = 0; i < m; ++i) {
    const uint32_t k = slots[i];
    pack_var(ih_ptr(ihs, ih_off, i), ih_len(ih_off, i), targets[i], &b.objs[k], b.vpool);
    if (b.objs[k].ihlen != BM_IH_MAIN) {
      b.nvar_slots++;
      b.vlive += bm_var_words(b.objs[k].ihlen);
    }
    restart_slot(b, k, start ? start[i] : 1);
    b.done[k] = BMPOW_PENDING;
    b.pending++;
    if (k < b.first_pending) b.first_pending = k;
  }
  return b.n > b.cap;
}

size_t take_done(BatchState& b, size_t cap, uint32_t* slot_out, uint64_t* nonce_out, uint64_t* trial_out,
                 uint8_t* done_out) {
  size_t k = 0;
  while (k < cap && b.finished_head < b.finished.size()) {
    const uint32_t s = b.finished[b.finished_head++];
    slot_out[k] = s;
    if (nonce_out) nonce_out[k] = b.nonce[s];
    if (trial_out) trial_out[k] = b.trial[s];
    if (done_out) done_out[k] = b.done[s];
    b.done[s] = BMPOW_FREE;
    if (b.objs[s].ihlen != BM_IH_MAIN) {
      b.nvar_slots--;
      b.vlive -= bm_var_words(b.objs[s].ihlen);
    }
    b.free_slots.push_back(s);
    ++k;
  }
  if (b.finished_head == b.finished.size()) {
    b.finished.clear();
    b.finished_head = 0;
  }
  return k;
}

void reset(BatchState& b, const uint64_t* start) {
  b.pending = 0;
  for (size_t i = 0; i < b.n; ++i) {
    restart_slot(b, i, start ? start[i] : 1);
    if (b.done[i] == BMPOW_FREE) continue;  // released slots stay free
    b.done[i] = BMPOW_PENDING;
    b.pending++;
  }
  b.first_pending = 0;
  b.finished.clear();
  b.finished_head = 0;
  b.broken = false;
}

namespace {
bool settle(BatchState& b, size_t o);
}

void set_pending(BatchState& b, size_t first, size_t count, bool pending) {
  for (size_t i = first; i < first + count; ++i) {
    if (pending && b.done[i] == BMPOW_PARKED) {
      b.done[i] = BMPOW_PENDING;
      b.pending++;
      settle(b, i);  // its windows may have completed while it was parked
    } else if (!pending && b.done[i] == BMPOW_PENDING) {
      b.done[i] = BMPOW_PARKED;
      b.pending--;
    }
  }
  if (pending && first < b.first_pending) b.first_pending = first;
}

// ---------------------------------------------------------------------------------------
// work items
// ---------------------------------------------------------------------------------------
uint32_t g_blocks_per_worker = 0;

namespace {

uint64_t blocks_per_worker(uint64_t chunk) {
  return g_blocks_per_worker ? g_blocks_per_worker
                             : std::max<uint64_t>(1, std::min<uint64_t>(kBlocksPerWorker, chunk / BM_BLOCK));
}

}  // namespace

void slice(const std::vector<Win>& wins, uint64_t C, uint64_t chunk, size_t S, StepPlan& p, uint32_t resident) {
  p.items.assign(S, std::vector<bm_item>());
  p.nchunks.assign(S, 0);
  p.nx = 0;
  p.C = C;
  std::vector<uint64_t> cut(S + 1);
  for (size_t s = 0; s <= S; ++s) cut[s] = C * s / S;
  size_t s = 0;
  for (const Win& w : wins) {
    uint64_t c = w.chunk0;
    const uint64_t cend = w.chunk0 + w.chunks;
    while (c < cend) {
      while (s < S && cut[s + 1] <= c) ++s;
      const uint64_t seg_end = std::min(cend, cut[s + 1]);
      bm_item it;
      std::memset(&it, 0, sizeof it);
      const uint64_t off = (c - w.chunk0) * chunk;
      it.start = w.start + off;
      it.count = std::min<uint64_t>(w.count - off, (seg_end - c) * chunk);
      it.obj = w.obj;
      it.chunk_base = p.nchunks[s];
      const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
      const uint64_t bpw = blocks_per_worker(chunk);
      uint64_t G = std::max<uint64_t>(1, (nblk + bpw - 1) / bpw);
      if (resident) G = std::min<uint64_t>(G, resident);
      it.g0 = 0;
      it.gn = (uint32_t)G;
      it.nwg = (uint32_t)G;
      it.xslot = BM_NO_XSLOT;
      p.items[s].push_back(it);
      p.nchunks[s] += (uint32_t)G;
      c = seg_end;
    }
  }
}

uint64_t expect_cap(uint64_t target, size_t S, uint64_t chunk) {
  // E = 2^64 / (target + 1): the expected trials to the first hit (each trial is <= target with
  // probability (target + 1) / 2^64)
  const double e = 18446744073709551616.0 / ((double)target + 1.0);
  const double cap = kExpectWindows * e;
  const uint64_t floor_ = (uint64_t)S * chunk;  // every piece gets at least one chunk of the object
  return cap < (double)floor_ ? floor_ : (cap >= 1.8e19 ? kU64Max : (uint64_t)cap);
}

void ShardRates::sample(size_t s, uint64_t trials, double ms) {
  if (s >= ema.size() || trials < min_trials || !(ms > 0)) return;
  const double r = (double)trials / ms;
  ema[s] = ema[s] > 0 ? (1 - kRateAlpha) * ema[s] + kRateAlpha * r : r;
}

bool ShardRates::weights(std::vector<double>& w) const {
  w.assign(ema.size(), 1.0);
  double mean = 0;
  for (double r : ema) {
    if (!(r > 0)) return false;
    mean += r;
  }
  if (ema.empty()) return false;
  mean /= (double)ema.size();
  for (size_t s = 0; s < ema.size(); ++s) w[s] = std::min(2.0, std::max(0.5, ema[s] / mean));
  return true;
}

void split_kinds(const std::vector<bm_obj>& objs, bool any_var, StepPlan& p) {
  const size_t S = p.items.size();
  p.nmain.assign(S, 0);
  p.chmain.assign(S, 0);
  std::vector<bm_item> var;
  for (size_t s = 0; s < S; ++s) {
    std::vector<bm_item>& v = p.items[s];
    if (!any_var) {
      p.nmain[s] = (uint32_t)v.size();
      p.chmain[s] = p.nchunks[s];
      continue;
    }
    var.clear();
    size_t k = 0;
    uint64_t cm = 0, cv = 0;
    for (const bm_item& it0 : v) {
      bm_item it = it0;
      const uint64_t nch = it.nwg;
      if (objs[it.obj].ihlen == BM_IH_MAIN) {
        it.chunk_base = (uint32_t)cm;
        cm += nch;
        v[k++] = it;
      } else {
        it.chunk_base = (uint32_t)cv;
        cv += nch;
        var.push_back(it);
      }
    }
    p.nmain[s] = (uint32_t)k;
    p.chmain[s] = (uint32_t)cm;
    std::copy(var.begin(), var.end(), v.begin() + (ptrdiff_t)k);
    p.nchunks[s] = (uint32_t)(cm + cv);
  }
}

// ---------------------------------------------------------------------------------------
// per-device stepping: claims from the frontier
// ---------------------------------------------------------------------------------------
bool XPool::needed(uint32_t x, const BatchState* b) const {
  if (!owner[x]) return false;
  if (ref[x]) return true;  // a launch in flight may still publish there
  const uint32_t o = owner[x] - 1;
  // its object still holds it, is searching and has items in flight (which may not carry the slot
  // yet: they were planned before it was allocated)
  return b && o < b->n && b->xs[o] == x + 1 && b->done[o] == BMPOW_PENDING && b->nfly[o] > 0;
}

int XPool::alloc(uint32_t obj, BatchState* b) {
  int got = -1;
  for (uint32_t x = 0; x < BM_XSLOTS && got < 0; ++x)
    if (owner[x] == 0 && ref[x] == 0) got = (int)x;
  if (got < 0) {
    // reclaim slots whose owner no longer needs them: released outside release_xslots (the object
    // restarted by init / reset / add, or settled while items planned before the slot were in flight)
    for (uint32_t x = 0; x < BM_XSLOTS; ++x) {
      if (!owner[x] || needed(x, b)) continue;
      const uint32_t o = owner[x] - 1;
      if (b && o < b->n && b->xs[o] == x + 1) b->xs[o] = 0;
      owner[x] = 0;
      if (got < 0) got = (int)x;
    }
  }
  if (got >= 0) owner[got] = obj + 1;
  return got;
}

size_t XPool::owned() const {
  size_t n = 0;
  for (uint32_t x = 0; x < BM_XSLOTS; ++x) n += owner[x] != 0;
  return n;
}

bool claimable(const BatchState& b, size_t o) {
  if (b.done[o] != BMPOW_PENDING) return false;
  const std::vector<OpenWin>& w = b.open[o];
  // pieces of the latest window left to hand out, needed unless a hit lies below that window
  if (!w.empty() && w.back().claimed < w.back().P && (!b.hit[o] || w.back().start <= b.nonce[o])) return true;
  // A new window only while it is fewer than kMaxOpen windows past the oldest open one: the running
  // window and the one staged behind it.  Without the cap a shard with nothing of its own kept opening
  // windows of an object whose answer another shard had found but not yet reported (its device knew
  // the bound, so each launch ended at once): a stream of empty launches that used up the run's
  // budget and, in the host-only unit, kept the engine's mutex from the reporting shard's SCHED_IDLE
  // stepper for seconds (tests/native/sched_sim.cpp, scenario batches).
  return !b.hit[o] && !b.top[o] && (w.empty() || (uint16_t)(b.wseq[o] - w.front().seq) < kMaxOpen);
}

namespace {

bool has_pieces(const BatchState& b, size_t o) {
  const std::vector<OpenWin>& w = b.open[o];
  return !w.empty() && w.back().claimed < w.back().P && (!b.hit[o] || w.back().start <= b.nonce[o]);
}

// An object whose search is over: FOUND once it has a hit and every open window starts above it;
// EXHAUSTED once the frontier passed 2^64 - 1 with no hit and nothing open.
bool settle(BatchState& b, size_t o) {
  if (b.done[o] != BMPOW_PENDING) return false;
  const std::vector<OpenWin>& w = b.open[o];
  if (b.hit[o] && (w.empty() || w.front().start > b.nonce[o])) {
    b.done[o] = BMPOW_DONE_FOUND;
    b.next[o] = b.nonce[o] == kU64Max ? kU64Max : b.nonce[o] + 1;
  } else if (!b.hit[o] && b.top[o] && w.empty() && b.lim[o] == kU64Max) {
    b.done[o] = BMPOW_DONE_EXHAUSTED;
    b.next[o] = kU64Max;
  } else {
    return false;
  }
  b.pending--;
  mark_finished(b, (uint32_t)o);
  return true;
}

}  // namespace

uint64_t resume_point(const BatchState& b, size_t o) {
  if (b.done[o] == BMPOW_DONE_FOUND || b.done[o] == BMPOW_DONE_EXHAUSTED) return b.next[o];
  if (!b.open[o].empty()) return b.open[o].front().start;
  if (b.top[o]) return b.lim[o] == kU64Max ? kU64Max : b.lim[o] + 1;
  return b.next[o];
}

namespace {
inline uint64_t sbit(size_t s) { return 1ULL << (s & 63); }
}  // namespace

bool plan_launch(BatchState& b, const PlanCtx& c, Launch& L) {
  while (b.first_pending < b.n && b.done[b.first_pending] != BMPOW_PENDING) ++b.first_pending;
  if (b.pending == 0 || b.broken) return false;
  const size_t S = std::max<size_t>(c.S, 1);
  const bool grouped = c.group && c.group->size() >= S;
  const size_t D = grouped ? std::max<size_t>(c.D, 1) : S;
  // the other shards on this shard's device: they never hold one of its objects at the same time
  uint64_t mates = 0;
  if (grouped)
    for (size_t t = 0; t < S; ++t)
      if (t != c.s && (*c.group)[t] == (*c.group)[c.s]) mates |= sbit(t);
  thread_local std::vector<uint32_t> cand, take;
  cand.clear();
  take.clear();
  size_t C = 0;  // claimable objects (by any shard)
  for (size_t i = b.first_pending; i < b.n; ++i) {
    if (!claimable(b, i)) continue;
    ++C;
    if (b.fly1[i] & mates) continue;  // another shard of this device has the object in flight
    cand.push_back((uint32_t)i);
  }
  if (cand.empty()) return false;
  const bool split = D > 1 && C < D;
  if (split || S == 1) {
    take = cand;
  } else {
    // fair share of the claimable objects, by the shard's rate
    const size_t q = std::max<size_t>(1, (size_t)std::ceil((double)C * c.weight / (double)S - 1e-9));
    auto pass = [&](auto pred) {
      for (uint32_t o : cand)
        if (take.size() < q && pred(o) && std::find(take.begin(), take.end(), o) == take.end()) take.push_back(o);
    };
    // windows with pieces left first (they hold up their objects), then the shard's own objects,
    // then objects no shard holds, then -- only when it found nothing -- other shards' objects
    pass([&](uint32_t o) { return has_pieces(b, o); });
    pass([&](uint32_t o) { return b.holder[o] == (int16_t)c.s; });
    pass([&](uint32_t o) { return b.holder[o] == kNoHolder; });
    if (take.empty()) pass([&](uint32_t) { return true; });
    std::sort(take.begin(), take.end());
  }
  const uint32_t iters = c.budget < ((uint64_t)1 << 26) ? BM_ITERS_SMALL : BM_ITERS;
  const uint64_t chunk = (uint64_t)BM_BLOCK * iters;
  const uint64_t budget_chunks = std::max<uint64_t>(1, c.budget / chunk);
  const uint64_t k = std::max<uint64_t>(1, budget_chunks / take.size());
  // the budget's remainder chunks, one each to the first objects: a launch claims its whole budget, so
  // the claims stay aligned to the run's limit and no small remainder launch follows
  const uint64_t spare = budget_chunks > k * take.size() ? budget_chunks - k * take.size() : 0;
  size_t nth = 0;
  const uint64_t bpw = blocks_per_worker(chunk);
  // columns of a split window's piece: the shard's resident workgroups (less the relay's) over the
  // split objects, at least 4 blocks per column
  const uint64_t share =
      c.resident ? std::max<uint64_t>(1, (c.resident > 1 ? c.resident - 1 : 1) / take.size()) : ~0ULL;
  L.claims.clear();
  L.xslots.clear();
  L.planned = 0;
  L.batch = &b;
  L.plan.items.assign(1, std::vector<bm_item>());
  L.plan.nchunks.assign(1, 0);
  L.plan.nx = 0;
  L.plan.iters = iters;
  L.plan.chunk = chunk;
  std::vector<bm_item>& items = L.plan.items[0];
  uint64_t acc = 0;
  for (uint32_t o : take) {
    std::vector<OpenWin>& ow = b.open[o];
    Claim cl;
    cl.obj = o;
    cl.gen = b.gen[o];
    if (has_pieces(b, o)) {
      OpenWin& w = ow.back();
      cl.start = w.start;
      cl.count = w.count;
      cl.G = w.G;
      cl.P = w.P;
      cl.piece = w.claimed++;
    } else {
      const uint64_t st = b.next[o], lim = b.lim[o];
      const uint16_t P = split ? (uint16_t)D : 1;
      uint64_t want = (k + (nth++ < spare ? 1 : 0)) * chunk;
      if (split) {
        const uint64_t cap = expect_cap(b.objs[o].target, P, chunk);
        want = std::min<uint64_t>(cap, (k * chunk > kU64Max / P) ? kU64Max : k * chunk * P);
      }
      const uint64_t room = lim - st;  // nonces after st up to lim
      if (want - 1 >= room) {
        want = room + 1;  // the window ends at lim (room + 1 wraps to 0 only for [0, 2^64): clamp)
        if (want == 0) want = kU64Max;
        b.top[o] = 1;
        b.next[o] = lim;
      } else {
        b.next[o] = st + want;
      }
      const uint64_t nblk = want / BM_BLOCK + (want % BM_BLOCK ? 1 : 0);
      uint64_t G;
      if (P == 1) {
        G = std::max<uint64_t>(1, (nblk + bpw - 1) / bpw);
        if (c.resident) G = std::min<uint64_t>(G, c.resident);
      } else {
        G = std::max<uint64_t>(1, std::min<uint64_t>(share, (nblk + 4 * P - 1) / (4 * P)));
      }
      ow.push_back(OpenWin{st, want, (uint32_t)G, P, 1, 0, b.wseq[o]++});
      cl.start = st;
      cl.count = want;
      cl.G = (uint32_t)G;
      cl.P = P;
      cl.piece = 0;
    }
    // holder and the cross-shard bound
    if (b.nfly[o] == 0) b.holder[o] = (int16_t)c.s;
    else if (b.holder[o] != (int16_t)c.s) b.holder[o] = kShared;
    b.nfly[o]++;
    if (b.fly1[o] & sbit(c.s)) b.fly2[o] |= sbit(c.s);
    else b.fly1[o] |= sbit(c.s);
    if (c.xp && !b.xs[o] && (cl.P > 1 || b.holder[o] == kShared)) {
      const int x = c.xp->alloc(o, &b);
      if (x >= 0) {
        b.xs[o] = (uint8_t)(x + 1);
        // a fresh slot starts at the object's least hit so far, if any: pieces of a window holding it
        // claimed after the object's previous slot went back stop at it, not at their window's end
        if (c.xreset) c.xreset((uint32_t)x, b.hit[o] ? b.nonce[o] : kU64Max);
      }
    }
    bm_item it;
    std::memset(&it, 0, sizeof it);
    it.start = cl.start;
    it.count = cl.count;
    it.obj = o;
    it.chunk_base = (uint32_t)acc;
    it.g0 = cl.G * cl.piece;
    it.gn = cl.G * cl.P;
    it.nwg = cl.G;
    it.xslot = BM_NO_XSLOT;
    if (b.xs[o] && c.xp) {
      it.xslot = b.xs[o] - 1u;
      c.xp->ref[it.xslot]++;
      L.xslots.push_back(it.xslot);
      L.plan.nx++;
    }
    it.pad = L.claims.size();
    acc += cl.G;
    items.push_back(it);
    // nonces of the piece: its columns' share of the window
    L.planned += cl.P == 1 ? cl.count : std::max<uint64_t>(1, cl.count / cl.P);
    L.claims.push_back(cl);
  }
  L.plan.nchunks[0] = (uint32_t)acc;
  L.plan.C = acc;
  split_kinds(b.objs, b.nvar_slots > 0, L.plan);
  return true;
}

namespace {

// Release the launch's holds on its cross-shard bound slots: a slot whose last in-flight item is
// gone goes back to the pool when its object no longer needs it (finished, restarted, or nothing in
// flight).
void release_xslots(BatchState& b, const Launch& L, XPool* xp) {
  if (!xp) return;
  for (uint32_t x : L.xslots) {
    if (xp->ref[x]) xp->ref[x]--;
    if (xp->ref[x] || !xp->owner[x]) continue;
    const uint32_t o = xp->owner[x] - 1;
    const bool mine = o < b.n && b.xs[o] == x + 1;
    if (!mine || b.done[o] != BMPOW_PENDING || b.nfly[o] == 0) {
      if (mine) b.xs[o] = 0;
      xp->owner[x] = 0;
    }
  }
}

// Give an object's cross-shard slot back once nothing needs it: no in-flight item carries it and the
// object is finished or has nothing in flight (a slot whose last carrying item completed
// while older items of its object were still in flight kept its owner, and nothing freed it later).
void free_idle_xslot(BatchState& b, uint32_t o, XPool* xp) {
  if (!xp || o >= b.n || !b.xs[o]) return;
  const uint32_t x = b.xs[o] - 1u;
  if (xp->ref[x] || (b.done[o] == BMPOW_PENDING && b.nfly[o] > 0)) return;
  if (xp->owner[x] == o + 1) xp->owner[x] = 0;
  b.xs[o] = 0;
}

// The item's piece is no longer in flight.
const Claim* unfly(BatchState& b, const Launch& L, const bm_item& it) {
  const Claim& cl = L.claims[it.pad];
  const uint32_t o = cl.obj;
  if (o >= b.n || b.gen[o] != cl.gen) return nullptr;  // stale: the slot restarted since the plan
  if (b.nfly[o]) b.nfly[o]--;
  if (b.nfly[o] == 0) b.holder[o] = kNoHolder;
  const uint64_t bit = sbit(L.shard);
  if (b.fly2[o] & bit) b.fly2[o] &= ~bit;
  else b.fly1[o] &= ~bit;
  return &cl;
}

// Price the object's applied items against its answer once that is final (WasteStats).  With no hit
// and nothing in flight, every applied item lies below any hit to come (later windows start at the
// frontier): none of them hashed past an answer.
void price_waste(BatchState& b, uint32_t o, WasteStats& w) {
  std::vector<WasteRec>& rs = b.wrec[o];
  if (rs.empty()) return;
  uint64_t h;
  if (b.done[o] == BMPOW_DONE_FOUND) h = b.nonce[o];
  else if (b.done[o] == BMPOW_DONE_EXHAUSTED || (!b.hit[o] && b.nfly[o] == 0)) h = kU64Max;
  else return;  // a hit that is not final yet, or items in flight that may hold one below these
  for (const WasteRec& r : rs) {
    uint64_t above = 0, hashed = 0;
    waste_of(r, h, above, hashed);
    w.hashed += hashed;
    if (r.P > 1) w.split += above;
    else if (r.start > h) w.later += above;
    else w.window += above;
  }
  rs.clear();
}

}  // namespace

void waste_of(const WasteRec& r, uint64_t h, uint64_t& above, uint64_t& hashed) {
  const uint64_t nblk = r.count / BM_BLOCK + (r.count % BM_BLOCK ? 1 : 0);
  const uint64_t gn = std::max<uint32_t>(r.gn, 1), nwg = std::max<uint32_t>(r.nwg, 1);
  // units of the item's queue whose block is at or below block x (bm_block_of: row k / nwg, column
  // g0 + k % nwg): the rows below x's, then the item's columns of x's row up to x
  auto upto = [&](uint64_t x) -> uint64_t {
    const uint64_t row = x / gn, rem = x - row * gn;
    return row * nwg + (rem + 1 > r.g0 ? std::min<uint64_t>(nwg, rem + 1 - r.g0) : 0);
  };
  const uint64_t units = nblk ? upto(nblk - 1) : 0;
  const uint64_t got = r.taken > nwg ? std::min<uint64_t>(r.taken - nwg, units) : 0;
  hashed = got * BM_BLOCK;
  if (h < r.start) {
    above = hashed;
    return;
  }
  const uint64_t hb = (h - r.start) / BM_BLOCK;
  const uint64_t below = hb >= nblk ? units : upto(hb);
  above = got > below ? (got - below) * BM_BLOCK : 0;
}

size_t apply_launch(BatchState& b, const Launch& L, XPool* xp, const std::function<void(uint32_t, uint64_t)>& publish,
                    WasteStats* waste) {
  const std::vector<bm_item>& items = L.plan.items[0];
  thread_local std::vector<uint32_t> touched;
  touched.clear();
  for (size_t k = 0; k < items.size(); ++k) {
    const Claim* cl = unfly(b, L, items[k]);
    if (!cl) continue;
    const uint32_t o = cl->obj;
    std::vector<OpenWin>& ow = b.open[o];
    auto w = std::lower_bound(ow.begin(), ow.end(), cl->start,
                              [](const OpenWin& x, uint64_t st) { return x.start < st; });
    if (w != ow.end() && w->start == cl->start && ++w->done == w->P) ow.erase(w);
    const bm_result& r = L.res[k];
    if (r.found && (!b.hit[o] || r.nonce < b.nonce[o])) {
      b.hit[o] = 1;
      b.nonce[o] = r.nonce;
      b.trial[o] = r.trial;
      if (b.xs[o] && publish) publish(b.xs[o] - 1u, r.nonce);
    }
    if (waste)
      b.wrec[o].push_back(WasteRec{cl->start, cl->count, items[k].g0, items[k].gn, items[k].nwg, r.pad, cl->P});
    touched.push_back(o);
  }
  size_t fin = 0;
  for (uint32_t o : touched) fin += settle(b, o) ? 1 : 0;
  if (waste)
    for (uint32_t o : touched) price_waste(b, o, *waste);
  release_xslots(b, L, xp);
  for (uint32_t o : touched) free_idle_xslot(b, o, xp);
  return fin;
}

void drop_launch(BatchState& b, const Launch& L, XPool* xp) {
  for (const bm_item& it : L.plan.items[0]) unfly(b, L, it);
  release_xslots(b, L, xp);
  for (const Claim& cl : L.claims)
    if (cl.obj < b.n && b.gen[cl.obj] == cl.gen) free_idle_xslot(b, cl.obj, xp);
  b.broken = true;
}

// ---------------------------------------------------------------------------------------
// min-trial probe
// ---------------------------------------------------------------------------------------
void MinTrial::init(size_t n, const uint64_t* start, const uint64_t* count, uint64_t* min_out, uint64_t* argmin_out) {
  cur.assign(start, start + n);
  left.assign(count, count + n);
  any.assign(n, 0);
  first = 0;
  for (size_t i = 0; i < n; ++i) {
    if (left[i] && left[i] - 1 > kU64Max - start[i]) left[i] = kU64Max - start[i] + 1;  // stop at 2^64-1
    min_out[i] = kU64Max;
    argmin_out[i] = start[i];
  }
}

bool MinTrial::plan(uint64_t total_chunks, std::vector<Win>& wins, uint64_t& C) {
  const uint64_t chunk = BM_CHUNK;
  while (first < left.size() && left[first] == 0) ++first;
  if (first == left.size()) return false;
  wins.clear();
  uint64_t acc = 0;
  for (size_t i = first; i < left.size() && acc < total_chunks; ++i) {
    if (left[i] == 0) continue;
    const uint64_t room = (total_chunks - acc) * chunk;
    const uint64_t want = std::min(left[i], room);
    const uint64_t ch = (want + chunk - 1) / chunk;
    wins.push_back({(uint32_t)i, cur[i], want, ch, acc});
    acc += ch;
  }
  C = acc;
  return true;
}

void MinTrial::reduce_parts(const std::vector<bm_item>& items, const bm_minpart* parts, uint64_t* min_out,
                            uint64_t* argmin_out) {
  for (const bm_item& it : items) {
    const uint64_t nch = it.nwg;
    uint64_t& mt = min_out[it.obj];
    uint64_t& mn = argmin_out[it.obj];
    for (uint64_t c = it.chunk_base; c < it.chunk_base + nch; ++c) {
      const bm_minpart& q = parts[c];
      if (!any[it.obj] || q.trial < mt || (q.trial == mt && q.nonce < mn)) {
        any[it.obj] = 1;
        mt = q.trial;
        mn = q.nonce;
      }
    }
  }
}

void MinTrial::advance(const std::vector<Win>& wins) {
  for (const Win& w : wins) {
    left[w.obj] -= w.count;
    if (left[w.obj]) cur[w.obj] += w.count;
  }
}

// ---------------------------------------------------------------------------------------
// receive-side verification
// ---------------------------------------------------------------------------------------
uint64_t padded_blocks(uint64_t m) { return (m + 17 + 127) / 128; }

void pad_into(const uint8_t* msg, uint64_t m, uint8_t* dst, uint64_t nblk) {
  const uint64_t total = nblk * 128;
  std::memcpy(dst, msg, m);
  std::memset(dst + m, 0, total - m);
  dst[m] = 0x80;
  const uint64_t bits_lo = m << 3, bits_hi = m >> 61;  // 128-bit big-endian bit length
  for (int j = 0; j < 8; ++j) {
    dst[total - 16 + j] = (uint8_t)(bits_hi >> (56 - 8 * j));
    dst[total - 8 + j] = (uint8_t)(bits_lo >> (56 - 8 * j));
  }
}

// pad_into with non-temporal 16-B stores, for a 16-B aligned destination that is written once and
// read by the DMA engine (the pinned staging): no read-for-ownership of the destination lines, so
// the copy moves ~2/3 of the bytes a cached copy does.  The caller fences (stream_fence) before the
// buffer is handed to the device.
void pad_into_stream(const uint8_t* msg, uint64_t m, uint8_t* dst, uint64_t nblk) {
  const uint64_t total = nblk * 128;
  const uint64_t full = m & ~(uint64_t)15;  // whole 16-B pieces of the message
  for (uint64_t o = 0; o < full; o += 16)
    _mm_stream_si128((__m128i*)(dst + o), _mm_loadu_si128((const __m128i*)(msg + o)));
  alignas(16) uint8_t tail[256];  // the rest of the message, the padding and the length: <= 2 blocks
  const uint64_t rest = total - full;
  std::memset(tail, 0, rest);
  std::memcpy(tail, msg + full, m - full);
  tail[m - full] = 0x80;
  const uint64_t bits_lo = m << 3, bits_hi = m >> 61;
  for (int j = 0; j < 8; ++j) {
    tail[rest - 16 + j] = (uint8_t)(bits_hi >> (56 - 8 * j));
    tail[rest - 8 + j] = (uint8_t)(bits_lo >> (56 - 8 * j));
  }
  for (uint64_t o = 0; o < rest; o += 16)
    _mm_stream_si128((__m128i*)(dst + full + o), _mm_load_si128((const __m128i*)(tail + o)));
}

void stream_fence() { _mm_sfence(); }

void plan_bins(VPart& pt, size_t nbins) {
  const size_t m = pt.orig.size();
  const size_t G = (m + BV_BLOCK - 1) / BV_BLOCK;
  pt.nbins = nbins;
  pt.bins.assign(nbins + 1 + G, 0);
  if (nbins == 0) return;
  // LPT: groups arrive longest first (the objects are sorted); min-heap of (load, bin)
  using LB = std::pair<uint64_t, uint32_t>;
  std::priority_queue<LB, std::vector<LB>, std::greater<LB>> heap;
  for (uint32_t b = 0; b < nbins; ++b) heap.push({0, b});
  std::vector<uint32_t> owner(G), count(nbins, 0);
  for (size_t g = 0; g < G; ++g) {
    LB top = heap.top();
    heap.pop();
    owner[g] = top.second;
    count[top.second]++;
    top.first += (uint64_t)pt.ho[g * BV_BLOCK].nblk + 2;
    heap.push(top);
  }
  uint32_t* off = pt.bins.data();
  for (size_t b = 0; b < nbins; ++b) off[b + 1] = off[b] + count[b];
  std::vector<uint32_t> fill(off, off + nbins);
  uint32_t* list = off + nbins + 1;
  for (size_t g = 0; g < G; ++g) list[fill[owner[g]]++] = (uint32_t)g;
}

int plan_verify(const std::vector<Span>& objs, size_t S, std::vector<VPart>& parts, uint64_t& total_blocks,
                size_t nbins) {
  const size_t n = objs.size();
  if (n > 0xffffffffULL) return BMPOW_E_ARG;
  // scratch kept across calls (a flood's vectors are tens of MB: fresh ones cost a page fault per
  // 4 KB, more than the planning itself)
  static thread_local std::vector<uint32_t> nblk, order;
  nblk.resize(n);
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t b = padded_blocks(objs[i].len - 8);
    if (b > 0xffffffffULL) return BMPOW_E_ARG;
    nblk[i] = (uint32_t)b;
    total += b;
  }
  if (total > 0xffffffffULL) return BMPOW_E_ARG;  // payload pool above 2^32 blocks (512 GiB)
  total_blocks = total;
  // stable counting sort by block count, descending (block counts are small: <= 2,049 for the
  // protocol's 256 KiB objects, larger ones fall into one overflow bucket sorted on their own)
  constexpr uint32_t kBuckets = 4096;
  order.resize(n);
  {
    std::vector<size_t> cnt(kBuckets + 1, 0);
    for (size_t i = 0; i < n; ++i) cnt[std::min(nblk[i], kBuckets)]++;
    std::vector<size_t> pos(kBuckets + 1, 0);
    size_t acc = 0;
    for (size_t b = kBuckets + 1; b-- > 0;) {  // descending
      pos[b] = acc;
      acc += cnt[b];
    }
    for (size_t i = 0; i < n; ++i) order[pos[std::min(nblk[i], kBuckets)]++] = (uint32_t)i;
    if (cnt[kBuckets] > 1)
      std::stable_sort(order.begin(), order.begin() + (ptrdiff_t)cnt[kBuckets],
                       [&](uint32_t a, uint32_t b) { return nblk[a] > nblk[b]; });
  }
  // parts are filled in place: a caller that passes the previous call's parts back keeps their
  // vectors' capacity
  size_t k = 0, used = 0;
  uint64_t acc = 0;
  for (size_t s = 0; s < S && k < n; ++s) {
    const uint64_t goal = total * (s + 1) / S;
    size_t k1 = k;
    for (uint64_t a = acc; k1 < n && (a < goal || s == S - 1); ++k1) a += nblk[order[k1]];
    if (k1 == k) continue;
    if (parts.size() <= used) parts.emplace_back();
    VPart& pt = parts[used++];
    pt.shard = s;
    const size_t m = k1 - k;
    pt.orig.resize(m);
    pt.ho.resize(m);
    uint64_t blk = 0;
    for (size_t j = 0; j < m; ++j) {
      const uint32_t i = order[k + j];
      pt.orig[j] = i;
      pt.ho[j].blk = (uint32_t)blk;
      pt.ho[j].nblk = nblk[i];
      pt.ho[j].nonce = 0;  // pad_range reads it with the payload
      blk += nblk[i];
    }
    acc += blk;
    k = k1;
    pt.blocks = blk;
    pt.eol.assign(m, 0);
    pt.bins.clear();
    pt.nbins = 0;
    if (nbins) plan_bins(pt, nbins);
  }
  parts.resize(used);
  return 0;
}

namespace {

// Persistent workers for parallel_for: a flood's padding calls it once per 64 MB staging chunk
// (17 times for 1.1 GB), and creating 15 threads per call cost more than the copy they share.
// One caller at a time uses the pool; a concurrent caller (or a forked child, which inherits the
// pool's state but not its threads) spawns threads of its own, as before.
class Pool {
 public:
  explicit Pool(size_t workers) : pid_(getpid()) {
    for (size_t w = 1; w <= workers; ++w) th_.emplace_back(&Pool::work, this, w);
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  size_t workers() const { return th_.size(); }
  bool usable() const { return getpid() == pid_; }
  std::mutex call_mu;  // held by the one caller using the pool
  // Run body over nparts contiguous parts of [0, n): part 0 on the caller, the others on workers.
  void run(size_t n, size_t nparts, const std::function<void(size_t, size_t)>& body) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      body_ = &body;
      n_ = n;
      nparts_ = nparts;
      pending_ = nparts - 1;
      ++gen_;
    }
    cv_.notify_all();
    body(0, n / nparts);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    body_ = nullptr;
  }

 private:
  void work(size_t id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t, size_t)>* body;
      size_t n, nparts;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
        if (id >= nparts_) continue;
        body = body_;
        n = n_;
        nparts = nparts_;
      }
      (*body)(n * id / nparts, n * (id + 1) / nparts);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  const pid_t pid_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t, size_t)>* body_ = nullptr;
  size_t n_ = 0, nparts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

constexpr size_t kMaxThreads = 16;  // the GPU box's CPU share

Pool& pool() {
  static Pool p(std::min<size_t>(kMaxThreads, std::max<size_t>(1, std::thread::hardware_concurrency())) - 1);
  return p;
}

}  // namespace

void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& body) {
  const size_t hw = std::max<size_t>(1, std::thread::hardware_concurrency());
  const size_t nth = std::max<size_t>(1, std::min<size_t>({kMaxThreads, hw, n / std::max<size_t>(grain, 1) + 1}));
  if (nth == 1) return body(0, n);
  Pool& p = pool();
  if (p.usable() && nth <= p.workers() + 1) {
    std::unique_lock<std::mutex> lk(p.call_mu, std::try_to_lock);
    if (lk.owns_lock()) return p.run(n, nth, body);
  }
  std::vector<std::thread> th;
  for (size_t t = 1; t < nth; ++t) th.emplace_back(body, n * t / nth, n * (t + 1) / nth);
  body(0, n / nth);
  for (auto& x : th) x.join();
}

void pad_range(const std::vector<Span>& objs, VPart& pt, size_t j0, size_t j1, uint64_t blk0, uint8_t* dst) {
  if (j1 <= j0) return;
  std::vector<bv_obj>& ho = pt.ho;
  const size_t m = j1 - j0;
  const uint64_t bytes = (uint64_t)(ho[j1 - 1].blk + ho[j1 - 1].nblk - ho[j0].blk) * 128;
  // a thread per ~2 MB (and per >= 64 objects), at most 16
  const size_t grain = std::max<size_t>(64, (size_t)(m / (bytes / (2u << 20) + 1)));
  parallel_for(m, grain, [&](size_t a, size_t b) {
    constexpr size_t kAhead = 8;  // objects are read in sorted order, i.e. scattered: prefetch them
    for (size_t j = j0 + a; j < j0 + b; ++j) {
      if (j + 2 * kAhead < j0 + b) __builtin_prefetch(&objs[pt.orig[j + 2 * kAhead]]);
      if (j + kAhead < j0 + b) {
        const Span& nx = objs[pt.orig[j + kAhead]];
        __builtin_prefetch(nx.p);
        __builtin_prefetch(nx.p + 64);
      }
      const Span& sp = objs[pt.orig[j]];
      ho[j].nonce = load_be64(sp.p);
      pt.eol[j] = sp.len >= 16 ? load_be64(sp.p + 8) : 0;
#ifdef BMSCHED_PAD_CACHED
      pad_into(sp.p + 8, sp.len - 8, dst + (uint64_t)(ho[j].blk - blk0) * 128, ho[j].nblk);
#else
      pad_into_stream(sp.p + 8, sp.len - 8, dst + (uint64_t)(ho[j].blk - blk0) * 128, ho[j].nblk);
#endif
    }
    stream_fence();  // this thread's streaming stores are globally visible before the join
  });
}

// Python ints until the true division by 2**16 (correctly rounded: the exact 128-bit product
// converted once, then an exact power-of-two scale), IEEE doubles after, and an exact
// int-vs-float comparison at the end.
int pow_sufficient(uint64_t pow, uint64_t len, uint64_t ntpb, uint64_t extra, int64_t recv, uint64_t eol) {
  if (ntpb < 1000) ntpb = 1000;
  if (extra < 1000) extra = 1000;
  __int128 ttl = (__int128)eol - (__int128)recv;
  if (ttl < 300) ttl = 300;
  const unsigned __int128 le = (unsigned __int128)len + extra;
  const unsigned __int128 prod = (unsigned __int128)ttl * le;
  // int -> double correctly rounded either way; the int64 conversion is the hardware one
  const double q = (prod >> 63) ? (double)prod / 65536.0 : (double)(int64_t)prod / 65536.0;
  const double x = (double)le + q;
  const double y = (double)ntpb * x;
  const double t = 18446744073709551616.0 / y;
  if (t >= 18446744073709551616.0) return 1;
  return pow <= (uint64_t)t ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// Service
// ---------------------------------------------------------------------------------------
Service::Service(ServiceOps ops, bool verify) : ops_(std::move(ops)), verify_(verify) {
  th_ = std::thread(&Service::loop, this);
}

Service::~Service() { stop(); }

void Service::stop() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stopping_ = true;
  }
  cv_in_.notify_all();
  cv_out_.notify_all();
  std::lock_guard<std::mutex> j(join_mu_);  // stop() may race from two threads
  if (th_.joinable()) th_.join();
}

int Service::submit(size_t n, const uint8_t* ihs, const uint64_t* targets, uint64_t* tickets_out,
                    const uint64_t* ih_off) {
  if (n == 0) return 0;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stopping_) return BMPOW_E_STATE;
    if (ih_off || !in_off_.empty()) {  // any length: the queue keeps per-object offsets from here on
      if (in_off_.empty())
        for (size_t i = 0; i <= in_ticket_.size(); ++i) in_off_.push_back(64 * i);
      const uint64_t base = in_ih_.size();
      for (size_t i = 1; i <= n; ++i) in_off_.push_back(base + (ih_off ? ih_off[i] - ih_off[0] : 64 * i));
    }
    if (ih_off) in_ih_.insert(in_ih_.end(), ihs + ih_off[0], ihs + ih_off[n]);
    else in_ih_.insert(in_ih_.end(), ihs, ihs + 64 * n);
    in_target_.insert(in_target_.end(), targets, targets + n);
    for (size_t i = 0; i < n; ++i) {
      const uint64_t t = next_ticket_++;
      in_ticket_.push_back(t);
      if (tickets_out) tickets_out[i] = t;
    }
    outstanding_ += n;
  }
  cv_in_.notify_all();
  return 0;
}

int Service::poll(size_t cap, int timeout_ms, uint64_t* tickets, uint64_t* nonce, uint64_t* trial, uint8_t* done,
                  std::string& err) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !out_.empty() || error_ || stopping_; };
  thread_local std::vector<Out> popped;
  // (a plain wait is used for < 0: GCC 11's ThreadSanitizer mis-reports timed waits)
  if (timeout_ms < 0) cv_out_.wait(lk, ready);
  else if (!cv_out_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) return 0;
  if (out_.empty() && error_) {
    err = err_;
    return error_;
  }
  cap = std::min<size_t>(cap, 0x7fffffff);
  const size_t k = std::min(cap, out_.size());
  popped.assign(out_.begin(), out_.begin() + (ptrdiff_t)k);
  out_.erase(out_.begin(), out_.begin() + (ptrdiff_t)k);
  outstanding_ -= k;
  lk.unlock();
  // the host re-check runs on the polling thread, outside the lock, while the next step runs
  for (size_t j = 0; j < k; ++j) {
    Done d = popped[j].d;
    const Out& o = popped[j];
    if (verify_ && d.done == BMPOW_DONE_FOUND &&
        ((o.var ? host_trial_len(o.ihv.data(), o.ihv.size(), d.nonce) : host_trial(o.ih, d.nonce)) != d.trial ||
         d.trial > o.target))
      d.done = BMPOW_DONE_BADHASH;
    tickets[j] = d.ticket;
    if (nonce) nonce[j] = d.nonce;
    if (trial) trial[j] = d.trial;
    if (done) done[j] = d.done;
  }
  return (int)k;
}

void Service::cancel() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    cancel_ = true;
    error_ = 0;
    err_.clear();
    in_ih_.clear();
    in_off_.clear();
    in_target_.clear();
    in_ticket_.clear();
    out_.clear();
    outstanding_ = 0;
  }
  cv_in_.notify_all();
}

size_t Service::outstanding() {
  std::lock_guard<std::mutex> lk(mu_);
  return outstanding_;
}

void Service::loop() {
  std::vector<uint8_t> ih;
  std::vector<uint64_t> off, tg, tk, slot_ticket, slot_target;
  std::vector<uint8_t> slot_ih;  // 64 B per slot: the object's initialHash, for the re-check
  std::vector<std::vector<uint8_t>> slot_ihv;  // per slot: an initialHash of another length
  std::vector<uint8_t> slot_var;               // per slot: 1 when slot_ihv holds its initialHash
  std::vector<uint32_t> slots;
  constexpr size_t kTake = 4096;
  std::vector<uint32_t> fs(kTake);
  std::vector<uint64_t> fn(kTake), ft(kTake);
  std::vector<uint8_t> fd(kTake);
  std::vector<Out> fin;
  size_t live = 0;  // objects in the session
  for (;;) {
    bool cancel = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_in_.wait(lk, [&] { return stopping_ || cancel_ || (!error_ && (live > 0 || !in_ticket_.empty())); });
      if (stopping_) return;
      cancel = cancel_;
      cancel_ = false;
      ih.swap(in_ih_);
      off.swap(in_off_);
      tg.swap(in_target_);
      tk.swap(in_ticket_);
    }
    fin.clear();
    std::string err;
    int rc = 0;
    if (cancel) {
      rc = ops_.reset(err);
      live = 0;
    }
    if (rc >= 0 && !tk.empty()) {
      slots.resize(tk.size());
      const uint64_t* ih_off = off.empty() ? nullptr : off.data();
      rc = ops_.add(tk.size(), ih.data(), ih_off, tg.data(), slots.data(), err);
      if (rc >= 0) {
        for (size_t i = 0; i < tk.size(); ++i) {
          if (slot_ticket.size() <= slots[i]) {
            slot_ticket.resize((size_t)slots[i] + 1);
            slot_target.resize((size_t)slots[i] + 1);
            slot_ih.resize(64 * ((size_t)slots[i] + 1));
            slot_ihv.resize((size_t)slots[i] + 1);
            slot_var.resize((size_t)slots[i] + 1);
          }
          slot_ticket[slots[i]] = tk[i];
          slot_target[slots[i]] = tg[i];
          const size_t len = ih_len(ih_off, i);
          const uint8_t* p = ih_ptr(ih.data(), ih_off, i);
          slot_var[slots[i]] = len != 64;
          if (len == 64) {
            memcpy(&slot_ih[64 * (size_t)slots[i]], p, 64);
            std::vector<uint8_t>().swap(slot_ihv[slots[i]]);
          } else {
            slot_ihv[slots[i]].assign(p, p + len);
          }
        }
        live += tk.size();
      }
    }
    if (rc >= 0 && live) rc = ops_.step(err);
    if (rc >= 0) {
      for (;;) {
        const size_t k = ops_.take(kTake, fs.data(), fn.data(), ft.data(), fd.data());
        for (size_t j = 0; j < k; ++j) {
          Out o;
          o.d = {slot_ticket[fs[j]], fn[j], ft[j], fd[j]};
          o.target = slot_target[fs[j]];
          if (slot_var[fs[j]]) {
            o.var = true;
            o.ihv = slot_ihv[fs[j]];
          } else {
            memcpy(o.ih, &slot_ih[64 * (size_t)fs[j]], 64);
          }
          fin.push_back(std::move(o));
        }
        live -= k;
        if (k < kTake) break;
      }
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!cancel_) {  // a cancel since this step started drops its results too
        out_.insert(out_.end(), fin.begin(), fin.end());
        if (rc < 0) {
          error_ = rc;
          err_ = err;
        }
      }
    }
    cv_out_.notify_all();
    ih.clear();
    off.clear();
    tg.clear();
    tk.clear();
  }
}

// ---------------------------------------------------------------------------------------
// Engine: one stepper thread per shard
// ---------------------------------------------------------------------------------------
Engine::Engine(EngineOps ops, size_t S, uint32_t resident, uint64_t step_trials)
    : ops_(std::move(ops)), S_(S), resident_(resident), D_(S), step_(step_trials), sh_(S) {
  rates.reset(S);
  stats.shard_ms.assign(S, 0.0);
  stats.shard_trials.assign(S, 0);
  for (size_t s = 0; s < S; ++s) {
    sh_[s].buf[0].buf = 0;
    sh_[s].buf[1].buf = 1;
    sh_[s].buf[0].shard = sh_[s].buf[1].shard = s;
  }
  for (size_t s = 0; s < S; ++s) th_.emplace_back(&Engine::stepper, this, s);
}

Engine::~Engine() {
  {
    std::lock_guard<std::mutex> lk(mu);
    stop_ = true;
    limit_ = claimed_;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

void Engine::set_throttle(size_t s, double ms) {
  std::lock_guard<std::mutex> lk(mu);
  if (s < S_) sh_[s].throttle_ms = ms;
}

void Engine::set_groups(std::unique_lock<std::mutex>& lk, const std::vector<uint16_t>& group, uint32_t resident) {
  // the per-object holdings (fly1/fly2, a window's smask) are read against the groups: nothing in flight
  drain(lk);
  if (group.size() == S_) {
    group_ = group;
    std::vector<uint16_t> ids(group);
    std::sort(ids.begin(), ids.end());
    D_ = (size_t)(std::unique(ids.begin(), ids.end()) - ids.begin());
  } else {
    group_.clear();
    D_ = S_;
  }
  resident_ = resident;
  cv_.notify_all();
}

bool Engine::can_plan() const {
  return b_ && !b_->broken && !error_ && !stop_ && claimed_ < limit_ && !(ops_.aborted && ops_.aborted());
}

void Engine::thread_info(std::vector<double>& cpu_s, std::vector<int>& policy) {
  cpu_s.assign(S_, 0.0);
  policy.assign(S_, -2);
  for (size_t s = 0; s < S_; ++s) {
    policy[s] = sh_[s].policy;
    timespec ts;
    if (sh_[s].have_clock && clock_gettime(sh_[s].cpu_clock, &ts) == 0) cpu_s[s] = (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
  }
}

void Engine::stepper(size_t s) {
  if (ops_.thread_init) ops_.thread_init(s);
  std::unique_lock<std::mutex> lk(mu);
  EShard& e = sh_[s];
  e.policy = sched_getscheduler(0);
  e.have_clock = pthread_getcpuclockid(pthread_self(), &e.cpu_clock) == 0;
  for (;;) {
    // 1. while fewer than two launches are in flight, plan the next one (it queues behind the
    //    running one on the shard's stream)
    if (e.q.size() < 2 && can_plan()) {
      if (e.throttle_ms > 0 && !e.throttled) {
        // A/B knob: a slow device -- the delay comes before the plan, never between the plan and the
        // enqueue (below)
        const double thr = e.throttle_ms;
        lk.unlock();
        std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(thr * 1000)));
        lk.lock();
        e.throttled = true;
        continue;  // the state changed meanwhile: check again
      }
      e.throttled = false;
      Launch& L = e.buf[e.next];
      PlanCtx c;
      c.s = s;
      c.S = S_;
      if (!group_.empty()) {
        c.group = &group_;
        c.D = D_;
      }
      c.budget = std::min<uint64_t>(step_, limit_ - claimed_);
      c.resident = resident_;
      std::vector<double> w;
      if (S_ > 1 && rates.weights(w)) c.weight = w[s];
      c.xp = &xp_;
      c.xreset = [this](uint32_t x, uint64_t v) {
        if (ops_.xstore) ops_.xstore(x, v);
      };
      if (plan_launch(*b_, c, L)) {
        e.next ^= 1;
        claimed_ += L.planned;
        stats.planned += L.planned;
        ++inflight_;
        e.q.push_back(&L);
        // Enqueued under the mutex, in one piece with the plan: a slot's reuse
        // (take_done + add, or a scratch re-init) writes the new object on every shard's stream under
        // this mutex too (init_slots), so a launch is queued either before that slot init -- it then
        // hashes the old record, its results are stale by the slot's generation, and the init resets
        // best[] / found[] behind it -- or after it, planned from the new generation.  Enqueued after the
        // unlock, a launch planned for the old occupant could run after the init and leave a hit of the
        // new object from the old window in best[], which the new object's first window then reported as
        // found: nonces between its frontier and that hit were never hashed.  An enqueue is a handful of
        // asynchronous HIP calls (~20 us), once per launch of ~80 ms.
        std::string err;
        L.t_launch = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
        const int rc = ops_.launch(L, err);
        if (rc < 0) {
          e.q.pop_back();
          e.next ^= 1;  // its buffer is free again
          --inflight_;
          applied_ += L.planned;
          drop_launch(*L.batch, L, &xp_);
          if (!error_) {
            error_ = rc;
            err_ = err;
          }
        }
        cv_.notify_all();
        continue;
      }
    }
    // 2. wait for the oldest launch and fold it in
    if (!e.q.empty()) {
      Launch& L = *e.q.front();
      lk.unlock();
      std::string err;
      const int rc = ops_.wait(L, err);
      lk.lock();
      e.q.pop_front();
      --inflight_;
      applied_ += L.planned;
      if (rc < 0) {
        drop_launch(*L.batch, L, &xp_);
        if (!error_) {
          error_ = rc;
          err_ = err;
        }
      } else {
        stats.launches++;
        stats.trials += L.trials;
        stats.kernel_ms += L.ms;
        stats.shard_ms[s] += L.ms;
        stats.shard_trials[s] += L.trials;
        rates.sample(s, L.trials, L.ms);
        apply_launch(
            *L.batch, L, &xp_,
            [this](uint32_t x, uint64_t v) {
              if (ops_.xstore) ops_.xstore(x, v);
            },
            &stats.waste);
      }
      cv_.notify_all();
      continue;
    }
    if (stop_) return;
    cv_.wait(lk);
  }
}

void Engine::drain(std::unique_lock<std::mutex>& lk) {
  limit_ = claimed_;
  cv_.wait(lk, [&] { return inflight_ == 0; });
}

void Engine::attach(std::unique_lock<std::mutex>& lk, BatchState* b) {
  if (b_ != b) {
    drain(lk);
    b_ = b;
    xp_ = XPool();  // nothing in flight: no slot is carried, and the owners were the old batch's objects
  }
  clear_error();
}

size_t Engine::xslots_owned(bool gc) {
  if (gc)
    for (uint32_t x = 0; x < BM_XSLOTS; ++x)
      if (xp_.owner[x] && !xp_.needed(x, b_)) {
        const uint32_t o = xp_.owner[x] - 1;
        if (b_ && o < b_->n && b_->xs[o] == x + 1) b_->xs[o] = 0;
        xp_.owner[x] = 0;
      }
  return xp_.owned();
}

void Engine::detach(std::unique_lock<std::mutex>& lk) {
  drain(lk);
  b_ = nullptr;
}

int Engine::run(std::unique_lock<std::mutex>& lk, uint64_t budget, bool lookahead, const std::function<bool()>& done,
                std::string& err) {
  if (!b_) {
    err = "no batch attached";
    return BMPOW_E_STATE;
  }
  if (b_->broken) {
    err = "a launch of this batch was lost to a device error: reset it";
    return BMPOW_E_STATE;
  }
  const uint64_t a0 = applied_;
  // Lookahead: with at least as many pending objects as shards, two launches per shard -- when a launch
  // completes and run() returns, the stepper stages its next launch at once, before the caller's next
  // call raises the limit (with one, it went on to wait for its other launch, and its device idled while
  // the host planned: C2 ran 2^28-trial launches at 99.78 % busy, profiles/r04/); with fewer (split
  // windows, each piece a fraction of 2E) one, since a piece claimed past the answer is waste.
  const uint64_t extra = lookahead ? (b_->pending >= S_ ? 2 : 1) * S_ * step_ : 0;
  const bool unbounded = budget == kU64Max || a0 + budget < a0 || a0 + budget + extra < a0 + budget;
  limit_ = unbounded ? kU64Max : a0 + budget + extra;
  cv_.notify_all();
  int rc = 0;
  for (;;) {
    if (error_) {
      err = err_;
      rc = error_;
      break;
    }
    if (ops_.aborted && ops_.aborted()) {
      err = "aborted";
      rc = BMPOW_E_ABORTED;
      break;
    }
    if (done && done()) break;
    if (!unbounded && applied_ - a0 >= budget) break;
    if (inflight_ == 0) {
      bool any = false;
      if (claimed_ < limit_ && b_->pending)
        for (size_t i = b_->first_pending; i < b_->n && !any; ++i) any = claimable(*b_, i);
      if (!any) break;
    }
    cv_.wait(lk);
  }
  // an unbounded call (a search bounded by its objects' lim), an error or an abort leaves nothing
  // more to claim; a bounded call keeps its lookahead launch per shard queued behind the running one
  if (unbounded || rc < 0) limit_ = claimed_;
  return rc;
}

int set_thread_background(const char* policy) {
  const char* env = std::getenv("BMPOW_THREAD_POLICY");
  const std::string p = (env && *env) ? env : (policy ? policy : "idle");
  sched_param sp;
  std::memset(&sp, 0, sizeof sp);
  if (p == "idle") {
    (void)pthread_setschedparam(pthread_self(), SCHED_IDLE, &sp);
  } else if (p == "batch") {
    (void)pthread_setschedparam(pthread_self(), SCHED_BATCH, &sp);
    (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), 19);
  }
  return sched_getscheduler(0);
}

}  // namespace bmsched
