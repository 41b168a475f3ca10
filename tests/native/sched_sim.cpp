// sched_sim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the host-only half of libbmpow_hip.so's scheduler (pybitmessage_amd/csrc/bmpow_sched.cpp,
// the code bmpow_host.hip runs between HIP calls) against a CPU stand-in for the gfx950 kernels,
// whose trial function is the C oracle's (oracle/bmpow_oracle.c).  Built and run by
// tests/test_native.py under ThreadSanitizer and under AddressSanitizer + UBSan, with the
// concurrency the library has: one host thread per shard (device) per step, producer threads
// feeding a shared session under one mutex (the library's g_mu) while a stepper thread steps it
// and a consumer pops finished objects, and the multi-threaded payload padding of the verifier.
//
// Every answer is checked against the oracle's sequential _doSafePoW search
// (src/proofofwork.py:100-111); exit status 0 = all scenarios passed.
#include <cmath>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../pybitmessage_amd/csrc/bmpow_sched.h"

extern "C" {
uint64_t bmo_trial(const uint8_t ih[64], uint64_t nonce);
int bmo_search(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials, uint64_t* nonce_out,
               uint64_t* trial_out);
int bmo_min_trial(const uint8_t ih[64], uint64_t start, uint64_t count, uint64_t* min_out, uint64_t* argmin_out);
uint64_t bmo_trial_len(const uint8_t* ih, size_t len, uint64_t nonce);
const uint64_t* bmo_k512(void);
int bmo_search_len(const uint8_t* ih, size_t len, uint64_t target, uint64_t start, uint64_t max_trials,
                   uint64_t* nonce_out, uint64_t* trial_out);
}

using namespace bmsched;

static int g_fail = 0;
#define CHECK(cond, ...)                            \
  do {                                              \
    if (!(cond)) {                                  \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                 \
      fprintf(stderr, "\n");                        \
      ++g_fail;                                     \
    }                                               \
  } while (0)

static void ih_of(const bm_obj& o, uint8_t ih[64]) {
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) ih[8 * i + j] = (uint8_t)(o.w[i] >> (56 - 8 * j));
}

// ---- the var form's words (bmsched::pack_var) consumed the way bm_search_var_kernel does ----
static const uint64_t kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static uint64_t g_k[80];  // K[t] (init_k)
static inline uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
// 80 rounds from state h over kw[t] = K[t] + W[t]
static void rounds_kw(uint64_t h[8], const uint64_t* kw) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    const uint64_t t1 = hh + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + kw[t];
    const uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void compress_w(uint64_t h[8], const uint64_t blk[16]) {
  uint64_t w[80], kw[80];
  for (int t = 0; t < 16; ++t) w[t] = blk[t];
  for (int t = 16; t < 80; ++t)
    w[t] = (ror64(w[t - 2], 19) ^ ror64(w[t - 2], 61) ^ (w[t - 2] >> 6)) + w[t - 7] +
           (ror64(w[t - 15], 1) ^ ror64(w[t - 15], 8) ^ (w[t - 15] >> 7)) + w[t - 16];
  for (int t = 0; t < 80; ++t) kw[t] = g_k[t] + w[t];
  rounds_kw(h, kw);
}
static uint64_t trial_from_pool(const bm_obj& o, const std::vector<uint64_t>& pool, uint64_t nonce) {
  uint64_t h[8], blk[16];
  memcpy(h, kIV, sizeof h);
  for (int i = 0; i < 16; ++i) blk[i] = pool[o.vword + i];
  blk[0] = nonce;
  compress_w(h, blk);
  for (uint32_t j = 1; j < o.nblk; ++j) rounds_kw(h, &pool[o.vword + 16 + 80 * (j - 1)]);
  for (int i = 0; i < 8; ++i) blk[i] = h[i];
  blk[8] = 0x8000000000000000ULL;
  for (int i = 9; i < 15; ++i) blk[i] = 0;
  blk[15] = 512;
  memcpy(h, kIV, sizeof h);
  compress_w(h, blk);
  return h[0];
}
// K[t]: the C oracle's FIPS 180-4 table (the stand-in shares no table with the library)
static void init_k() {
  const uint64_t* k = bmo_k512();
  for (int i = 0; i < 80; ++i) g_k[i] = k[i];
}

// ---- CPU stand-in for one shard's device state and kernels ----
struct SimShard {
  std::vector<uint64_t> best;
  std::vector<uint32_t> found;
  std::vector<bm_result> res;
};

// bm_search_kernel + bm_resolve_kernel for one shard: per item, nonces in order up to the first hit
// (the device's early exit gives the same per-object minimum); res[k] = the object's shard minimum.
static uint64_t sim_trial(const bm_obj& o, const std::vector<uint64_t>& vpool, uint64_t nonce) {
  if (o.ihlen != BM_IH_MAIN) return trial_from_pool(o, vpool, nonce);
  uint8_t ih[64];
  ih_of(o, ih);
  return bmo_trial(ih, nonce);
}

// The nonces an item's workgroups hash (bmpow_layout.h): columns [g0, g0 + nwg) of gn, column c taking
// blocks c, c + gn, ... of BM_BLOCK nonces -- visited here in ascending nonce order (row by row), so
// the first hit is the item's minimum, whatever the device's early exit skips above it.
template <typename F>
static void for_each_block(const bm_item& it, F&& fn) {
  const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
  for (uint64_t row = 0;; ++row) {
    bool any = false;
    for (uint64_t c = it.g0; c < (uint64_t)it.g0 + it.nwg; ++c) {
      const uint64_t blk = row * it.gn + c;
      if (blk >= nblk) continue;
      any = true;
      const uint64_t lo = blk * BM_BLOCK, hi = std::min<uint64_t>(it.count, lo + BM_BLOCK);
      if (!fn(c - it.g0, it.start + lo, hi - lo)) return;
    }
    if (!any) return;
  }
}

static void sim_step_shard(const std::vector<bm_obj>& objs, const std::vector<uint64_t>& vpool,
                           const std::vector<bm_item>& items, SimShard& sh) {
  if (sh.best.size() < objs.size()) {
    sh.best.resize(objs.size(), kU64Max);
    sh.found.resize(objs.size(), 0);
  }
  for (const bm_item& it : items) {
    for_each_block(it, [&](uint64_t, uint64_t first, uint64_t cnt) {
      for (uint64_t j = 0; j < cnt; ++j) {
        const uint64_t n = first + j;
        if (sim_trial(objs[it.obj], vpool, n) <= objs[it.obj].target) {
          if (!sh.found[it.obj] || n < sh.best[it.obj]) sh.best[it.obj] = n;
          sh.found[it.obj] = 1;
          return false;
        }
      }
      return true;
    });
  }
  sh.res.resize(items.size());
  for (size_t k = 0; k < items.size(); ++k) {
    const uint32_t o = items[k].obj;
    bm_result r;
    r.nonce = sh.best[o];
    r.found = sh.found[o];
    r.pad = 0;
    if (r.found) {
      r.trial = sim_trial(objs[o], vpool, r.nonce);
    } else {
      r.trial = 0;
    }
    sh.res[k] = r;
  }
  // bm_resolve_kernel puts each item's object back to "no hit" after reading it
  for (const bm_item& it : items) {
    sh.best[it.obj] = kU64Max;
    sh.found[it.obj] = 0;
  }
}

// One bounded step over S shards, one host thread per shard (as one stream per device).
static bool sim_step(BatchState& b, std::vector<SimShard>& shards, uint64_t budget, uint64_t step_trials,
                     uint32_t resident = 24, const double* weights = nullptr) {
  StepPlan p;
  if (!plan_step(b, budget, step_trials, shards.size(), p, resident, weights)) return false;
  // every window's columns [0, gn) are covered exactly once over the shards' items; a window split
  // over the shards has one item per shard and a cross-shard bound slot of its own
  for (size_t wi = 0; wi < p.wins.size(); ++wi) {
    std::vector<std::pair<uint64_t, uint64_t>> cols;  // (start of the item's sub-range, column)
    for (size_t s = 0; s < shards.size(); ++s)
      for (const bm_item& it : p.items[s])
        if (it.obj == p.wins[wi].obj) {
          CHECK(it.nwg >= 1 && it.g0 + it.nwg <= it.gn && it.gn >= 1, "item columns");
          CHECK(resident == 0 || it.nwg <= resident || it.xslot != BM_NO_XSLOT, "item above the resident cap");
          for (uint32_t c = it.g0; c < it.g0 + it.nwg; ++c) cols.push_back({it.start, c});
          if (it.xslot != BM_NO_XSLOT) CHECK(it.xslot < p.nx, "xslot %u of %u", it.xslot, p.nx);
        }
    std::sort(cols.begin(), cols.end());
    CHECK(std::adjacent_find(cols.begin(), cols.end()) == cols.end(), "a column dealt twice (window %zu)", wi);
  }
  uint64_t wgs = 0, items_wg = 0;
  for (size_t s = 0; s < shards.size(); ++s) {
    wgs += p.nchunks[s];
    for (const bm_item& it : p.items[s]) items_wg += it.nwg;
  }
  CHECK(wgs == items_wg, "launch workgroups %llu != items' %llu", (unsigned long long)wgs, (unsigned long long)items_wg);
  for (size_t s = 0; s < shards.size(); ++s) {
    // two launches per shard (split_kinds): 64-byte objects, then var-form ones, chunk_base from 0 in each
    uint64_t cm = 0, cv = 0;
    for (size_t k = 0; k < p.items[s].size(); ++k) {
      const bm_item& it = p.items[s][k];
      const bool main_kind = k < p.nmain[s];
      CHECK(main_kind == (b.objs[it.obj].ihlen == BM_IH_MAIN), "item %zu of shard %zu in the wrong launch", k, s);
      uint64_t& c = main_kind ? cm : cv;
      CHECK(it.chunk_base == c, "chunk_base %u, want %llu", it.chunk_base, (unsigned long long)c);
      c += it.nwg;
    }
    CHECK(cm == p.chmain[s] && cm + cv == p.nchunks[s], "shard %zu chunk totals", s);
  }
  std::vector<std::thread> th;
  for (size_t s = 0; s < shards.size(); ++s)
    th.emplace_back(sim_step_shard, std::cref(b.objs), std::cref(b.vpool), std::cref(p.items[s]), std::ref(shards[s]));
  for (auto& t : th) t.join();
  std::vector<const bm_result*> res(shards.size());
  for (size_t s = 0; s < shards.size(); ++s) res[s] = shards[s].res.data();
  apply_step(b, p, res);
  // every slot's device state is (UINT64_MAX, 0) between steps (bmpow_host.hip relies on it: a reused
  // scratch slot is not reset)
  for (size_t s = 0; s < shards.size(); ++s)
    for (size_t i = 0; i < b.n && i < shards[s].found.size(); ++i)
      CHECK(!shards[s].found[i] && shards[s].best[i] == kU64Max, "object %zu keeps a hit on shard %zu", i, s);
  return true;
}

struct Obj {
  uint8_t ih[64];
  uint64_t target, start;
};

static std::vector<Obj> random_objs(std::mt19937_64& rng, size_t n, uint64_t max_div) {
  std::vector<Obj> v(n);
  for (auto& o : v) {
    for (auto& c : o.ih) c = (uint8_t)rng();
    o.target = kU64Max / (1 + rng() % max_div);
    o.start = 1;
  }
  return v;
}

static void expect_exact(const Obj& o, int done, uint64_t nonce, uint64_t trial, const char* what, size_t i) {
  uint64_t n = 0, t = 0;
  const uint64_t budget = kU64Max - o.start + 1 == 0 ? kU64Max : kU64Max - o.start + 1;
  const int hit = bmo_search(o.ih, o.target, o.start, budget, &n, &t);
  if (hit) {
    CHECK(done == BMPOW_DONE_FOUND && nonce == n && trial == t, "%s: object %zu: got (%d, %llu) want %llu", what, i,
          done, (unsigned long long)nonce, (unsigned long long)n);
  } else {
    CHECK(done == BMPOW_DONE_EXHAUSTED, "%s: object %zu: want EXHAUSTED, got %d", what, i, done);
  }
}

// ---- scenario 1: whole batches, many shard layouts and step sizes ----
static void scenario_batches() {
  std::mt19937_64 rng(1);
  struct Case { size_t n, S; uint64_t budget, max_div; };
  const Case cases[] = {{40, 1, 0, 3000}, {300, 3, 3001, 2000}, {2500, 2, 1 << 20, 500}, {600, 8, 1 << 14, 5000},
                        {5000, 1, 1 << 22, 200}, {17, 5, 1, 50000}};
  for (const Case& c : cases) {
    std::vector<Obj> objs = random_objs(rng, c.n, c.max_div);
    std::vector<uint8_t> ihs(64 * c.n);
    std::vector<uint64_t> tg(c.n), st(c.n);
    for (size_t i = 0; i < c.n; ++i) {
      memcpy(&ihs[64 * i], objs[i].ih, 64);
      tg[i] = objs[i].target;
      st[i] = objs[i].start;
    }
    BatchState b;
    init(b, c.n, ihs.data(), tg.data(), st.data());
    std::vector<SimShard> shards(c.S);
    int steps = 0;
    while (sim_step(b, shards, c.budget, 1 << 16)) ++steps;
    CHECK(b.pending == 0, "batch n=%zu left %zu pending", c.n, b.pending);
    for (size_t i = 0; i < c.n; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "batch", i);
    fprintf(stderr, "batches: n=%zu S=%zu budget=%llu: %d steps\n", c.n, c.S, (unsigned long long)c.budget, steps);
  }
}

// ---- scenario 1c: initialHashes of any length (the var form, pack_var + split_kinds) ----
static void scenario_var() {
  std::mt19937_64 rng(21);
  // the var pool's words, consumed as bm_search_var_kernel does, give the oracle's trial at every
  // SHA-512 block edge of the first hash's message (8 + L + 17 bytes)
  for (size_t L : std::initializer_list<size_t>{0, 1, 7, 8, 63, 65, 100, 103, 104, 111, 112, 127, 128, 200, 231, 232, 239, 240, 255, 256, 359,
                   360, 1000, 4096}) {
    std::vector<uint8_t> ih(L);
    for (auto& c : ih) c = (uint8_t)rng();
    std::vector<uint64_t> pool(3, 7);  // an object not at word 0
    bm_obj o;
    pack_var(ih.data(), L, 5, &o, pool);
    CHECK(o.ihlen == L && o.target == 5 && o.vword == 3, "pack_var header L=%zu", L);
    CHECK(pool.size() == 3 + bm_var_words(L), "pack_var words L=%zu", L);
    for (uint64_t n : std::initializer_list<uint64_t>{0, 1, 2, 1ull << 32, 0xfedcba9876543210ull, kU64Max}) {
      const uint64_t want = bmo_trial_len(ih.data(), L, n);
      CHECK(trial_from_pool(o, pool, n) == want, "var trial L=%zu n=%llu", L, (unsigned long long)n);
      CHECK(host_trial_len(ih.data(), L, n) == want, "host_trial_len L=%zu", L);
    }
  }
  // mixed batches over 1..4 shards: every answer the sequential search's
  for (size_t S : std::initializer_list<size_t>{1, 2, 4}) {
    const size_t n = 150;
    std::vector<std::vector<uint8_t>> ihs(n);
    std::vector<uint8_t> cat;
    std::vector<uint64_t> off(1, 0), tg(n);
    for (size_t i = 0; i < n; ++i) {
      const size_t L = (i % 3 == 0) ? 64 : (size_t)(rng() % 300);
      ihs[i].resize(L);
      for (auto& c : ihs[i]) c = (uint8_t)rng();
      cat.insert(cat.end(), ihs[i].begin(), ihs[i].end());
      off.push_back(cat.size());
      tg[i] = kU64Max / (1 + rng() % 3000);
    }
    BatchState b;
    init(b, n, cat.data(), tg.data(), nullptr, off.data());
    std::vector<SimShard> shards(S);
    while (sim_step(b, shards, 1 << 14, 1 << 12)) {
    }
    for (size_t i = 0; i < n; ++i) {
      uint64_t nn = 0, t = 0;
      const int hit = bmo_search_len(ihs[i].data(), ihs[i].size(), tg[i], 1, kU64Max, &nn, &t);
      CHECK(hit && b.done[i] == BMPOW_DONE_FOUND && b.nonce[i] == nn && b.trial[i] == t,
            "var batch S=%zu object %zu (L=%zu): got %llu want %llu", S, i, ihs[i].size(),
            (unsigned long long)b.nonce[i], (unsigned long long)nn);
    }
  }
  // a session: var objects added, taken, the pool emptied once no slot holds one (new epoch)
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  const uint64_t e0 = b.vpool_epoch;
  std::vector<uint8_t> ih(100, 0x5a);
  const uint64_t off[2] = {0, 100}, t1 = kU64Max / 50;
  std::vector<uint32_t> sl;
  add(b, 1, ih.data(), &t1, nullptr, sl, off);
  CHECK(b.nvar_slots == 1 && b.vpool.size() == bm_var_words(100), "session var add");
  std::vector<SimShard> shards(2);
  while (sim_step(b, shards, 1 << 13, 1 << 12)) {
  }
  uint32_t slot;
  uint64_t nn, tt;
  uint8_t dn;
  CHECK(take_done(b, 1, &slot, &nn, &tt, &dn) == 1 && dn == BMPOW_DONE_FOUND, "session var take");
  CHECK(b.nvar_slots == 0, "var slot released");
  uint64_t wn = 0, wt = 0;
  bmo_search_len(ih.data(), 100, t1, 1, kU64Max, &wn, &wt);
  CHECK(nn == wn && tt == wt, "session var answer");
  uint8_t ih64[64] = {1};
  add(b, 1, ih64, &t1, nullptr, sl);
  CHECK(b.vpool.empty() && b.vpool_epoch == e0 + 1, "var pool emptied at the next add");
  fprintf(stderr, "var: pack_var at every block edge, mixed batches over 1/2/4 shards, session pool reuse\n");
}

// ---- scenario 1b: over several shards a window is capped near the expected trials to a hit ----
static void scenario_expect_cap() {
  std::mt19937_64 rng(11);
  for (uint64_t E : {1000ull, 1000000ull, 12700000ull, 1ull << 40}) {
    std::vector<Obj> objs = random_objs(rng, 1, 1);
    objs[0].target = kU64Max / E;
    BatchState b;
    init(b, 1, objs[0].ih, &objs[0].target, &objs[0].start);
    for (size_t S : {1, 2, 8}) {
      StepPlan p;
      CHECK(plan_step(b, 0, 1 << 28, S, p), "plan_step");
      const uint64_t window = p.wins[0].chunks * p.chunk;
      const uint64_t full = ((uint64_t)1 << 28) * S;
      if (S == 1) {
        CHECK(window == full, "S=1: window %llu != budget", (unsigned long long)window);
      } else {
        const uint64_t cap = std::max<uint64_t>(S * p.chunk, (uint64_t)(kExpectWindows * (double)E));
        CHECK(window <= std::min(full, cap) + p.chunk && window >= S * p.chunk, "E=%llu S=%zu: window %llu",
              (unsigned long long)E, S, (unsigned long long)window);
      }
    }
    std::vector<SimShard> shards(8);
    if (E <= 1000000) {  // and the capped steps still give the exact answer
      while (sim_step(b, shards, 0, 1 << 16)) {
      }
      expect_exact(objs[0], b.done[0], b.nonce[0], b.trial[0], "expect_cap", 0);
    }
  }
  // as many objects as shards: object-sharded, no cap (each window a shard's whole share)
  std::vector<Obj> objs = random_objs(rng, 8, 1);
  std::vector<uint8_t> ihs(64 * 8);
  std::vector<uint64_t> tg(8), st(8, 1);
  for (size_t i = 0; i < 8; ++i) {
    memcpy(&ihs[64 * i], objs[i].ih, 64);
    tg[i] = kU64Max / 1000;
  }
  BatchState b;
  init(b, 8, ihs.data(), tg.data(), st.data());
  StepPlan p;
  plan_step(b, 0, 1 << 28, 8, p);
  for (const Win& w : p.wins)
    CHECK(w.chunks * p.chunk == ((uint64_t)1 << 28), "object-sharded window capped: %llu", (unsigned long long)w.count);
}

// ---- scenario 1d: slices weighted by the shards' measured rates (ShardRates) ----
static void scenario_weights() {
  ShardRates r;
  r.reset(3);
  std::vector<double> w;
  CHECK(!r.weights(w) && w.size() == 3 && w[0] == 1.0, "no samples: equal weights");
  r.sample(0, kRateMinTrials - 1, 1.0);  // too short a launch to measure
  CHECK(r.ema[0] == 0.0, "short launch ignored");
  r.sample(0, 1ull << 28, 40.0);
  r.sample(1, 1ull << 28, 80.0);
  CHECK(!r.weights(w), "weights need every shard sampled");
  r.sample(2, 1ull << 28, 400.0);  // 10x slower than shard 0: clamped
  CHECK(r.weights(w), "weights once every shard has a sample");
  const double mean = ((1 << 28) / 40.0 + (1 << 28) / 80.0 + (1 << 28) / 400.0) / 3;
  CHECK(std::fabs(w[0] - std::min(2.0, (1 << 28) / 40.0 / mean)) < 1e-12 && w[2] == 0.5, "clamped weights %f %f %f",
        w[0], w[1], w[2]);
  r.sample(1, 1ull << 28, 40.0);  // the average moves a quarter of the way
  CHECK(std::fabs(r.ema[1] - (0.75 * (1 << 28) / 80.0 + 0.25 * (1 << 28) / 40.0)) < 1e-6, "ema step");

  // a weighted step: each shard's chunks in proportion to its weight, and the answers still exact
  std::mt19937_64 rng(31);
  const double wt[4] = {1.0, 0.5, 2.0, 1.25};
  const size_t n = 400;
  std::vector<Obj> objs = random_objs(rng, n, 4000);
  std::vector<uint8_t> ihs(64 * n);
  std::vector<uint64_t> tg(n), st(n);
  for (size_t i = 0; i < n; ++i) {
    memcpy(&ihs[64 * i], objs[i].ih, 64);
    tg[i] = objs[i].target;
    st[i] = objs[i].start;
  }
  BatchState b;
  init(b, n, ihs.data(), tg.data(), st.data());
  StepPlan p;
  CHECK(plan_step(b, (uint64_t)1 << 22, 1 << 20, 4, p, 0, wt), "weighted plan");
  uint64_t tot = 0;
  for (size_t s = 0; s < 4; ++s) tot += p.nchunks[s];
  for (size_t s = 0; s < 4; ++s) {
    const double share = (double)p.nchunks[s] / (double)tot, want = wt[s] / 4.75;
    CHECK(std::fabs(share - want) < 0.02, "shard %zu share %.4f want %.4f", s, share, want);
  }
  std::vector<SimShard> shards(4);
  while (sim_step(b, shards, (uint64_t)1 << 16, 1 << 14, 24, wt)) {
  }
  for (size_t i = 0; i < n; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "weighted", i);
  fprintf(stderr, "weights: rate averages, clamping, weighted slices exact over 4 shards\n");
}

// ---- scenario 2: windows clipped at the top of the nonce space ----
static void scenario_top_of_space() {
  std::mt19937_64 rng(2);
  std::vector<Obj> objs = random_objs(rng, 24, 1);
  for (size_t i = 0; i < objs.size(); ++i) {
    objs[i].start = kU64Max - (i % 6) * 700;
    objs[i].target = i % 3 == 0 ? 0 : (i % 3 == 1 ? kU64Max : kU64Max / 900);
  }
  std::vector<uint8_t> ihs(64 * objs.size());
  std::vector<uint64_t> tg(objs.size()), st(objs.size());
  for (size_t i = 0; i < objs.size(); ++i) {
    memcpy(&ihs[64 * i], objs[i].ih, 64);
    tg[i] = objs[i].target;
    st[i] = objs[i].start;
  }
  for (size_t S : {1, 3}) {
    BatchState b;
    init(b, objs.size(), ihs.data(), tg.data(), st.data());
    std::vector<SimShard> shards(S);
    while (sim_step(b, shards, 1000, 1 << 16)) {
    }
    for (size_t i = 0; i < objs.size(); ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "top", i);
  }
}

// ---- scenario 3: a shared session fed by producer threads (PowService's use of the library) ----
static void scenario_session() {
  std::mutex mu;  // the library's g_mu: every entry point holds it
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  std::vector<SimShard> shards(2);
  std::vector<Obj> all;
  std::vector<int> slot_owner;                     // slot -> index into `all` (live objects)
  std::vector<std::array<uint64_t, 3>> results;  // per `all` index: done, nonce, trial
  std::atomic<int> producers_left{4};
  std::atomic<bool> stop{false};
  std::condition_variable cv;

  auto producer = [&](int id) {
    std::mt19937_64 rng(100 + id);
    for (int burst = 0; burst < 25; ++burst) {
      const size_t m = 1 + rng() % 40;
      std::vector<Obj> objs = random_objs(rng, m, 4000);
      std::vector<uint8_t> ihs(64 * m);
      std::vector<uint64_t> tg(m);
      for (size_t i = 0; i < m; ++i) {
        memcpy(&ihs[64 * i], objs[i].ih, 64);
        tg[i] = objs[i].target;
      }
      {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<uint32_t> slots;
        add(b, m, ihs.data(), tg.data(), nullptr, slots);
        b.cap = std::max(b.cap, b.n);  // the device side's reallocation
        for (SimShard& sh : shards)      // ... and its reset of the added slots' best[] / found[]
          for (uint32_t sl : slots)
            if (sl < sh.best.size()) {
              sh.best[sl] = kU64Max;
              sh.found[sl] = 0;
            }
        for (size_t i = 0; i < m; ++i) {
          if (slot_owner.size() <= slots[i]) slot_owner.resize(slots[i] + 1, -1);
          CHECK(slot_owner[slots[i]] == -1, "slot %u handed out while live", slots[i]);
          slot_owner[slots[i]] = (int)all.size();
          all.push_back(objs[i]);
          results.push_back({0, 0, 0});
        }
      }
      cv.notify_all();
      std::this_thread::sleep_for(std::chrono::microseconds(200 + rng() % 800));
    }
    producers_left--;
    cv.notify_all();
  };
  auto consumer = [&]() {
    uint32_t slot[64];
    uint64_t nonce[64], trial[64];
    uint8_t done[64];
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      // wait() (pthread_cond_wait), not wait_for: GCC 11's wait_for uses pthread_cond_clockwait,
      // which its ThreadSanitizer does not intercept (false "double lock" reports)
      cv.wait(lk, [&]() { return b.finished_head < b.finished.size() || stop.load(); });
      const size_t k = take_done(b, 64, slot, nonce, trial, done);
      for (size_t j = 0; j < k; ++j) {
        const int a = slot_owner[slot[j]];
        CHECK(a >= 0, "finished slot %u has no owner", slot[j]);
        if (a < 0) continue;
        results[a] = {done[j], nonce[j], trial[j]};
        slot_owner[slot[j]] = -1;
      }
      if (stop.load() && k == 0 && b.finished_head == b.finished.size()) return;
    }
  };
  auto stepper = [&]() {
    for (;;) {
      bool stepped;
      {
        std::lock_guard<std::mutex> lk(mu);
        stepped = sim_step(b, shards, 1 << 13, 1 << 16);
      }
      cv.notify_all();
      if (!stepped) {
        if (producers_left.load() == 0) {
          std::lock_guard<std::mutex> lk(mu);
          if (b.pending == 0) break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(300));
      }
    }
    stop.store(true);
    cv.notify_all();
  };
  std::vector<std::thread> th;
  for (int i = 0; i < 4; ++i) th.emplace_back(producer, i);
  th.emplace_back(stepper);
  th.emplace_back(consumer);
  for (auto& t : th) t.join();
  for (size_t i = 0; i < all.size(); ++i)
    expect_exact(all[i], (int)results[i][0], results[i][1], results[i][2], "session", i);
  size_t live = 0;
  for (int o : slot_owner) live += o >= 0;
  CHECK(live == 0, "%zu slots still owned after the session drained", live);
  CHECK(b.n < all.size(), "slots were not reused (%zu slots for %zu objects)", b.n, all.size());
  fprintf(stderr, "session: %zu objects through %zu slots\n", all.size(), b.n);
}

// ---- scenario 4: min-trial planning and reduction ----
static void scenario_min_trial() {
  std::mt19937_64 rng(4);
  const size_t n = 60;
  std::vector<Obj> objs = random_objs(rng, n, 1);
  std::vector<uint64_t> start(n), count(n), mn(n), arg(n);
  for (size_t i = 0; i < n; ++i) {
    start[i] = i % 7 == 0 ? kU64Max - rng() % 3000 : rng() % 100000;
    count[i] = i % 11 == 0 ? 0 : rng() % 30000;
  }
  std::vector<bm_obj> ob(n);
  for (size_t i = 0; i < n; ++i) pack_obj(objs[i].ih, 0, &ob[i]);
  for (size_t S : {1, 4}) {
    MinTrial mt;
    mt.init(n, start.data(), count.data(), mn.data(), arg.data());
    StepPlan p;
    uint64_t C = 0;
    while (mt.plan(9, p.wins, C)) {  // 9 chunks of BM_CHUNK per step: ranges span steps and shards
      slice(p.wins, C, BM_CHUNK, S, p, S == 4 ? 3 : 0);  // with and without a column cap
      std::vector<std::thread> th;
      std::vector<std::vector<bm_minpart>> parts(S);
      for (size_t s = 0; s < S; ++s)
        th.emplace_back([&, s]() {  // bm_mintrial_kernel: per chunk, the first minimum
          parts[s].assign(p.nchunks[s], bm_minpart{kU64Max, kU64Max});
          uint8_t ih[64];
          for (const bm_item& it : p.items[s]) {
            ih_of(ob[it.obj], ih);
            for_each_block(it, [&](uint64_t w, uint64_t first, uint64_t cnt) {
              bm_minpart& q = parts[s][it.chunk_base + w];
              for (uint64_t j = 0; j < cnt; ++j) {
                const uint64_t t = bmo_trial(ih, first + j);
                if (t < q.trial || (t == q.trial && first + j < q.nonce)) q = {t, first + j};
              }
              return true;
            });
          }
        });
      for (auto& t : th) t.join();
      for (size_t s = 0; s < S; ++s) mt.reduce_parts(p.items[s], parts[s].data(), mn.data(), arg.data());
      mt.advance(p.wins);
    }
    for (size_t i = 0; i < n; ++i) {
      uint64_t wm = 0, wa = 0;
      bmo_min_trial(objs[i].ih, start[i], count[i], &wm, &wa);
      CHECK(mn[i] == wm && arg[i] == wa, "min-trial object %zu (S=%zu): got (%llu, %llu) want (%llu, %llu)", i, S,
            (unsigned long long)mn[i], (unsigned long long)arg[i], (unsigned long long)wm, (unsigned long long)wa);
    }
  }
}

// ---- scenario 5: verification layout and multi-threaded padding ----
static void scenario_verify() {
  std::mt19937_64 rng(5);
  std::vector<std::vector<uint8_t>> bufs;
  const size_t lens[] = {8, 9, 16, 119, 120, 127, 128, 135, 136, 1000, 4096, 262144 + 8};
  for (int r = 0; r < 900; ++r) {
    const size_t len = r < 12 ? lens[r] : 8 + rng() % 20000;
    std::vector<uint8_t> v(len);
    for (auto& c : v) c = (uint8_t)rng();
    bufs.push_back(std::move(v));
  }
  std::vector<Span> spans;
  for (auto& v : bufs) spans.push_back({v.data(), v.size()});
  for (size_t S : {1, 3}) {
    std::vector<VPart> parts;
    uint64_t total = 0;
    CHECK(plan_verify(spans, S, parts, total) == 0, "plan_verify failed");
    uint64_t seen = 0;
    std::vector<int> hits(spans.size(), 0);
    for (VPart& pt : parts) {
      seen += pt.blocks;
      for (size_t j = 1; j < pt.ho.size(); ++j) CHECK(pt.ho[j].nblk <= pt.ho[j - 1].nblk, "not sorted by blocks");
      std::vector<uint8_t> pool(pt.blocks * 128, 0xEE);
      pad_range(spans, pt, 0, pt.orig.size(), 0, pool.data());
      for (size_t j = 0; j < pt.orig.size(); ++j) {
        const Span& sp = spans[pt.orig[j]];
        hits[pt.orig[j]]++;
        const uint64_t m = sp.len - 8, nb = padded_blocks(m);
        CHECK(pt.ho[j].nblk == nb && pt.ho[j].nonce == load_be64(sp.p), "object descriptor");
        CHECK(pt.eol[j] == (sp.len >= 16 ? load_be64(sp.p + 8) : 0), "expiresTime of object %u", pt.orig[j]);
        std::vector<uint8_t> want(nb * 128, 0);
        memcpy(want.data(), sp.p + 8, m);
        want[m] = 0x80;
        for (int k = 0; k < 8; ++k) want[nb * 128 - 1 - k] = (uint8_t)((m << 3) >> (8 * k));
        want[nb * 128 - 9] = (uint8_t)(m >> 61);
        CHECK(memcmp(want.data(), pool.data() + (uint64_t)pt.ho[j].blk * 128, nb * 128) == 0, "padding of object %u",
              pt.orig[j]);
      }
    }
    CHECK(seen == total, "blocks");
    for (int h : hits) CHECK(h == 1, "object placed %d times", h);
    // the binned verification kernel's work bins: every group in exactly one bin, longest first
    // within a bin, and LPT's bound on the most loaded bin (average + one group)
    for (VPart& pt : parts) {
      for (size_t nbins : {4, 8, 1024}) {
        plan_bins(pt, nbins);
        const size_t G = (pt.orig.size() + BV_BLOCK - 1) / BV_BLOCK;
        CHECK(pt.nbins == nbins && pt.bins.size() == nbins + 1 + G, "bins layout");
        CHECK(pt.bins[0] == 0 && pt.bins[nbins] == G, "bin offsets");
        std::vector<int> got(G, 0);
        uint64_t tot = 0, mx = 0, maxcost = 0;
        for (size_t b = 0; b < nbins; ++b) {
          uint64_t load = 0, prev = ~0ull;
          for (uint32_t i = pt.bins[b]; i < pt.bins[b + 1]; ++i) {
            const uint32_t g = pt.bins[nbins + 1 + i];
            CHECK(g < G, "group index");
            got[g]++;
            const uint64_t c = pt.ho[(size_t)g * BV_BLOCK].nblk + 2;
            for (size_t j = (size_t)g * BV_BLOCK; j < std::min(pt.orig.size(), (size_t)(g + 1) * BV_BLOCK); ++j)
              CHECK(pt.ho[j].nblk + 2 <= c, "a group's cost is its longest object");
            CHECK(c <= prev, "bin not longest first");
            prev = c;
            load += c;
            maxcost = std::max(maxcost, c);
          }
          tot += load;
          mx = std::max(mx, load);
        }
        for (int h : got) CHECK(h == 1, "group dealt %d times", h);
        CHECK(mx <= tot / nbins + maxcost, "LPT bound: %llu > %llu + %llu", (unsigned long long)mx,
              (unsigned long long)(tot / nbins), (unsigned long long)maxcost);
      }
    }
  }
}

// ---- scenario 5b: concurrent padding: several callers at once share (or fall back from) the
// persistent workers of parallel_for, each into its own staging, every byte checked ----
static void scenario_verify_concurrent() {
  std::mt19937_64 rng(9);
  std::vector<std::vector<uint8_t>> bufs;
  for (int r = 0; r < 4000; ++r) {
    std::vector<uint8_t> v(8 + rng() % 6000);
    for (auto& c : v) c = (uint8_t)rng();
    bufs.push_back(std::move(v));
  }
  std::vector<Span> spans;
  for (auto& v : bufs) spans.push_back({v.data(), v.size()});
  std::vector<std::thread> th;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int rep = 0; rep < 3; ++rep) {
        std::vector<VPart> parts;
        uint64_t total = 0;
        if (plan_verify(spans, 1 + (size_t)t % 2, parts, total) != 0) {
          bad++;
          return;
        }
        for (VPart& pt : parts) {
          std::vector<uint8_t> pool(pt.blocks * 128 + 16, 0xEE);
          pad_range(spans, pt, 0, pt.orig.size(), 0, pool.data());
          for (size_t j = 0; j < pt.orig.size(); ++j) {
            const Span& sp = spans[pt.orig[j]];
            const uint64_t m = sp.len - 8;
            const uint8_t* got = pool.data() + (uint64_t)pt.ho[j].blk * 128;
            if (memcmp(got, sp.p + 8, m) != 0 || got[m] != 0x80 || pt.ho[j].nonce != load_be64(sp.p)) bad++;
          }
        }
      }
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0, "concurrent padding: %d mismatches", bad.load());
}

// ---- scenario 6: the library's continuous-batching service (bmpow_service_*) over the stand-in ----
static void scenario_service() {
  std::mutex gmu;  // the library's g_mu: every op takes it
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  std::vector<SimShard> shards(2);
  std::atomic<int> fail_step{0}, corrupt{0};
  ServiceOps ops;
  ops.add = [&](size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* tg, uint32_t* slots,
                std::string&) {
    std::lock_guard<std::mutex> lk(gmu);
    std::vector<uint32_t> sl;
    add(b, n, ihs, tg, nullptr, sl, ih_off);
    b.cap = std::max(b.cap, b.n);
    for (SimShard& sh : shards)
      for (uint32_t x : sl)
        if (x < sh.best.size()) {
          sh.best[x] = kU64Max;
          sh.found[x] = 0;
        }
    std::copy(sl.begin(), sl.end(), slots);
    return 0;
  };
  ops.step = [&](std::string& err) {
    std::lock_guard<std::mutex> lk(gmu);
    if (fail_step.load()) {
      err = "injected step failure";
      return (int)BMPOW_E_HIP;
    }
    sim_step(b, shards, 1 << 13, 1 << 16);
    return 0;
  };
  ops.take = [&](size_t cap, uint32_t* slot, uint64_t* nonce, uint64_t* trial, uint8_t* done) {
    std::lock_guard<std::mutex> lk(gmu);
    const size_t k = take_done(b, cap, slot, nonce, trial, done);
    if (k && corrupt.exchange(0)) trial[0] ^= 1;  // a wrong device answer for the host re-check to catch
    return k;
  };
  ops.reset = [&](std::string&) {
    std::lock_guard<std::mutex> lk(gmu);
    b = BatchState();
    init(b, 0, nullptr, nullptr, nullptr);
    shards.assign(2, SimShard());
    return 0;
  };
  Service svc(ops, true);
  auto submit_objs = [&](const std::vector<Obj>& objs, std::vector<uint64_t>& tk) {
    std::vector<uint8_t> ihs(64 * objs.size());
    std::vector<uint64_t> tg(objs.size());
    for (size_t i = 0; i < objs.size(); ++i) {
      memcpy(&ihs[64 * i], objs[i].ih, 64);
      tg[i] = objs[i].target;
    }
    tk.resize(objs.size());
    return svc.submit(objs.size(), ihs.data(), tg.data(), tk.data());
  };
  uint64_t tk[64], nn[64], tv[64];
  uint8_t dn[64];
  std::string err;

  // producers and one consumer: tickets unique, every answer exact
  std::mutex tmu;
  std::vector<std::pair<uint64_t, Obj>> sent;
  size_t total = 0;
  for (int id = 0; id < 4; ++id)
    for (int burst = 0; burst < 20; ++burst) total += 1 + (id * 7 + burst * 13) % 40;
  std::vector<std::array<uint64_t, 4>> got;  // ticket, done, nonce, trial
  std::thread consumer([&] {
    while (got.size() < total) {
      const int k = svc.poll(64, -1, tk, nn, tv, dn, err);
      CHECK(k > 0, "poll returned %d (%s)", k, err.c_str());
      if (k <= 0) return;
      for (int j = 0; j < k; ++j) got.push_back({tk[j], dn[j], nn[j], tv[j]});
    }
  });
  std::vector<std::thread> prod;
  for (int id = 0; id < 4; ++id)
    prod.emplace_back([&, id] {
      std::mt19937_64 rng(300 + id);
      for (int burst = 0; burst < 20; ++burst) {
        std::vector<Obj> objs = random_objs(rng, 1 + (id * 7 + burst * 13) % 40, 4000);
        std::vector<uint64_t> t;
        std::lock_guard<std::mutex> lk(tmu);  // tickets recorded before a poll can return them
        CHECK(submit_objs(objs, t) == 0, "submit failed");
        for (size_t i = 0; i < objs.size(); ++i) sent.emplace_back(t[i], objs[i]);
      }
    });
  for (auto& t : prod) t.join();
  consumer.join();
  std::sort(sent.begin(), sent.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  std::sort(got.begin(), got.end());
  CHECK(sent.size() == total && got.size() == total, "sent %zu got %zu of %zu", sent.size(), got.size(), total);
  for (size_t i = 0; i < std::min(sent.size(), got.size()); ++i) {
    CHECK(sent[i].first == i && got[i][0] == i, "ticket %zu: sent %llu got %llu", i,
          (unsigned long long)sent[i].first, (unsigned long long)got[i][0]);
    expect_exact(sent[i].second, (int)got[i][1], got[i][2], got[i][3], "service", i);
  }
  CHECK(svc.outstanding() == 0, "outstanding %zu after draining", svc.outstanding());

  // cancel drops in-flight objects that never finish; the service goes on
  std::mt19937_64 rng(77);
  std::vector<Obj> never = random_objs(rng, 3, 1), easy = random_objs(rng, 1, 100);
  for (Obj& o : never) o.target = 0;
  std::vector<uint64_t> t;
  submit_objs(never, t);
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  svc.cancel();
  CHECK(svc.outstanding() == 0, "outstanding after cancel");
  submit_objs(easy, t);
  int k = svc.poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == 1 && tk[0] == t[0], "after cancel: k=%d", k);
  if (k == 1) expect_exact(easy[0], dn[0], nn[0], tv[0], "after cancel", 0);

  // a failing step surfaces as the poll's error; nothing steps until cancel; then it recovers
  submit_objs(never, t);
  fail_step = 1;
  k = svc.poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == BMPOW_E_HIP && err == "injected step failure", "error poll: k=%d err=%s", k, err.c_str());
  fail_step = 0;
  svc.cancel();
  submit_objs(easy, t);
  k = svc.poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == 1 && tk[0] == t[0], "after error: k=%d", k);
  if (k == 1) expect_exact(easy[0], dn[0], nn[0], tv[0], "after error", 0);

  // initialHashes of other lengths in one submit beside 64-byte ones (bmpow_service_submit_var):
  // exact answers, re-checked on the host at their own length
  {
    const size_t lens[5] = {0, 64, 5, 104, 300};
    std::vector<uint8_t> cat;
    std::vector<uint64_t> off(1, 0), tgv(5, kU64Max / 700), tkv(5);
    std::vector<std::vector<uint8_t>> ihv(5);
    for (size_t i = 0; i < 5; ++i) {
      ihv[i].resize(lens[i]);
      for (auto& c : ihv[i]) c = (uint8_t)rng();
      cat.insert(cat.end(), ihv[i].begin(), ihv[i].end());
      off.push_back(cat.size());
    }
    submit_objs(easy, t);  // a 64-byte object queued first: the queue switches to offsets
    CHECK(svc.submit(5, cat.data(), tgv.data(), tkv.data(), off.data()) == 0, "var submit");
    size_t seen = 0;
    while (seen < 6) {
      k = svc.poll(64, -1, tk, nn, tv, dn, err);
      CHECK(k > 0, "var poll %d", k);
      if (k <= 0) break;
      for (int j = 0; j < k; ++j, ++seen) {
        if (tk[j] == t[0]) {
          expect_exact(easy[0], dn[j], nn[j], tv[j], "before var", 0);
          continue;
        }
        const size_t i = tk[j] - tkv[0];
        uint64_t wn = 0, wt = 0;
        bmo_search_len(ihv[i].data(), lens[i], tgv[i], 1, kU64Max, &wn, &wt);
        CHECK(i < 5 && dn[j] == BMPOW_DONE_FOUND && nn[j] == wn && tv[j] == wt, "var service object %zu", i);
      }
    }
  }

  // the host re-check reports a wrong trial as BMPOW_DONE_BADHASH
  corrupt = 1;
  submit_objs(easy, t);
  k = svc.poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == 1 && dn[0] == BMPOW_DONE_BADHASH, "corrupted answer: k=%d done=%d", k, k > 0 ? dn[0] : -1);
  {  // ... also for an initialHash of another length
    std::vector<uint8_t> ih7(7, 3);
    const uint64_t off7[2] = {0, 7}, t7 = kU64Max / 30;
    uint64_t tk7 = 0;
    corrupt = 1;
    svc.submit(1, ih7.data(), &t7, &tk7, off7);
    k = svc.poll(64, -1, tk, nn, tv, dn, err);
    CHECK(k == 1 && tk[0] == tk7 && dn[0] == BMPOW_DONE_BADHASH, "corrupted var answer: k=%d", k);
  }
  // stop() wakes a poll blocked on an idle service
  std::thread waiter([&] {
    uint64_t a[4], b2[4], c[4];
    uint8_t d[4];
    std::string e2;
    const int r = svc.poll(4, -1, a, b2, c, d, e2);
    CHECK(r == 0, "poll woken by stop returned %d", r);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  svc.stop();
  waiter.join();
  CHECK(submit_objs(easy, t) == BMPOW_E_STATE, "submit after stop");
  fprintf(stderr, "service: %zu objects from 4 producers, cancel and error recovery\n", total);
}

int main() {
  init_k();
  scenario_batches();
  scenario_var();
  scenario_expect_cap();
  scenario_weights();
  scenario_top_of_space();
  scenario_session();
  scenario_min_trial();
  scenario_verify();
  scenario_verify_concurrent();
  scenario_service();
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  fprintf(stderr, "sched_sim: all scenarios passed\n");
  return 0;
}
