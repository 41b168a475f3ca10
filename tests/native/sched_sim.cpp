// sched_sim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Drives the host-only half of libbmpow_hip.so's scheduler (pybitmessage_amd/csrc/bmpow_sched.cpp,
// the code bmpow_host.hip runs between HIP calls) against a CPU stand-in for the gfx950 kernels,
// whose trial function is the C oracle's (oracle/bmpow_oracle.c).  Built and run by
// tests/test_native.py under ThreadSanitizer and under AddressSanitizer + UBSan, with the
// concurrency the library has: the engine's stepper thread per shard (each with a launch queued
// behind its running one, shards of unequal speed), producer threads adding objects to a session
// while those launches are in flight, a consumer popping finished objects, the service thread,
// and the multi-threaded payload padding of the verifier.
//
// Every answer is checked against the oracle's sequential _doSafePoW search
// (src/proofofwork.py:100-111); exit status 0 = all scenarios passed.
#include <cmath>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <set>
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

// The nonces an item's workgroups hash (bmpow_layout.h): columns [g0, g0 + nwg) of gn, column c taking
// blocks c, c + gn, ... of BM_BLOCK nonces -- visited here in ascending nonce order (row by row).
// (The min-trial probe's static columns.)
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

// bm_block_of (bmpow_kernels.h): the k-th block an item's queue hands out
static uint64_t block_of(const bm_item& it, uint64_t k) {
  if (it.gn == it.nwg) return k;
  const uint64_t row = k / it.nwg;
  return row * it.gn + it.g0 + (k - row * it.nwg);
}

static uint64_t sim_trial(const bm_obj& o, const std::vector<uint64_t>& vpool, uint64_t nonce) {
  if (o.ihlen != BM_IH_MAIN) return trial_from_pool(o, vpool, nonce);
  uint8_t ih[64];
  ih_of(o, ih);
  return bmo_trial(ih, nonce);
}

// ---- CPU stand-in for the devices: the engine's device side (bmsched::EngineOps) ----
// Each shard has a command queue (its stream): table uploads, slot inits and launches run in the
// order they were enqueued, by the shard's stepper when it waits for a launch.  The device state
// (the table copy, best[], found[]) persists across launches as on the GPU, and a launch emulates
// bm_search_kernel's observable behaviour: an item's blocks taken in queue order, the relay folding
// the cross-shard table into best[] before each block, the early exit at a block above best[], the
// wave's lowest hit atomicMin'd into best[] and published to every row of an xslot.
struct SimDev {
  std::vector<bm_obj> objs;
  std::vector<uint64_t> vpool;
  std::vector<uint64_t> best;
  std::vector<uint32_t> found;
};

struct SimCmd {
  enum Kind { kUpload, kSlots, kVpool, kLaunch } kind;
  std::vector<bm_obj> recs;
  std::vector<uint32_t> slots;
  std::vector<uint64_t> words;
  Launch* L = nullptr;
  std::vector<bm_item> items;
  size_t n = 0;
};

class SimLib {
 public:
  SimLib(size_t S, uint32_t resident, uint64_t step, std::vector<double> slowdown = {})
      : S_(S), dev_(S), q_(S), qmu_(S), slow_(std::move(slowdown)), xb_(new std::atomic<uint64_t>[S * BM_XSLOTS]) {
    slow_.resize(S, 1.0);
    for (size_t i = 0; i < S * BM_XSLOTS; ++i) xb_[i].store(kU64Max);
    policy_.assign(S, -2);
    EngineOps ops;
    ops.launch = [this](Launch& L, std::string&) {
      std::lock_guard<std::mutex> lk(qmu_[L.shard]);
      SimCmd c;
      c.kind = SimCmd::kLaunch;
      c.L = &L;
      c.items = L.plan.items[0];
      q_[L.shard].push_back(std::move(c));
      return 0;
    };
    ops.wait = [this](Launch& L, std::string& err) { return exec_until(L, err); };
    ops.xstore = [this](uint32_t x, uint64_t v) {
      for (size_t r = 0; r < S_; ++r) xb_[r * BM_XSLOTS + x].store(v, std::memory_order_relaxed);
    };
    ops.aborted = [this] { return abort_.load(); };
    ops.thread_init = [this](size_t s) {
      const int pol = set_thread_background("idle");
      std::lock_guard<std::mutex> lk(pmu_);
      policy_[s] = pol;
    };
    eng_.reset(new Engine(ops, S, resident, step));
  }
  ~SimLib() { eng_.reset(); }
  Engine& eng() { return *eng_; }
  std::atomic<bool> abort_{false};
  std::vector<int> policies() {
    std::lock_guard<std::mutex> lk(pmu_);
    return policy_;
  }
  // batch_upload: the whole table, best = UINT64_MAX, found = 0 (stream-ordered)
  void upload(const BatchState& b) {
    for (size_t s = 0; s < S_; ++s) {
      SimCmd c;
      c.kind = SimCmd::kUpload;
      c.recs = b.objs;
      c.words = b.vpool;
      c.n = b.n;
      std::lock_guard<std::mutex> lk(qmu_[s]);
      q_[s].push_back(std::move(c));
    }
  }
  // init_slots (bm_slots_init_kernel) and the var pool's copy, behind what is queued
  void init_slots(const BatchState& b, const std::vector<uint32_t>& slots) {
    for (size_t s = 0; s < S_; ++s) {
      SimCmd v;
      v.kind = SimCmd::kVpool;
      v.words = b.vpool;
      SimCmd c;
      c.kind = SimCmd::kSlots;
      c.slots = slots;
      for (uint32_t k : slots) c.recs.push_back(b.objs[k]);
      std::lock_guard<std::mutex> lk(qmu_[s]);
      q_[s].push_back(std::move(v));
      q_[s].push_back(std::move(c));
    }
  }
  uint64_t xb(size_t row, uint32_t x) const { return xb_[row * BM_XSLOTS + x].load(std::memory_order_relaxed); }

 private:
  int exec_until(Launch& L, std::string& err) {
    const size_t s = L.shard;
    for (;;) {
      SimCmd c;
      {
        std::lock_guard<std::mutex> lk(qmu_[s]);
        if (q_[s].empty()) {
          err = "launch not in its queue";
          return BMPOW_E_HIP;
        }
        c = std::move(q_[s].front());
        q_[s].pop_front();
      }
      SimDev& d = dev_[s];
      switch (c.kind) {
        case SimCmd::kUpload:
          d.objs = c.recs;
          d.vpool = c.words;
          d.best.assign(std::max(c.n, d.best.size()), kU64Max);
          d.found.assign(d.best.size(), 0);
          break;
        case SimCmd::kVpool:
          d.vpool = c.words;
          break;
        case SimCmd::kSlots:
          for (size_t i = 0; i < c.slots.size(); ++i) {
            const uint32_t k = c.slots[i];
            if (d.objs.size() <= k) {
              d.objs.resize(k + 1);
              d.best.resize(k + 1, kU64Max);
              d.found.resize(k + 1, 0);
            }
            d.objs[k] = c.recs[i];
            d.best[k] = kU64Max;
            d.found[k] = 0;
          }
          break;
        case SimCmd::kLaunch: {
          uint64_t trials = 0;
          std::vector<bm_result> res(c.items.size());
          const auto t0 = std::chrono::steady_clock::now();
          for (size_t k = 0; k < c.items.size(); ++k) res[k] = run_item(s, d, c.items[k], trials);
          const double slow = slow_[s];  // a shard `slow` times slower: it idles (slow - 1) x its hashing time
          if (slow > 1) std::this_thread::sleep_for((std::chrono::steady_clock::now() - t0) * (slow - 1));
          if (c.L == &L) {
            L.res = std::move(res);
            L.trials = trials;
            L.ms = std::max(1e-3, (double)trials * 1e-6);
            return 0;
          }
          err = "launches completed out of order";
          return BMPOW_E_HIP;
        }
      }
    }
  }
  bm_result run_item(size_t s, SimDev& d, const bm_item& it, uint64_t& trials) {
    const bm_obj& o = d.objs[it.obj];
    uint64_t& best = d.best[it.obj];
    uint32_t& found = d.found[it.obj];
    const uint64_t nblk = (it.count + BM_BLOCK - 1) / BM_BLOCK;
    uint64_t k = 0;
    for (;; ++k) {
      const uint64_t blk = block_of(it, k);
      if (blk >= nblk) break;
      if (it.xslot != BM_NO_XSLOT) {  // the relay folds the other shards' hits in
        const uint64_t v = xb_[s * BM_XSLOTS + it.xslot].load(std::memory_order_relaxed);
        if (v < best) best = v;
      }
      const uint64_t first = it.start + blk * BM_BLOCK;
      if (best < first) break;  // early exit above the running minimum
      const uint64_t cnt = std::min<uint64_t>(BM_BLOCK, it.count - blk * BM_BLOCK);
      trials += cnt;
      if (log_blocks_) {
        std::lock_guard<std::mutex> lk(logmu_);
        blocks_.push_back({it.obj, first, cnt});
      }
      for (uint64_t j = 0; j < cnt; ++j) {
        if (sim_trial(o, d.vpool, first + j) <= o.target) {
          const uint64_t n = first + j;
          if (n < best) best = n;
          found = 1;
          if (it.xslot != BM_NO_XSLOT)
            for (size_t r = 0; r < S_; ++r) xb_[r * BM_XSLOTS + it.xslot].store(best, std::memory_order_relaxed);
          break;  // the block's lowest hit (a wave's ctz); the next block starts above it
        }
      }
    }
    bm_result r;
    std::memset(&r, 0, sizeof r);
    r.nonce = best;
    r.found = found;
    r.trial = found ? sim_trial(o, d.vpool, best) : 0;
    // the units the item's queue handed out: the k hashed, plus one per workgroup that it took and did
    // not hash (bm_resolve_kernel's pad; the one sweep stands for the item's nwg workgroups)
    r.pad = (uint32_t)(k + it.nwg);
    items_.fetch_add(1);
    return r;
  }

 public:
  // Hashed blocks (object, first nonce, nonces), logged while log_blocks_ (the waste scenario)
  struct Blk {
    uint32_t obj;
    uint64_t first, cnt;
  };
  std::atomic<bool> log_blocks_{false};
  std::mutex logmu_;
  std::vector<Blk> blocks_;
  std::atomic<uint64_t> items_{0};  // items run

 private:
  const size_t S_;
  std::vector<SimDev> dev_;
  std::vector<std::deque<SimCmd>> q_;
  std::vector<std::mutex> qmu_;
  std::vector<double> slow_;
  std::unique_ptr<std::atomic<uint64_t>[]> xb_;
  std::mutex pmu_;
  std::vector<int> policy_;
  std::unique_ptr<Engine> eng_;
};

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

static void pack_list(const std::vector<Obj>& objs, std::vector<uint8_t>& ihs, std::vector<uint64_t>& tg,
                      std::vector<uint64_t>& st) {
  ihs.resize(64 * objs.size());
  tg.resize(objs.size());
  st.resize(objs.size());
  for (size_t i = 0; i < objs.size(); ++i) {
    memcpy(&ihs[64 * i], objs[i].ih, 64);
    tg[i] = objs[i].target;
    st[i] = objs[i].start;
  }
}

// bmpow_batch_step until nothing is pending: the steppers claim `budget` per call plus one lookahead
// launch per shard, which stays in flight across calls.  Returns the calls made.
static int solve(SimLib& lib, BatchState& b, uint64_t budget) {
  int calls = 0;
  for (;;) {
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().attach(lk, &b);
    std::string err;
    const int rc = lib.eng().run(lk, budget, true, [&b] { return b.pending == 0; }, err);
    CHECK(rc == 0, "run: %d %s", rc, err.c_str());
    ++calls;
    if (rc < 0 || b.pending == 0) return calls;
    CHECK(calls < 1000000, "no progress");
    if (calls >= 1000000) return calls;
  }
}

// ---- scenario 1: whole batches over 1..8 shards, budgets from one chunk up ----
static void scenario_batches() {
  std::mt19937_64 rng(1);
  struct Case { size_t n, S; uint64_t budget, step, max_div; };
  const Case cases[] = {{40, 1, 0, 1 << 16, 3000},      {300, 3, 3001, 1 << 14, 2000}, {2500, 2, 1 << 20, 1 << 18, 500},
                        {600, 8, 1 << 14, 1 << 13, 5000}, {5000, 1, 1 << 22, 1 << 20, 200}, {17, 5, 1, 1 << 12, 50000},
                        {7, 8, 1 << 16, 1 << 15, 20000}};
  for (const Case& c : cases) {
    std::vector<Obj> objs = random_objs(rng, c.n, c.max_div);
    std::vector<uint8_t> ihs;
    std::vector<uint64_t> tg, st;
    pack_list(objs, ihs, tg, st);
    SimLib lib(c.S, 24, c.step);
    BatchState b;
    init(b, c.n, ihs.data(), tg.data(), st.data());
    lib.upload(b);
    const int calls = solve(lib, b, c.budget ? c.budget : c.step * c.S);
    CHECK(b.pending == 0, "batch n=%zu left %zu pending", c.n, b.pending);
    for (size_t i = 0; i < c.n; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "batch", i);
    {
      std::unique_lock<std::mutex> lk(lib.eng().mu);
      lib.eng().detach(lk);
      CHECK(lib.eng().in_flight() == 0, "launches in flight after detach");
      for (size_t i = 0; i < c.n; ++i) CHECK(b.nfly[i] == 0 && b.holder[i] == kNoHolder, "object %zu still held", i);
      CHECK(lib.eng().stats.launches > 0, "no launch counted");
    }
    const double per_launch =
        (double)lib.eng().stats.planned / (double)std::max<uint64_t>(1, lib.eng().stats.launches) / (double)c.step;
    fprintf(stderr, "batches: n=%zu S=%zu budget=%llu: %d calls, %llu launches, %.2f steps planned per launch\n", c.n,
            c.S, (unsigned long long)c.budget, calls, (unsigned long long)lib.eng().stats.launches, per_launch);
    // Budgets of a step or more finish in a few calls (a shard opening windows past an answer another
    // shard had not yet reported once made this thousands, kMaxOpen), and a launch claims its whole
    // step (the remainder chunks are dealt out, not dropped).
    if (c.budget == 0 || c.budget >= (1u << 16)) CHECK(calls <= 20, "n=%zu S=%zu: %d calls", c.n, c.S, calls);
    if (c.budget == 0 && c.S == 1) CHECK(per_launch > 0.99, "n=%zu: %.2f steps per launch", c.n, per_launch);
  }
}

// ---- scenario 2: initialHashes of any length (the var form, pack_var + split_kinds) ----
static void scenario_var() {
  std::mt19937_64 rng(21);
  // the var pool's words, consumed as bm_search_var_kernel does, give the oracle's trial at every
  // SHA-512 block edge of the first hash's message (8 + L + 17 bytes)
  for (size_t L : std::initializer_list<size_t>{0, 1, 7, 8, 63, 65, 100, 103, 104, 111, 112, 127, 128, 200, 231, 232,
                                                239, 240, 255, 256, 359, 360, 1000, 4096}) {
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
    SimLib lib(S, 24, 1 << 12);
    BatchState b;
    init(b, n, cat.data(), tg.data(), nullptr, off.data());
    lib.upload(b);
    solve(lib, b, 1 << 14);
    for (size_t i = 0; i < n; ++i) {
      uint64_t nn = 0, t = 0;
      const int hit = bmo_search_len(ihs[i].data(), ihs[i].size(), tg[i], 1, kU64Max, &nn, &t);
      CHECK(hit && b.done[i] == BMPOW_DONE_FOUND && b.nonce[i] == nn && b.trial[i] == t,
            "var batch S=%zu object %zu (L=%zu): got %llu want %llu", S, i, ihs[i].size(),
            (unsigned long long)b.nonce[i], (unsigned long long)nn);
    }
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
  // a session: var objects added, taken, the pool emptied once no slot holds one (new epoch)
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  const uint64_t e0 = b.vpool_epoch;
  std::vector<uint8_t> ih(100, 0x5a);
  const uint64_t off[2] = {0, 100}, t1 = kU64Max / 50;
  std::vector<uint32_t> sl;
  SimLib lib(2, 24, 1 << 12);
  add(b, 1, ih.data(), &t1, nullptr, sl, off);
  b.cap = b.n;
  lib.upload(b);
  CHECK(b.nvar_slots == 1 && b.vpool.size() == bm_var_words(100), "session var add");
  solve(lib, b, 1 << 13);
  {
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
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

  // steady churn of var-form objects beside one that stays (parked): the pool is repacked once
  // released words outnumber live ones, so it stays bounded, and moved objects keep exact answers
  {
    BatchState c;
    init(c, 0, nullptr, nullptr, nullptr);
    c.cap = 1 << 20;
    SimLib vl(2, 16, 1 << 12);
    std::vector<uint8_t> keep(500, 0x33);  // ahead of it in the pool: a first object that finishes in round 0
    const uint64_t koff[3] = {0, 250, 500}, kt[2] = {kU64Max, kU64Max / 100};
    std::vector<uint32_t> ks;
    add(c, 2, keep.data(), kt, nullptr, ks, koff);
    ks.erase(ks.begin());
    set_pending(c, ks[0], 1, false);  // parked: its words stay live
    vl.init_slots(c, {0, 1});
    size_t max_pool = 0, compactions = 0, moved = 0;
    for (int round = 0; round < 120; ++round) {
      const size_t m = 6;
      std::vector<std::vector<uint8_t>> ihv(m);
      std::vector<uint8_t> cat;
      std::vector<uint64_t> off(1, 0), tg(m);
      for (size_t i = 0; i < m; ++i) {
        ihv[i].resize(100 + rng() % 700);
        for (auto& x : ihv[i]) x = (uint8_t)rng();
        cat.insert(cat.end(), ihv[i].begin(), ihv[i].end());
        off.push_back(cat.size());
        tg[i] = kU64Max / (1 + rng() % 400);
      }
      std::unique_lock<std::mutex> lk(vl.eng().mu);
      vl.eng().attach(lk, &c);
      const uint64_t ep = c.vpool_epoch;
      std::vector<uint32_t> slots;
      add(c, m, cat.data(), tg.data(), nullptr, slots, off.data());
      if (c.vpool_epoch != ep) ++compactions;
      if (!c.vmoved.empty()) {
        ++moved;
        vl.init_slots(c, c.vmoved);  // bmpow_host.hip: after the (drained) pool re-upload
        c.vmoved.clear();
      }
      vl.init_slots(c, slots);
      vl.eng().notify();
      std::string err;
      CHECK(vl.eng().run(lk, kU64Max, false, [&c] { return c.pending == 0; }, err) == 0, "churn run %s", err.c_str());
      uint32_t fs[8];
      uint64_t fn[8], ft[8];
      uint8_t fd[8];
      const size_t k = take_done(c, 8, fs, fn, ft, fd);
      CHECK(k == m + (round == 0), "churn round %d: %zu of %zu finished", round, k, m);
      for (size_t j = 0; j < k; ++j) {
        if (fs[j] == 0) continue;  // the first object (round 0)
        const size_t i = std::find(slots.begin(), slots.end(), fs[j]) - slots.begin();
        uint64_t wn = 0, wt = 0;
        bmo_search_len(ihv[i].data(), ihv[i].size(), tg[i], 1, kU64Max, &wn, &wt);
        CHECK(fd[j] == BMPOW_DONE_FOUND && fn[j] == wn && ft[j] == wt, "churn object answer");
      }
      max_pool = std::max(max_pool, c.vpool.size());
    }
    CHECK(compactions > 0 && moved > 0, "the pool was never repacked (%zu) or nothing moved (%zu)", compactions, moved);
    CHECK(max_pool < 2 * c.vlive + ((size_t)1 << 16) + 6 * bm_var_words(800), "var pool grew to %zu words (live %zu)",
          max_pool, c.vlive);
    // the parked object, moved by the compactions, still gives its exact answer
    {
      std::unique_lock<std::mutex> lk(vl.eng().mu);
      set_pending(c, ks[0], 1, true);
      vl.eng().notify();
      std::string err;
      vl.eng().run(lk, kU64Max, false, [&c] { return c.pending == 0; }, err);
      uint64_t wn = 0, wt = 0;
      bmo_search_len(keep.data() + 250, 250, kt[1], 1, kU64Max, &wn, &wt);
      CHECK(c.done[ks[0]] == BMPOW_DONE_FOUND && c.nonce[ks[0]] == wn && c.trial[ks[0]] == wt, "moved object answer");
      vl.eng().detach(lk);
    }
    fprintf(stderr, "var: pool churn bounded (max %zu words, %zu compactions)\n", max_pool, compactions);
  }
  fprintf(stderr, "var: pack_var at every block edge, mixed batches over 1/2/4 shards, session pool reuse\n");
}

// ---- scenario 3: fewer objects than shards -- windows split in interleaved pieces ----
static void scenario_split() {
  std::mt19937_64 rng(11);
  // planning: one object over 8 shards, every shard plans in turn -- the first window is cut into 8
  // pieces, each a shard's columns [p G, (p + 1) G) of the window's 8 G, expect_cap nonces long
  {
    std::vector<Obj> objs = random_objs(rng, 1, 1);
    const uint64_t E = 12700000;
    objs[0].target = kU64Max / E;
    BatchState b;
    init(b, 1, objs[0].ih, &objs[0].target, &objs[0].start);
    XPool xp;
    std::vector<std::pair<uint32_t, uint32_t>> cols;
    for (size_t s = 0; s < 8; ++s) {
      Launch L;
      PlanCtx c;
      c.s = s;
      c.S = 8;
      c.budget = 1 << 28;
      c.resident = 129;
      c.xp = &xp;
      CHECK(plan_launch(b, c, L), "plan shard %zu", s);
      CHECK(L.claims.size() == 1 && L.claims[0].piece == s && L.claims[0].P == 8, "shard %zu claim", s);
      const bm_item& it = L.plan.items[0][0];
      CHECK(it.start == 1 && it.count == expect_cap(objs[0].target, 8, L.plan.chunk), "split window %llu",
            (unsigned long long)it.count);
      CHECK(it.gn == 8 * it.nwg && it.g0 == s * it.nwg && it.nwg <= 128, "piece columns g0=%u nwg=%u gn=%u", it.g0,
            it.nwg, it.gn);
      CHECK(it.xslot != BM_NO_XSLOT && it.xslot == (uint32_t)b.xs[0] - 1, "split piece without a cross-shard slot");
      for (uint32_t g = it.g0; g < it.g0 + it.nwg; ++g) cols.push_back({it.gn, g});
    }
    std::sort(cols.begin(), cols.end());
    CHECK(std::adjacent_find(cols.begin(), cols.end()) == cols.end() && cols.size() == cols.back().first,
          "pieces do not cover the window's columns exactly once");
    CHECK(b.open[0].size() == 1 && b.open[0][0].claimed == 8 && b.holder[0] == kShared, "window state");
    // a ninth plan starts the next window at the frontier
    Launch L;
    PlanCtx c;
    c.S = 8;
    c.budget = 1 << 28;
    c.resident = 129;
    c.xp = &xp;
    CHECK(plan_launch(b, c, L) && L.claims[0].start == 1 + b.open[0][0].count && L.claims[0].piece == 0,
          "next window");
  }
  // exact answers for single objects over 2, 3 and 8 shards, easy to hard
  for (uint64_t E : {1000ull, 30000ull, 400000ull}) {
    for (size_t S : {2, 3, 8}) {
      std::vector<Obj> objs = random_objs(rng, 2, 1);
      objs[0].target = kU64Max / E;
      objs[1].target = kU64Max / (E / 2 + 1);
      std::vector<uint8_t> ihs;
      std::vector<uint64_t> tg, st;
      pack_list(objs, ihs, tg, st);
      SimLib lib(S, 64, 1 << 16);
      BatchState b;
      init(b, 2, ihs.data(), tg.data(), st.data());
      lib.upload(b);
      solve(lib, b, (uint64_t)S << 16);
      for (size_t i = 0; i < 2; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "split", i);
      std::unique_lock<std::mutex> lk(lib.eng().mu);
      lib.eng().detach(lk);
    }
  }
  fprintf(stderr, "split: interleaved pieces over 8 shards, exact over 2/3/8 shards\n");
}

// ---- scenario 3b: device groups -- shards sharing a device never hold one object at once ----
// Round 6: 8 shards on ONE device split tail objects into 8 pieces whose kernels raced
// each other on the same SIMDs; now the shards of a device form a group (PlanCtx::group): no split
// within a group, no object on two of its shards at once, and a split window has one piece per group.
static void scenario_groups() {
  std::mt19937_64 rng(23);
  // planning, one group of 8 shards, 3 hard objects: each of the first three shards takes one object
  // whole (P = 1), the others find nothing; the holders' staged plans take their own objects' next windows
  {
    std::vector<Obj> objs = random_objs(rng, 3, 1);
    for (Obj& o : objs) o.target = kU64Max / 50000000;
    std::vector<uint8_t> ihs;
    std::vector<uint64_t> tg, st;
    pack_list(objs, ihs, tg, st);
    BatchState b;
    init(b, 3, ihs.data(), tg.data(), st.data());
    const std::vector<uint16_t> one(8, 0);
    XPool xp;
    std::vector<uint32_t> got(8, ~0u);
    for (size_t s = 0; s < 8; ++s) {
      Launch L;
      L.shard = s;
      PlanCtx c;
      c.s = s;
      c.S = 8;
      c.group = &one;
      c.D = 1;
      c.budget = 1 << 20;
      c.resident = 1024;
      c.xp = &xp;
      const bool ok = plan_launch(b, c, L);
      if (s < 3) {
        CHECK(ok && L.claims.size() == 1 && L.claims[0].P == 1, "one group: shard %zu took %zu claims", s,
              ok ? L.claims.size() : 0);
        if (ok) got[s] = L.claims[0].obj;
        CHECK(ok && L.plan.items[0][0].xslot == BM_NO_XSLOT, "one group: an object of one shard needs no bound");
      } else {
        CHECK(!ok, "one group: shard %zu found work although every object is held by another shard", s);
      }
    }
    CHECK(got[0] != got[1] && got[1] != got[2] && got[0] != got[2], "one group: an object on two shards");
    Launch L2;
    L2.shard = 1;
    PlanCtx c;
    c.s = 1;
    c.S = 8;
    c.group = &one;
    c.D = 1;
    c.budget = 1 << 20;
    c.resident = 1024;
    c.xp = &xp;
    CHECK(plan_launch(b, c, L2) && L2.claims.size() == 1 && L2.claims[0].obj == got[1] &&
              L2.claims[0].start > b.open[got[1]][0].start,
          "one group: the holder's staged launch takes its object's next window");
  }
  // planning, two groups of three shards, one object: a window of P = 2 pieces, one per group
  {
    std::vector<Obj> objs = random_objs(rng, 1, 1);
    objs[0].target = kU64Max / 12700000;
    BatchState b;
    init(b, 1, objs[0].ih, &objs[0].target, &objs[0].start);
    const std::vector<uint16_t> two = {0, 0, 0, 1, 1, 1};
    XPool xp;
    auto plan = [&](size_t s, Launch& L) {
      L.shard = s;
      PlanCtx c;
      c.s = s;
      c.S = 6;
      c.group = &two;
      c.D = 2;
      c.budget = 1 << 28;
      c.resident = 1025;
      c.xp = &xp;
      return plan_launch(b, c, L);
    };
    Launch a, m, x;
    CHECK(plan(0, a) && a.claims[0].P == 2 && a.claims[0].piece == 0, "two groups: the first piece of two");
    CHECK(a.plan.items[0][0].count == expect_cap(objs[0].target, 2, a.plan.chunk), "two groups: a 2E window");
    CHECK(!plan(1, m), "two groups: a shard of the same device took a piece beside its mate");
    CHECK(plan(4, x) && x.claims[0].piece == 1 && x.claims[0].start == a.claims[0].start, "two groups: the other "
          "device takes the second piece");
    CHECK(x.plan.items[0][0].xslot != BM_NO_XSLOT, "two groups: a split window without its cross-shard bound");
  }
  // exact answers and the waste accounting: one group of 8 (no split: nothing past the answers but the
  // rows in flight, here none -- the stand-in's sweep stops at the next block), 2 x 3 and 3 x 2 shards
  struct Case { std::vector<uint16_t> group; size_t n; uint64_t div; };
  const Case cases[] = {{std::vector<uint16_t>(8, 0), 24, 60000},
                        {{0, 0, 0, 1, 1, 1}, 3, 150000},
                        {{0, 0, 1, 1, 2, 2}, 20, 50000},
                        {std::vector<uint16_t>(4, 0), 3, 500000}};
  for (const Case& cs : cases) {
    const size_t S = cs.group.size();
    std::vector<Obj> objs = random_objs(rng, cs.n, 1);
    for (Obj& o : objs) o.target = kU64Max / (cs.div / 2 + rng() % cs.div);
    std::vector<uint8_t> ihs;
    std::vector<uint64_t> tg, st;
    pack_list(objs, ihs, tg, st);
    std::vector<double> slow(S, 1.0);
    slow[S - 1] = 2.0;
    SimLib lib(S, 64, 1 << 16, slow);
    lib.log_blocks_ = true;
    {
      std::unique_lock<std::mutex> lk(lib.eng().mu);
      lib.eng().set_groups(lk, cs.group, 64);
    }
    BatchState b;
    init(b, cs.n, ihs.data(), tg.data(), st.data());
    lib.upload(b);
    solve(lib, b, (uint64_t)S << 16);
    for (size_t i = 0; i < cs.n; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "groups", i);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
    const WasteStats& w = lib.eng().stats.waste;
    // the truth from the stand-in's log: nonces of blocks hashed that start above the object's answer
    uint64_t past = 0;
    {
      std::lock_guard<std::mutex> g(lib.logmu_);
      for (const auto& x : lib.blocks_)
        if (x.first > b.nonce[x.obj]) past += x.cnt;
    }
    const uint64_t est = w.window + w.later + w.split, trials = lib.eng().stats.trials, items = lib.items_.load();
    CHECK(lib.eng().groups() == std::set<uint16_t>(cs.group.begin(), cs.group.end()).size(), "groups counted");
    // the estimate counts whole blocks: within one block per item of the truth
    CHECK(est >= past && est - past <= (uint64_t)BM_BLOCK * items, "groups: waste estimate %llu, truth %llu",
          (unsigned long long)est, (unsigned long long)past);
    CHECK(w.hashed >= trials && w.hashed - trials <= (uint64_t)BM_BLOCK * items,
          "groups: hashed estimate %llu against %llu trials", (unsigned long long)w.hashed, (unsigned long long)trials);
    if (lib.eng().groups() == 1) CHECK(w.split == 0, "one group: split pieces");
    fprintf(stderr, "groups: S=%zu D=%zu n=%zu exact; past the answers %llu (window %llu, later %llu, split %llu) of "
            "%llu trials\n", S, lib.eng().groups(), cs.n, (unsigned long long)past, (unsigned long long)w.window,
            (unsigned long long)w.later, (unsigned long long)w.split, (unsigned long long)trials);
  }
}

// ---- scenario 4: shards of unequal speed (one 3x slower): exact, and the others not gated ----
static void scenario_unequal() {
  std::mt19937_64 rng(41);
  for (size_t S : {1, 2, 3, 5, 8}) {
    const size_t n = 20 * S;
    std::vector<Obj> objs = random_objs(rng, n, 1);
    for (Obj& o : objs) o.target = kU64Max / (2000 + rng() % 30000);
    std::vector<uint8_t> ihs;
    std::vector<uint64_t> tg, st;
    pack_list(objs, ihs, tg, st);
    std::vector<double> slow(S, 1.0);
    slow[0] = 3.0;  // shard 0 runs 3x slower
    SimLib lib(S, 24, 1 << 14, slow);
    {
      std::lock_guard<std::mutex> lk(lib.eng().mu);
      lib.eng().rates.min_trials = 1024;  // the stand-in's launches are small: let them set the weights
    }
    BatchState b;
    init(b, n, ihs.data(), tg.data(), st.data());
    lib.upload(b);
    solve(lib, b, (uint64_t)S << 16);
    for (size_t i = 0; i < n; ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "unequal", i);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
    const EngineStats& es = lib.eng().stats;
    if (S >= 2) {
      double others = 0;
      for (size_t s = 1; s < S; ++s) others += (double)es.shard_trials[s];
      others /= (double)(S - 1);
      // not lockstep: a fast shard hashes well over the slow one's share (its fair share of the
      // objects follows its measured rate, and the others take over its objects at the end)
      CHECK(others > 1.8 * (double)es.shard_trials[0], "S=%zu: fast shards %.0f trials each, slow shard %llu", S,
            others, (unsigned long long)es.shard_trials[0]);
      fprintf(stderr, "unequal: S=%zu slow shard %llu trials, the others %.0f each\n", S,
              (unsigned long long)es.shard_trials[0], others);
    }
  }
}

// ---- scenario 5: windows clipped at the top of the nonce space ----
static void scenario_top_of_space() {
  std::mt19937_64 rng(2);
  std::vector<Obj> objs = random_objs(rng, 24, 1);
  for (size_t i = 0; i < objs.size(); ++i) {
    objs[i].start = kU64Max - (i % 6) * 700;
    objs[i].target = i % 3 == 0 ? 0 : (i % 3 == 1 ? kU64Max : kU64Max / 900);
  }
  std::vector<uint8_t> ihs;
  std::vector<uint64_t> tg, st;
  pack_list(objs, ihs, tg, st);
  for (size_t S : {1, 3, 30}) {
    SimLib lib(S, 24, 1 << 16);
    BatchState b;
    init(b, objs.size(), ihs.data(), tg.data(), st.data());
    lib.upload(b);
    solve(lib, b, 1000);
    for (size_t i = 0; i < objs.size(); ++i) expect_exact(objs[i], b.done[i], b.nonce[i], b.trial[i], "top", i);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
}

// ---- scenario 6: bounded single-object searches (bmpow_search: the scratch batch re-initialised per
// call, windows cut at the call's last nonce, the previous call's lookahead still in flight) ----
static void scenario_bounded() {
  std::mt19937_64 rng(6);
  for (size_t S : {1, 2, 4}) {
    SimLib lib(S, 16, 1 << 13);
    BatchState b;
    b.cap = 1;
    for (int obj = 0; obj < 12; ++obj) {
      std::vector<Obj> o = random_objs(rng, 1, 1);
      o[0].target = kU64Max / (20000 + rng() % 200000);
      uint64_t start = 1 + (obj % 3) * 777;
      o[0].start = start;
      const uint64_t chunk = 3000 + rng() % 40000;  // the caller's max_trials per call
      int calls = 0;
      for (;;) {
        std::unique_lock<std::mutex> lk(lib.eng().mu);
        lib.eng().attach(lk, &b);
        const size_t cap = b.cap;
        init(b, 1, o[0].ih, &o[0].target, &start);
        b.cap = cap;
        lib.init_slots(b, {0});
        b.lim[0] = start + chunk - 1;
        std::string err;
        const int rc = lib.eng().run(lk, kU64Max, false, [&b] { return b.done[0] != BMPOW_PENDING; }, err);
        CHECK(rc == 0, "bounded run %d %s", rc, err.c_str());
        ++calls;
        if (b.done[0] == BMPOW_DONE_FOUND) {
          CHECK(b.nonce[0] >= start && b.nonce[0] < start + chunk, "hit outside the call's range");
          expect_exact(o[0], b.done[0], b.nonce[0], b.trial[0], "bounded", (size_t)obj);
          break;
        }
        CHECK(b.done[0] == BMPOW_PENDING && resume_point(b, 0) == start + chunk, "NOT_FOUND resumes at %llu, want %llu",
              (unsigned long long)resume_point(b, 0), (unsigned long long)(start + chunk));
        start += chunk;
        if (calls > 2000) {
          CHECK(false, "bounded search did not finish");
          break;
        }
      }
    }
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
  fprintf(stderr, "bounded: resumed single-object searches exact over 1/2/4 shards\n");
}

// ---- scenario 7: producers feed a running session (PowService's use of the library): adds while
// launches are in flight, slots reused, a consumer popping finished objects ----
static void scenario_session() {
  std::mutex gmu;  // the library's g_mu: every entry point holds it
  const size_t S = 3;
  SimLib lib(S, 24, 1 << 13);
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  b.cap = 1 << 20;  // (no reallocation in the stand-in)
  std::vector<Obj> all;
  std::vector<int> slot_owner;                     // slot -> index into `all` (live objects)
  std::vector<std::array<uint64_t, 3>> results;  // per `all` index: done, nonce, trial
  std::atomic<int> producers_left{4};
  std::atomic<bool> stop{false};

  auto producer = [&](int id) {
    std::mt19937_64 rng(100 + id);
    for (int burst = 0; burst < 25; ++burst) {
      const size_t m = 1 + rng() % 40;
      std::vector<Obj> objs = random_objs(rng, m, 4000);
      std::vector<uint8_t> ihs;
      std::vector<uint64_t> tg, st;
      pack_list(objs, ihs, tg, st);
      {
        std::lock_guard<std::mutex> g(gmu);
        std::unique_lock<std::mutex> lk(lib.eng().mu);
        std::vector<uint32_t> slots;
        add(b, m, ihs.data(), tg.data(), nullptr, slots);
        lib.init_slots(b, slots);
        lib.eng().notify();
        for (size_t i = 0; i < m; ++i) {
          if (slot_owner.size() <= slots[i]) slot_owner.resize(slots[i] + 1, -1);
          CHECK(slot_owner[slots[i]] == -1, "slot %u handed out while live", slots[i]);
          slot_owner[slots[i]] = (int)all.size();
          all.push_back(objs[i]);
          results.push_back({0, 0, 0});
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200 + rng() % 800));
    }
    producers_left--;
  };
  auto runner = [&]() {  // the service thread: step, pop the finished objects
    uint32_t slot[64];
    uint64_t nonce[64], trial[64];
    uint8_t done[64];
    for (;;) {
      std::unique_lock<std::mutex> g(gmu);
      std::unique_lock<std::mutex> lk(lib.eng().mu);
      lib.eng().attach(lk, &b);
      std::string err;
      const int rc = lib.eng().run(lk, S << 13, true,
                                   [&] { return b.finished_head < b.finished.size() || b.pending == 0; }, err);
      CHECK(rc == 0, "session run %d %s", rc, err.c_str());
      for (;;) {
        const size_t k = take_done(b, 64, slot, nonce, trial, done);
        for (size_t j = 0; j < k; ++j) {
          const int a = slot_owner[slot[j]];
          CHECK(a >= 0, "finished slot %u has no owner", slot[j]);
          if (a < 0) continue;
          results[a] = {done[j], nonce[j], trial[j]};
          slot_owner[slot[j]] = -1;
        }
        if (k < 64) break;
      }
      const bool idle = b.pending == 0;
      if (producers_left.load() == 0 && idle && b.finished_head == b.finished.size()) break;
      if (idle) {  // let the producers in
        lk.unlock();
        g.unlock();
        std::this_thread::sleep_for(std::chrono::microseconds(300));
      }
    }
    stop.store(true);
  };
  std::vector<std::thread> th;
  for (int i = 0; i < 4; ++i) th.emplace_back(producer, i);
  th.emplace_back(runner);
  for (auto& t : th) t.join();
  {
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
  for (size_t i = 0; i < all.size(); ++i)
    expect_exact(all[i], (int)results[i][0], results[i][1], results[i][2], "session", i);
  size_t live = 0;
  for (int o : slot_owner) live += o >= 0;
  CHECK(live == 0, "%zu slots still owned after the session drained", live);
  CHECK(b.n < all.size(), "slots were not reused (%zu slots for %zu objects)", b.n, all.size());
  fprintf(stderr, "session: %zu objects through %zu slots while the steppers ran\n", all.size(), b.n);
}

// ---- scenario 7b: slot reuse while a shard is throttled ----
// Producers and a consumer churn a session's slots over 4 shards while shard 1 sleeps 2 ms before each
// of its plans.  Round 4 slept between the plan and the enqueue: a slot could be released and re-filled
// (its init queued on every stream) in between, the stale launch then ran after the init, hashed the
// NEW object over the OLD window and left a real but high hit in best[], which the new object's first
// window reported -- nonces between its frontier and that hit were never hashed.  Every answer must be
// exact, and once the session has drained no cross-shard slot may still be owned (round 4 leaked slots
// whose last carrying item completed while older items of the object were in flight).
static void scenario_session_churn() {
  std::mutex gmu;
  const size_t S = 4;
  SimLib lib(S, 24, 1 << 12);
  lib.eng().set_throttle(1, 2.0);
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  b.cap = 1 << 20;
  std::vector<Obj> all;
  std::vector<int> slot_owner;
  std::vector<std::array<uint64_t, 3>> results;
  std::atomic<int> producers_left{3};
  auto producer = [&](int id) {
    std::mt19937_64 rng(300 + id);
    for (int burst = 0; burst < 30; ++burst) {
      const size_t m = 1 + rng() % 6;
      std::vector<Obj> objs = random_objs(rng, m, 1);
      // easy and hard objects mixed: hard ones run their frontiers far up, so a stale launch of their
      // slot hashes a window well above a new easy object's first window
      for (Obj& o : objs) o.target = kU64Max / (rng() % 3 ? 200 + rng() % 3000 : 20000 + rng() % 60000);
      std::vector<uint8_t> ihs;
      std::vector<uint64_t> tg, st;
      pack_list(objs, ihs, tg, st);
      {
        std::lock_guard<std::mutex> g(gmu);
        std::unique_lock<std::mutex> lk(lib.eng().mu);
        std::vector<uint32_t> slots;
        add(b, m, ihs.data(), tg.data(), nullptr, slots);
        lib.init_slots(b, slots);
        lib.eng().notify();
        for (size_t i = 0; i < m; ++i) {
          if (slot_owner.size() <= slots[i]) slot_owner.resize(slots[i] + 1, -1);
          slot_owner[slots[i]] = (int)all.size();
          all.push_back(objs[i]);
          results.push_back({0, 0, 0});
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100 + rng() % 2000));
    }
    producers_left--;
  };
  auto runner = [&]() {
    uint32_t slot[64];
    uint64_t nonce[64], trial[64];
    uint8_t done[64];
    for (;;) {
      std::unique_lock<std::mutex> g(gmu);
      std::unique_lock<std::mutex> lk(lib.eng().mu);
      lib.eng().attach(lk, &b);
      std::string err;
      const int rc = lib.eng().run(lk, S << 12, true,
                                   [&] { return b.finished_head < b.finished.size() || b.pending == 0; }, err);
      CHECK(rc == 0, "churn run %d %s", rc, err.c_str());
      // pop (and so free for reuse) at once, while the other shards' launches are in flight
      const size_t k = take_done(b, 64, slot, nonce, trial, done);
      for (size_t j = 0; j < k; ++j) {
        const int a = slot_owner[slot[j]];
        if (a < 0) continue;
        results[a] = {done[j], nonce[j], trial[j]};
        slot_owner[slot[j]] = -1;
      }
      const bool idle = b.pending == 0;
      if (producers_left.load() == 0 && idle && b.finished_head == b.finished.size()) break;
      lk.unlock();
      g.unlock();
      if (idle) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < 3; ++i) th.emplace_back(producer, i);
  th.emplace_back(runner);
  for (auto& t : th) t.join();
  size_t owned = 0;
  {
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().drain(lk);
    owned = lib.eng().xslots_owned();
    lib.eng().detach(lk);
  }
  for (size_t i = 0; i < all.size(); ++i)
    expect_exact(all[i], (int)results[i][0], results[i][1], results[i][2], "churn", i);
  CHECK(owned == 0, "%zu cross-shard slots still owned after the session drained", owned);
  CHECK(b.n < all.size(), "slots were not reused (%zu slots for %zu objects)", b.n, all.size());
  fprintf(stderr, "session_churn: %zu objects through %zu slots, shard 1 throttled; %zu slots owned at the end\n",
          all.size(), b.n, owned);
}

// ---- scenario 8: rate averages, fair shares, the steppers' scheduling class ----
static void scenario_rates_policy() {
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

  // object mode: a shard takes its weighted fair share, its own objects first
  std::mt19937_64 rng(31);
  std::vector<Obj> objs = random_objs(rng, 400, 4000);
  std::vector<uint8_t> ihs;
  std::vector<uint64_t> tg, st;
  pack_list(objs, ihs, tg, st);
  BatchState b;
  init(b, 400, ihs.data(), tg.data(), st.data());
  Launch L0, L1, L2;
  PlanCtx c;
  c.S = 4;
  c.budget = 1 << 22;
  c.weight = 0.5;
  CHECK(plan_launch(b, c, L0) && L0.claims.size() == 50, "weight 0.5 of 400 over 4 shards: %zu", L0.claims.size());
  c.s = 1;
  c.weight = 2.0;
  CHECK(plan_launch(b, c, L1) && L1.claims.size() == 200 && L1.claims[0].obj == 50, "weight 2: %zu from %u",
        L1.claims.size(), L1.claims.empty() ? 0u : L1.claims[0].obj);
  c.s = 0;
  c.weight = 0.5;
  CHECK(plan_launch(b, c, L2) && L2.claims.size() == 50 && L2.claims[0].obj == 0 && L2.claims[0].start > 1,
        "shard 0 continues its own objects");
  // the steppers run at SCHED_IDLE, as the reference's PoW threads (bitmsghash.cpp:149)
  SimLib lib(3, 8, 1 << 12);
  {
    BatchState bb;
    init(bb, 5, ihs.data(), tg.data(), st.data());
    lib.upload(bb);
    solve(lib, bb, 1 << 14);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
  for (int p : lib.policies()) CHECK(p == SCHED_IDLE, "stepper thread policy %d, want SCHED_IDLE", p);
  fprintf(stderr, "rates: averages, clamping, weighted fair shares; steppers at SCHED_IDLE\n");
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

// ---- scenario 9: the library's continuous-batching service (bmpow_service_*) over the engine ----
static void scenario_service() {
  std::mutex gmu;  // the library's g_mu: every op takes it
  SimLib lib(2, 24, 1 << 13);
  BatchState b;
  init(b, 0, nullptr, nullptr, nullptr);
  b.cap = 1 << 20;
  std::atomic<int> fail_step{0}, corrupt{0};
  ServiceOps ops;
  ops.add = [&](size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* tg, uint32_t* slots,
                std::string&) {
    std::lock_guard<std::mutex> g(gmu);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    std::vector<uint32_t> sl;
    add(b, n, ihs, tg, nullptr, sl, ih_off);
    lib.init_slots(b, sl);
    lib.eng().notify();
    std::copy(sl.begin(), sl.end(), slots);
    return 0;
  };
  ops.step = [&](std::string& err) {
    std::lock_guard<std::mutex> g(gmu);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    if (fail_step.load()) {
      err = "injected step failure";
      return (int)BMPOW_E_HIP;
    }
    lib.eng().attach(lk, &b);
    return lib.eng().run(lk, 2 << 13, true, [&] { return b.finished_head < b.finished.size() || b.pending == 0; },
                         err);
  };
  ops.take = [&](size_t cap, uint32_t* slot, uint64_t* nonce, uint64_t* trial, uint8_t* done) {
    std::lock_guard<std::mutex> g(gmu);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    const size_t k = take_done(b, cap, slot, nonce, trial, done);
    if (k && corrupt.exchange(0)) trial[0] ^= 1;  // a wrong device answer for the host re-check to catch
    return k;
  };
  ops.reset = [&](std::string&) {
    std::lock_guard<std::mutex> g(gmu);
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
    init(b, 0, nullptr, nullptr, nullptr);
    b.cap = 1 << 20;
    lib.upload(b);
    return 0;
  };
  auto svc = std::make_unique<Service>(ops, true);
  auto submit_objs = [&](const std::vector<Obj>& objs, std::vector<uint64_t>& tk) {
    std::vector<uint8_t> ihs;
    std::vector<uint64_t> tg, st;
    pack_list(objs, ihs, tg, st);
    tk.resize(objs.size());
    return svc->submit(objs.size(), ihs.data(), tg.data(), tk.data());
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
      const int k = svc->poll(64, -1, tk, nn, tv, dn, err);
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
  CHECK(svc->outstanding() == 0, "outstanding %zu after draining", svc->outstanding());

  // cancel drops in-flight objects that never finish; the service goes on
  std::mt19937_64 rng(77);
  std::vector<Obj> never = random_objs(rng, 3, 1), easy = random_objs(rng, 1, 100);
  for (Obj& o : never) o.target = 0;
  std::vector<uint64_t> t;
  submit_objs(never, t);
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  svc->cancel();
  CHECK(svc->outstanding() == 0, "outstanding after cancel");
  submit_objs(easy, t);
  int k = svc->poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == 1 && tk[0] == t[0], "after cancel: k=%d", k);
  if (k == 1) expect_exact(easy[0], dn[0], nn[0], tv[0], "after cancel", 0);

  // a failing step surfaces as the poll's error; nothing steps until cancel; then it recovers
  submit_objs(never, t);
  fail_step = 1;
  k = svc->poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == BMPOW_E_HIP && err == "injected step failure", "error poll: k=%d err=%s", k, err.c_str());
  fail_step = 0;
  svc->cancel();
  submit_objs(easy, t);
  k = svc->poll(64, -1, tk, nn, tv, dn, err);
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
    CHECK(svc->submit(5, cat.data(), tgv.data(), tkv.data(), off.data()) == 0, "var submit");
    size_t seen = 0;
    while (seen < 6) {
      k = svc->poll(64, -1, tk, nn, tv, dn, err);
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
  k = svc->poll(64, -1, tk, nn, tv, dn, err);
  CHECK(k == 1 && dn[0] == BMPOW_DONE_BADHASH, "corrupted answer: k=%d done=%d", k, k > 0 ? dn[0] : -1);
  {  // ... also for an initialHash of another length
    std::vector<uint8_t> ih7(7, 3);
    const uint64_t off7[2] = {0, 7}, t7 = kU64Max / 30;
    uint64_t tk7 = 0;
    corrupt = 1;
    svc->submit(1, ih7.data(), &t7, &tk7, off7);
    k = svc->poll(64, -1, tk, nn, tv, dn, err);
    CHECK(k == 1 && tk[0] == tk7 && dn[0] == BMPOW_DONE_BADHASH, "corrupted var answer: k=%d", k);
  }
  // stop() wakes a poll blocked on an idle service
  std::thread waiter([&] {
    uint64_t a[4], b2[4], c[4];
    uint8_t d[4];
    std::string e2;
    const int r = svc->poll(4, -1, a, b2, c, d, e2);
    CHECK(r == 0, "poll woken by stop returned %d", r);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  svc->stop();
  waiter.join();
  CHECK(submit_objs(easy, t) == BMPOW_E_STATE, "submit after stop");
  svc.reset();
  {
    std::unique_lock<std::mutex> lk(lib.eng().mu);
    lib.eng().detach(lk);
  }
  fprintf(stderr, "service: %zu objects from 4 producers, cancel and error recovery\n", total);
}

static const char* g_only = nullptr;  // sched_sim NAME: that scenario alone

template <typename F>
static void timed(const char* name, F f) {
  if (g_only && std::strcmp(g_only, name) != 0) return;
  const auto t0 = std::chrono::steady_clock::now();
  f();
  fprintf(stderr, "  [%s: %.1f s]\n", name, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
}

int main(int argc, char** argv) {
  if (argc > 1) g_only = argv[1];
  init_k();
  timed("batches", scenario_batches);
  timed("var", scenario_var);
  timed("split", scenario_split);
  timed("groups", scenario_groups);
  timed("unequal", scenario_unequal);
  timed("top_of_space", scenario_top_of_space);
  timed("bounded", scenario_bounded);
  timed("session", scenario_session);
  timed("session_churn", scenario_session_churn);
  timed("rates_policy", scenario_rates_policy);
  timed("min_trial", scenario_min_trial);
  timed("verify", scenario_verify);
  timed("verify_concurrent", scenario_verify_concurrent);
  timed("service", scenario_service);
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  fprintf(stderr, "sched_sim: all scenarios passed\n");
  return 0;
}
