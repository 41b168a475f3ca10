// bmpow_host.hip -- C ABI (include/bmpow.h) and host scheduler of libbmpow_hip.so.
//
// Replaces the reference's native PoW entry points:
//   BitmessagePOW          src/bitmsghash/bitmsghash.cpp:127-165  (pthreads + OpenSSL)
//   do_opencl_pow/initCL   src/openclpow.py:31-111                (pyopencl window loop)
//
// Scheduler (round 4: per-device stepping, bmsched::Engine in bmpow_sched.cpp).  One stepper thread
// and stream per shard (device, or a stream of one).  Whenever a shard has fewer than two launches
// in flight, its stepper claims windows from the objects' frontiers under the engine's mutex --
// its fair share of the objects, each a window of its step's budget, or one piece each of windows
// split over every shard when fewer objects than shards are pending -- and enqueues the launch
// behind the running one: items up, bm_search_kernel (+ the var-form kernel), bm_resolve_kernel,
// results home.  When a launch completes, its per-item minima are folded into the objects (the host
// min-reduction over shards; no RCCL: no data moves between GPUs); an object is final once every
// window below its least hit has completed on whichever shard ran it.  No shard waits for another.
// The entry points (bounded searches, batch steps, the service) let the steppers claim a trial
// budget and wait for what they need, so the caller polls its shutdown flag between bounded calls
// (dev/powinterrupttest.py:22-37).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sched.h>

#include "../../include/bmpow.h"
#include "bmpow_kernels.h"
#include "bmpow_sched.h"

namespace {

constexpr uint64_t kU64Max = ~0ULL;
// Per shard per launch: ~80 ms on one MI355X, the interrupt granularity of a batch.  Against 2^28, the
// launch's tail and the host's planning between launches cost half as much: C2 6.683 / 6.679 against
// 6.668 / 6.658 GH/s, the C5 sample 6.667 / 6.674 against 6.662 / 6.664 (same box, twice each;
// 2^30 no better; profiles/r03/step_trials_ab.txt).
constexpr uint64_t kDefaultStepTrials = 1ULL << 29;

thread_local std::string g_err;
// A first-come first-served mutex.  The library's entry points take it one at a time, and the batch
// service's thread takes it for every step (up to a launch, ~80 ms) and again right after: with a plain
// std::mutex a serial run() beside a busy service waited 0.3-36 s for it -- until the batch was nearly
// done (tools/diag/run_beside_service.py, profiles/r05/run_beside_service/).  Tickets hand it out in
// arrival order, and waiting() lets a service step end at its next completed launch when a caller waits.
class FairMutex {
 public:
  void lock() {
    std::unique_lock<std::mutex> lk(m_);
    const uint64_t t = next_.fetch_add(1, std::memory_order_relaxed);
    cv_.wait(lk, [&] { return serving_.load(std::memory_order_relaxed) == t; });
  }
  void unlock() {
    {
      std::lock_guard<std::mutex> lk(m_);
      serving_.fetch_add(1, std::memory_order_relaxed);
    }
    cv_.notify_all();
  }
  // take the lock only if it comes free (no holder, no one queued) within d; false otherwise (the
  // process's exit hook: a call still running in another thread is left alone)
  bool try_lock_for(std::chrono::milliseconds d) {
    std::unique_lock<std::mutex> lk(m_);
    if (!cv_.wait_for(lk, d, [&] {
          return serving_.load(std::memory_order_relaxed) == next_.load(std::memory_order_relaxed);
        }))
      return false;
    next_.fetch_add(1, std::memory_order_relaxed);  // our ticket is the one being served
    return true;
  }
  // threads waiting for the lock (while one holds it)
  uint64_t waiting() const {
    const uint64_t n = next_.load(std::memory_order_relaxed), s = serving_.load(std::memory_order_relaxed);
    return n > s + 1 ? n - s - 1 : 0;
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> next_{0}, serving_{0};
};
FairMutex g_mu;  // one entry point at a time (the steppers never take it)
// run()'s single-object state (g_ones, g_xone, the call ring, the streams run() launches on): held by a
// 64-byte run() for its whole call -- which releases g_mu while it waits for its windows, so the batch
// service steps between them -- and by every entry point that frees or re-plans that state (device
// selection, shutdown, the split knob).  Lock order: g_one_mu, then g_mu.
std::timed_mutex g_one_mu;
std::atomic<int> g_abort{0};
std::atomic<uint64_t> g_step_trials{kDefaultStepTrials};  // read without the lock (bmpow_get_step_trials)

int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPTRY(expr)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return set_err(BMPOW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));           \
  } while (0)

// How a stepper waits for its launch (BMPOW_WAIT, read once):
//   "sleep" (default): query the launch's event and sleep between queries for 1/32 of the time waited
//     so far (20 us .. 1 ms) -- a few hundred queries per second of launch, and while two launches
//     are in flight a late wake-up costs the GPU nothing (the next launch is already queued);
//   "block": hipEventSynchronize on an event created with hipEventBlockingSync, with the device's
//     hipDeviceScheduleBlockingSync flag set (measured on MI355X: without the flag the wait spins at
//     one CPU per stepper, profiles/r04/);
//   "spin": HIP's default wait (busy); "poll": query the event every 50 us.
enum WaitMode { kWaitSleep, kWaitBlock, kWaitSpin, kWaitPoll };
WaitMode g_wait = kWaitSleep;
// run()'s single-object path (search_one): BMPOW_WAIT1 "auto" (default) spins on the result word when
// the call's answer is due within a few ms and sleeps between polls otherwise, "spin" / "sleep" force
// one (A/B); BMPOW_ONE=0 sends run() through the engine instead (A/B).
enum OneWait { kOneAuto, kOneSpin, kOneSleep };
OneWait g_one_wait = kOneAuto;
// The wait's fault check: an event recorded behind each launch, queried every g_one_query sleeping
// polls (BMPOW_ONE_QUERY=N, 0: never).  BMPOW_ONE_EVENT=0 queries the stream instead (A/B):
// hipStreamQuery cost the process 0.13 - 1.0 CPU-s per s during a 2^33 sweep, an event query 0.012
// (tools/diag/one_cpu.py, profiles/r05/one_cpu.jsonl).
int g_one_query = 8;
bool g_one_event = true;
bool g_spin_yield = true;  // BMPOW_SPIN_YIELD=0: a spinning wait never yields (A/B)
// Forced pieces that share a device each run on their own slice of its CUs (a CU-masked stream, CUs
// [j N / m, (j + 1) N / m) of the mask for piece j of m -- the mask's bits are dealt to the XCDs in turn,
// so a slice holds N / 8m CUs of every XCD): the pieces then never compete for a SIMD, as pieces on
// separate GPUs do not (tools/diag/cumask_probe.hip: 8 streams of 32 CUs each run side by side).
// BMPOW_SPLIT_CUMASK=0 shares the whole device instead (A/B).
bool g_split_cumask = true;
bool g_one_enabled = true;
// BMPOW_TRACE=1: the single-object path's set-up and tear-down steps on stderr, with the state of every
// stream they wait on (a diagnostic; tools/diag/rss_layout.py).
bool g_trace = false;
bool g_run_stream = true;  // run() on its own stream per device (run_stream); BMPOW_RUN_STREAM=0: the shard's
#define BM_TRACE(...)                                                      \
  do {                                                                     \
    if (g_trace) {                                                         \
      std::fprintf(stderr, "[bmpow %.3f] ", now_ms());                     \
      std::fprintf(stderr, __VA_ARGS__);                                   \
      std::fputc('\n', stderr);                                            \
    }                                                                      \
  } while (0)

// One of a shard's two engine launch buffers (the running launch and the one staged behind it).
struct LaunchBuf {
  bm_item* h_items = nullptr;  // pinned: items, then 2 + n counters (zeroed on the host)
  bm_item* d_items = nullptr;
  bm_result* h_res = nullptr;  // pinned: results, then the trials counter
  bm_result* d_res = nullptr;
  size_t cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evd = nullptr;  // search start / end, launch done
};

// Pinned staging of slot records for the slot-init kernel (an add while launches are in flight):
// reused once the kernel that read it has run.
struct UpBuf {
  uint8_t* h = nullptr;
  uint8_t* d = nullptr;  // the device's address of h
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};

struct Shard {
  int dev = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // per-step staging of the min-trial probe (capacity grows): its items, then its counters
  bm_item* d_items = nullptr;
  bm_result* d_res = nullptr;
  unsigned long long* d_trials = nullptr;
  unsigned long long* d_queue = nullptr;
  bm_item* h_items = nullptr;      // pinned, the same layout
  bm_result* h_res = nullptr;      // pinned
  size_t item_cap = 0;
  // step bookkeeping: items [0, nmain) / chunks [0, chmain) are 64-byte objects (bm_search_kernel),
  // the rest var-form objects (bm_search_var_kernel)
  uint32_t nitems = 0, nchunks = 0, nmain = 0, chmain = 0;
  // min-trial probe: one bm_minpart per workgroup of a launch (grow-only)
  bm_minpart* d_parts = nullptr;
  bm_minpart* h_parts = nullptr;  // pinned
  size_t parts_cap = 0;
  // the engine's launches (searches)
  LaunchBuf lb[2];
  // launch buffers outgrown while the stepper held the engine's mutex: freed by the same stepper after
  // its next wait, without the mutex (hipFree / hipHostFree wait for the device)
  std::vector<void*> retired_dev, retired_host;
  std::vector<UpBuf> up;
  double t_prev_done = 0;  // steady-clock ms when the stepper last saw a launch complete
  // address search: the fixed-base comb tables (v * 2^(W i) * G) for W = 16 ([0]) and 24 ([1]),
  // built on first use and shared by the shards of one device (owns_table marks the freeing one)
  ec::ge* d_table[2] = {nullptr, nullptr};
  bool owns_table[2] = {false, false};
  // one-shot verification (bmpow_verify_batch*, bmpow_pow_values): buffers kept across calls
  // (grow-only), so a flood pays neither allocation nor first-touch page faults; two pinned
  // staging chunks let the padding of chunk c+1 overlap the DMA of chunk c
  uint8_t* h_vstage[2] = {nullptr, nullptr};
  hipEvent_t ev_vstage[2] = {nullptr, nullptr};
  uint4* d_vpool = nullptr;
  size_t d_vpool_cap = 0;
  bv_obj* d_vobj = nullptr;
  uint64_t* d_vpow = nullptr;
  uint64_t* h_vpow = nullptr;  // pinned
  size_t vobj_cap = 0;
  uint32_t* d_vbins = nullptr;  // work bins of the binned verification kernel (grow-only)
  size_t vbins_cap = 0;
  int cus = 0;                  // compute units of the device (the binned kernel: 4 bins per CU)
  uint32_t resident = 0;        // bm_search_kernel workgroups resident on the device (occupancy x CUs)
  unsigned long long* d_xb = nullptr;  // the cross-shard bound table as this device addresses it
};

std::vector<Shard> g_shards;
// The cross-shard bound (bmpow_layout.h): BM_MAX_SHARDS rows of BM_XSLOTS words, host-pinned, coherent
// and mapped into every device; allocated with the shard set.
unsigned long long* g_xb = nullptr;
// Columns a work item may get per shard.  Shards of one device form one device group of the engine
// (bmsched::PlanCtx::group): they never hold one object at once and never split a window among
// themselves, so an item may have all of its device's resident workgroups (g_dev_resident).  Under the
// rehearsal knob (bmpow_set_engine_split: every shard its own group, as separate GPUs) the pieces of a
// split window share a device, and each gets the device's resident workgroups over the shards sharing
// it (g_resident), so every piece's sweep is on the chip at once.
uint32_t g_resident = 0, g_dev_resident = 0;
bool g_engine_split = false;
// The per-device steppers over the shard set (created with it; bmsched::Engine).
std::unique_ptr<bmsched::Engine> g_engine;
bool g_inited = false;
bmpow_stats g_stats{};

// Bytes of a step's upload for n items: the items, then 2 + n counters.
size_t stage_bytes(size_t n) { return n * sizeof(bm_item) + (2 + n) * sizeof(unsigned long long); }

// Grow the shard's item staging to hold n items.  Called while a step's item list is being
// filled, so the host items already written (s.nitems of them) move to the new buffer; the device
// copies and the results are (re)written after the fill.
int ensure_items(Shard& s, size_t n) {
  if (n <= s.item_cap) return 0;
  size_t cap = std::max<size_t>(n, 2 * s.item_cap);
  HIPTRY(hipSetDevice(s.dev));
  bm_item* h_items = nullptr;
  HIPTRY(hipHostMalloc(&h_items, stage_bytes(cap), hipHostMallocDefault));
  if (s.h_items) {
    std::memcpy(h_items, s.h_items, std::min<size_t>(s.nitems, s.item_cap) * sizeof(bm_item));
    HIPTRY(hipHostFree(s.h_items));
  }
  s.h_items = h_items;
  if (s.d_items) {
    HIPTRY(hipFree(s.d_items));
    HIPTRY(hipFree(s.d_res));
    HIPTRY(hipHostFree(s.h_res));
  }
  HIPTRY(hipMalloc(&s.d_items, stage_bytes(cap)));
  HIPTRY(hipMalloc(&s.d_res, (cap + 1) * sizeof(bm_result)));
  HIPTRY(hipHostMalloc(&s.h_res, (cap + 1) * sizeof(bm_result), hipHostMallocDefault));
  s.item_cap = cap;
  return 0;
}

// Grow an engine launch buffer to n items (only ever called for a buffer not in flight).  Called from
// engine_launch, under the engine's mutex: the old buffers are not freed here -- hipFree and hipHostFree
// wait for the whole device, every shard's launches in flight included -- but retired,
// and free_retired releases them from the stepper's wait, outside the mutex.
int ensure_launch_buf(Shard& s, LaunchBuf& lb, size_t n) {
  if (n <= lb.cap) return 0;
  const size_t cap = std::max<size_t>({n, 2 * lb.cap, 1024});
  HIPTRY(hipSetDevice(s.dev));
  if (lb.h_items) s.retired_host.push_back(lb.h_items);
  if (lb.d_items) s.retired_dev.push_back(lb.d_items);
  if (lb.h_res) s.retired_host.push_back(lb.h_res);
  if (lb.d_res) s.retired_dev.push_back(lb.d_res);
  lb.h_items = nullptr;
  lb.d_items = nullptr;
  lb.h_res = nullptr;
  lb.d_res = nullptr;
  lb.cap = 0;
  HIPTRY(hipHostMalloc(&lb.h_items, stage_bytes(cap), hipHostMallocDefault));
  HIPTRY(hipMalloc(&lb.d_items, stage_bytes(cap)));
  HIPTRY(hipHostMalloc(&lb.h_res, (cap + 1) * sizeof(bm_result), hipHostMallocDefault));
  HIPTRY(hipMalloc(&lb.d_res, (cap + 1) * sizeof(bm_result)));
  lb.cap = cap;
  return 0;
}

// Free the launch buffers the shard's stepper outgrew (ensure_launch_buf); none is in flight.
void free_retired(Shard& s) {
  for (void* p : s.retired_dev) (void)hipFree(p);
  for (void* p : s.retired_host) (void)hipHostFree(p);
  s.retired_dev.clear();
  s.retired_host.clear();
}

void free_shard(Shard& s) {
  if (s.dev < 0) return;
  (void)hipSetDevice(s.dev);
  if (s.stream) (void)hipStreamSynchronize(s.stream);
  free_retired(s);
  if (s.d_items) (void)hipFree(s.d_items);
  if (s.d_res) (void)hipFree(s.d_res);
  if (s.h_items) (void)hipHostFree(s.h_items);
  if (s.h_res) (void)hipHostFree(s.h_res);
  if (s.d_parts) (void)hipFree(s.d_parts);
  if (s.h_parts) (void)hipHostFree(s.h_parts);
  for (LaunchBuf& lb : s.lb) {
    if (lb.h_items) (void)hipHostFree(lb.h_items);
    if (lb.d_items) (void)hipFree(lb.d_items);
    if (lb.h_res) (void)hipHostFree(lb.h_res);
    if (lb.d_res) (void)hipFree(lb.d_res);
    if (lb.ev0) (void)hipEventDestroy(lb.ev0);
    if (lb.ev1) (void)hipEventDestroy(lb.ev1);
    if (lb.evd) (void)hipEventDestroy(lb.evd);
  }
  for (UpBuf& u : s.up) {
    if (u.h) (void)hipHostFree(u.h);
    if (u.ev) (void)hipEventDestroy(u.ev);
  }
  for (int c = 0; c < 2; ++c)
    if (s.d_table[c] && s.owns_table[c]) (void)hipFree(s.d_table[c]);
  for (int c = 0; c < 2; ++c) {
    if (s.h_vstage[c]) (void)hipHostFree(s.h_vstage[c]);
    if (s.ev_vstage[c]) (void)hipEventDestroy(s.ev_vstage[c]);
  }
  if (s.d_vpool) (void)hipFree(s.d_vpool);
  if (s.d_vobj) (void)hipFree(s.d_vobj);
  if (s.d_vpow) (void)hipFree(s.d_vpow);
  if (s.h_vpow) (void)hipHostFree(s.h_vpow);
  if (s.d_vbins) (void)hipFree(s.d_vbins);
  if (s.ev0) (void)hipEventDestroy(s.ev0);
  if (s.ev1) (void)hipEventDestroy(s.ev1);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = Shard();
}

int make_shard(int dev, Shard& s) {
  s.dev = dev;
  HIPTRY(hipSetDevice(dev));
  HIPTRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  HIPTRY(hipEventCreate(&s.ev0));
  HIPTRY(hipEventCreate(&s.ev1));
  for (LaunchBuf& lb : s.lb) {
    HIPTRY(hipEventCreate(&lb.ev0));
    HIPTRY(hipEventCreate(&lb.ev1));
    HIPTRY(hipEventCreateWithFlags(&lb.evd, hipEventDisableTiming |
                                                (g_wait == kWaitBlock ? hipEventBlockingSync : 0)));
  }
  HIPTRY(hipDeviceGetAttribute(&s.cus, hipDeviceAttributeMultiprocessorCount, dev));
  s.resident = (uint32_t)std::max(1, bm_search_resident_per_cu()) * (uint32_t)s.cus;
  if (const char* e = std::getenv("BMPOW_COLUMNS"))  // A/B knob: columns per shard and window
    if (std::atoi(e) > 0) s.resident = (uint32_t)std::atoi(e);
  return ensure_items(s, 1024);
}

std::vector<int> visible_gfx950() {
  std::vector<int> out;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return out;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
    if (std::strncmp(p.gcnArchName, "gfx950", 6) == 0) out.push_back(i);
  }
  return out;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- the engine's device side (bmsched::EngineOps) ----
int engine_launch(bmsched::Launch& L, std::string& err);
int engine_wait(bmsched::Launch& L, std::string& err);

void engine_xstore(uint32_t x, uint64_t v) {
  // every shard's row: the relays poll their own row (bm_relay); plain stores to coherent pinned memory
  for (size_t r = 0; r < g_shards.size(); ++r) __atomic_store_n(&g_xb[r * BM_XSLOTS + x], (unsigned long long)v, __ATOMIC_RELAXED);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
}

void make_engine() {
  bmsched::EngineOps ops;
  ops.launch = engine_launch;
  ops.wait = engine_wait;
  ops.xstore = engine_xstore;
  ops.aborted = [] { return g_abort.load() != 0; };
  ops.thread_init = [](size_t s) {
    (void)hipSetDevice(g_shards[s].dev);
    if (g_wait == kWaitBlock) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    bmsched::set_thread_background();
  };
  g_engine.reset(new bmsched::Engine(ops, g_shards.size(), g_resident, g_step_trials.load()));
  if (const char* e = std::getenv("BMPOW_THROTTLE")) {  // A/B knob "shard:ms" (the throttled-shard GPU test)
    const char* c = std::strchr(e, ':');
    if (c) g_engine->set_throttle((size_t)std::atoi(e), std::atof(c + 1));
  }
}

// Hand the engine its device groups (one per physical device, or every shard its own under
// bmpow_set_engine_split) and the matching column cap; drains what is in flight.
void apply_engine_groups() {
  if (!g_engine) return;
  std::vector<uint16_t> group;
  uint32_t resident = g_resident;
  if (!g_engine_split) {
    std::vector<int> devs;
    for (const Shard& sh : g_shards) {
      size_t g = (size_t)(std::find(devs.begin(), devs.end(), sh.dev) - devs.begin());
      if (g == devs.size()) devs.push_back(sh.dev);
      group.push_back((uint16_t)g);
    }
    resident = g_dev_resident;
  }
  std::unique_lock<std::mutex> lk(g_engine->mu);
  g_engine->set_groups(lk, group, resident);
}

void free_one();

int select_devices(const std::vector<int>& ids) {
  g_engine.reset();  // joins the steppers once their launches are applied
  free_one();
  for (auto& s : g_shards) free_shard(s);
  g_shards.clear();
  if (ids.size() > BM_MAX_SHARDS) return set_err(BMPOW_E_ARG, "more than BM_MAX_SHARDS shards");
  const auto vis = visible_gfx950();
  for (int id : ids) {
    if (std::find(vis.begin(), vis.end(), id) == vis.end())
      return set_err(BMPOW_E_ARG, "device " + std::to_string(id) + " is not a visible gfx950 device");
  }
  g_shards.resize(ids.size());
  for (size_t i = 0; i < ids.size(); ++i) {
    int rc = make_shard(ids[i], g_shards[i]);
    if (rc < 0) return rc;
  }
  if (!g_xb) {
    HIPTRY(hipHostMalloc(&g_xb, sizeof(unsigned long long) * BM_MAX_SHARDS * BM_XSLOTS,
                         hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    for (size_t i = 0; i < (size_t)BM_MAX_SHARDS * BM_XSLOTS; ++i) g_xb[i] = ~0ULL;
  }
  g_resident = ~0u;
  g_dev_resident = ~0u;
  for (auto& sh : g_shards) {
    HIPTRY(hipSetDevice(sh.dev));
    void* dp = nullptr;
    HIPTRY(hipHostGetDevicePointer(&dp, g_xb, 0));
    sh.d_xb = (unsigned long long*)dp;
    // Shards sharing a device split its resident workgroups -- over the kernels that can run at once:
    // the device's hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4) bound the streams whose
    // kernels overlap, so 8 shards on one GPU get a quarter of it each, not an eighth (an eighth left 2
    // waves per SIMD while 4 shards ran: 5.5 against 6.7 GH/s, profiles/r04/final/).
    const uint32_t same = (uint32_t)std::count_if(g_shards.begin(), g_shards.end(),
                                                  [&](const Shard& o) { return o.dev == sh.dev; });
    uint32_t hwq = 4;
    if (const char* e = std::getenv("GPU_MAX_HW_QUEUES"))
      if (std::atoi(e) > 0) hwq = (uint32_t)std::atoi(e);
    g_resident = std::min<uint32_t>(g_resident, std::max<uint32_t>(1, sh.resident / std::min(same, hwq)));
    g_dev_resident = std::min<uint32_t>(g_dev_resident, std::max<uint32_t>(1, sh.resident));
  }
  make_engine();
  apply_engine_groups();
  return (int)g_shards.size();
}

bool g_exited = false;  // bmpow_atexit ran: no stream may be created again (see g_masked)

int init_locked() {
  if (g_exited) return set_err(BMPOW_E_STATE, "the process is exiting (bmpow_atexit ran)");
  if (g_inited) return (int)g_shards.size();
  if (const char* w = std::getenv("BMPOW_WAIT"))
    g_wait = std::strcmp(w, "spin") == 0    ? kWaitSpin
             : std::strcmp(w, "poll") == 0  ? kWaitPoll
             : std::strcmp(w, "block") == 0 ? kWaitBlock
                                            : kWaitSleep;
  if (const char* w = std::getenv("BMPOW_WAIT1"))
    g_one_wait = std::strcmp(w, "spin") == 0 ? kOneSpin : std::strcmp(w, "sleep") == 0 ? kOneSleep : kOneAuto;
  if (const char* w = std::getenv("BMPOW_ONE_QUERY")) g_one_query = std::max(0, std::atoi(w));
  if (const char* w = std::getenv("BMPOW_ONE_EVENT")) g_one_event = std::atoi(w) != 0;
  if (const char* w = std::getenv("BMPOW_SPLIT_CUMASK")) g_split_cumask = std::atoi(w) != 0;
  if (const char* w = std::getenv("BMPOW_SPIN_YIELD")) g_spin_yield = std::atoi(w) != 0;
  if (const char* w = std::getenv("BMPOW_ONE")) g_one_enabled = std::atoi(w) != 0;
  if (const char* w = std::getenv("BMPOW_TRACE")) g_trace = std::atoi(w) != 0;
  if (const char* w = std::getenv("BMPOW_RUN_STREAM")) g_run_stream = std::atoi(w) != 0;
  const auto vis = visible_gfx950();
  // Release everything at exit, before the HIP runtime's own exit handlers: they were registered when
  // the runtime initialised (by the call above), and atexit runs handlers last-registered first.  Without
  // it the stepper threads were joined by g_engine's static destructor, and the streams kept for the
  // process destroyed by the runtime, after its teardown (a traced process with CU-masked streams alive
  // ended in a segfault inside the runtime's exit handlers, round 5).
  static bool hooked = false;
  if (!hooked) {
    hooked = true;
    std::atexit(bmpow_atexit);
  }
  if (vis.empty()) return set_err(BMPOW_E_NODEV, "no gfx950 (MI355X) device visible to the HIP runtime");
  std::vector<int> ids = vis;
  if (const char* e = std::getenv("BMPOW_BLOCKS_PER_WORKER"))  // A/B knob
    if (std::atoi(e) > 0) bmsched::g_blocks_per_worker = (uint32_t)std::atoi(e);
  if (const char* env = std::getenv("BMPOW_DEVICES")) {
    ids.clear();
    std::string e(env);
    size_t pos = 0;
    while (pos <= e.size()) {
      size_t c = e.find(',', pos);
      std::string tok = e.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
      if (!tok.empty()) ids.push_back(std::atoi(tok.c_str()));
      if (c == std::string::npos) break;
      pos = c + 1;
    }
    if (ids.empty()) return set_err(BMPOW_E_ARG, "BMPOW_DEVICES names no device");
  }
  int rc = select_devices(ids);
  if (rc < 0) return rc;
  g_inited = true;
  return rc;
}

using bmsched::pack_obj;

}  // namespace

// ---------------------------------------------------------------------------------------
// Batch state: the object table and per-object running minimum stay in HBM for the
// lifetime of the batch (one copy per shard).  best[]/found[] persist across launches: a launch
// queued behind another on the same stream stops at once above the hit the earlier one left there;
// a slot is reset on the device when it gets a new object (slot init, stream-ordered).
// ---------------------------------------------------------------------------------------
struct bmpow_batch : bmsched::BatchState {
  struct Dev {
    bm_obj* d_obj = nullptr;
    unsigned long long* d_best = nullptr;  // running minimum hit nonce (valid where d_found)
    uint32_t* d_found = nullptr;           // 1 once the object has a hit on this shard
    uint64_t* d_vpool = nullptr;           // copy of vpool (var-form objects' words), vcap words
  };
  std::vector<Dev> dev;  // one per shard (indexed like g_shards)
  size_t vcap = 0;         // words allocated per shard for the var pool
  size_t vsynced = 0;      // vpool words already on the devices (of epoch vepoch)
  uint64_t vepoch = ~0ULL;
};

namespace {

// The batch's launches must be finished before its device buffers change: drains the engine when
// it is working on b.
void quiesce(std::unique_lock<std::mutex>& lk, bmpow_batch* b) {
  if (g_engine && g_engine->attached() == b) g_engine->drain(lk);
}

void batch_free_dev(bmpow_batch* b) {
  for (size_t s = 0; s < b->dev.size() && s < g_shards.size(); ++s) {
    (void)hipSetDevice(g_shards[s].dev);
    (void)hipStreamSynchronize(g_shards[s].stream);
    if (b->dev[s].d_obj) (void)hipFree(b->dev[s].d_obj);
    if (b->dev[s].d_best) (void)hipFree(b->dev[s].d_best);
    if (b->dev[s].d_found) (void)hipFree(b->dev[s].d_found);
    if (b->dev[s].d_vpool) (void)hipFree(b->dev[s].d_vpool);
  }
  b->dev.clear();
  b->vcap = 0;
  b->vsynced = 0;
  b->vepoch = ~0ULL;
}

// Bring the devices' copy of the var pool up to date: the words appended since the last sync (one
// copy per shard, into words no launch reads yet), or all of them after a reallocation or a new
// epoch (bmsched::add emptied it), which first drains the batch's launches.
int sync_vpool(std::unique_lock<std::mutex>& lk, bmpow_batch* b) {
  const size_t n = b->vpool.size();
  if (b->vepoch != b->vpool_epoch) {
    b->vsynced = 0;
    b->vepoch = b->vpool_epoch;
  }
  if (n == b->vsynced) return 0;
  const bool grow = n > b->vcap;
  const size_t cap = grow ? std::max<size_t>(n, 2 * b->vcap) : b->vcap;
  const size_t from = grow ? 0 : b->vsynced;
  if (grow || from == 0) quiesce(lk, b);
  for (size_t s = 0; s < g_shards.size(); ++s) {
    Shard& sh = g_shards[s];
    HIPTRY(hipSetDevice(sh.dev));
    if (grow) {
      if (b->dev[s].d_vpool) {
        HIPTRY(hipStreamSynchronize(sh.stream));  // no launch may still read the old copy
        HIPTRY(hipFree(b->dev[s].d_vpool));
        b->dev[s].d_vpool = nullptr;
      }
      HIPTRY(hipMalloc(&b->dev[s].d_vpool, cap * sizeof(uint64_t)));
    }
    // the host vector may be appended to before an async copy ran: a synchronous copy
    HIPTRY(hipMemcpy(b->dev[s].d_vpool + from, b->vpool.data() + from, (n - from) * sizeof(uint64_t),
                     hipMemcpyHostToDevice));
  }
  b->vcap = cap;
  b->vsynced = n;
  return 0;
}

int batch_upload(std::unique_lock<std::mutex>& lk, bmpow_batch* b) {
  b->dev.assign(g_shards.size(), bmpow_batch::Dev());
  const size_t n = std::max<size_t>(b->cap, std::max<size_t>(b->n, 1));
  b->cap = n;
  for (size_t s = 0; s < g_shards.size(); ++s) {
    Shard& sh = g_shards[s];
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipMalloc(&b->dev[s].d_obj, n * sizeof(bm_obj)));
    HIPTRY(hipMalloc(&b->dev[s].d_best, n * sizeof(unsigned long long)));
    HIPTRY(hipMalloc(&b->dev[s].d_found, n * sizeof(uint32_t)));
    if (b->n) {
      HIPTRY(hipMemcpyAsync(b->dev[s].d_obj, b->objs.data(), b->n * sizeof(bm_obj), hipMemcpyHostToDevice,
                            sh.stream));
      HIPTRY(hipMemsetAsync(b->dev[s].d_best, 0xFF, b->n * sizeof(unsigned long long), sh.stream));
      HIPTRY(hipMemsetAsync(b->dev[s].d_found, 0, b->n * sizeof(uint32_t), sh.stream));
    }
  }
  for (auto& sh : g_shards) {
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipStreamSynchronize(sh.stream));
  }
  return sync_vpool(lk, b);
}

int batch_init(std::unique_lock<std::mutex>& lk, bmpow_batch* b, size_t n, const uint8_t* ihs,
               const uint64_t* targets, const uint64_t* start, const uint64_t* ih_off = nullptr) {
  bmsched::init(*b, n, ihs, targets, start, ih_off);
  return batch_upload(lk, b);
}

// Write objects into slots of the devices' tables -- the record, best = UINT64_MAX, found = 0 --
// on each shard's stream, behind whatever is in flight there (bm_slots_init_kernel reading the
// records from pinned staging).  Called under the engine's mutex, under which the steppers also plan
// AND enqueue their launches, so every launch planned for the slot's previous occupant is queued
// before this init: it hashes the old record, its results are stale by the slot's generation, and the
// init resets best[] / found[] behind it (bmsched::Engine::stepper).
int init_slots(bmpow_batch* b, const uint32_t* slots, size_t m) {
  if (m == 0) return 0;
  const size_t rec = m * sizeof(bm_obj), bytes = rec + m * sizeof(uint32_t);
  for (size_t s = 0; s < g_shards.size(); ++s) {
    Shard& sh = g_shards[s];
    HIPTRY(hipSetDevice(sh.dev));
    UpBuf* u = nullptr;
    for (UpBuf& x : sh.up) {
      if (x.pending && hipEventQuery(x.ev) == hipSuccess) x.pending = false;
      if (!x.pending && (!u || (x.cap >= bytes && u->cap < bytes))) u = &x;
    }
    if (!u) {
      sh.up.emplace_back();
      u = &sh.up.back();
      HIPTRY(hipEventCreateWithFlags(&u->ev, hipEventDisableTiming));
    }
    if (u->cap < bytes) {
      if (u->h) HIPTRY(hipHostFree(u->h));
      u->h = nullptr;
      u->cap = 0;
      const size_t cap = std::max<size_t>(bytes, 64 << 10);
      HIPTRY(hipHostMalloc(&u->h, cap, hipHostMallocMapped));
      void* dp = nullptr;
      HIPTRY(hipHostGetDevicePointer(&dp, u->h, 0));
      u->d = (uint8_t*)dp;
      u->cap = cap;
    }
    bm_obj* recs = reinterpret_cast<bm_obj*>(u->h);
    for (size_t i = 0; i < m; ++i) recs[i] = b->objs[slots[i]];
    std::memcpy(u->h + rec, slots, m * sizeof(uint32_t));
    HIPTRY(bm_launch_slots_init(sh.stream, b->dev[s].d_obj, b->dev[s].d_best, b->dev[s].d_found,
                                reinterpret_cast<const bm_obj*>(u->d), reinterpret_cast<const uint32_t*>(u->d + rec),
                                (uint32_t)m));
    HIPTRY(hipEventRecord(u->ev, sh.stream));
    u->pending = true;
  }
  return 0;
}

// Append m objects to a live session (bmsched::add: released slots first, then the table grows --
// device buffers reallocated at twice the size and re-uploaded from the host mirror, after the
// batch's launches drained).  Otherwise only the slots written go up (init_slots), behind the
// launches in flight: the steppers go on.  lk holds the engine's mutex.
int batch_add_locked(std::unique_lock<std::mutex>& lk, bmpow_batch* b, size_t m, const uint8_t* ihs,
                     const uint64_t* targets, const uint64_t* start, uint32_t* slot_out,
                     const uint64_t* ih_off = nullptr) {
  if (b->dev.size() != g_shards.size()) return set_err(BMPOW_E_STATE, "device set changed under a live batch");
  const size_t fresh = m > b->free_slots.size() ? m - b->free_slots.size() : 0;
  if (b->n + fresh > 0xffffffffULL) return set_err(BMPOW_E_ARG, "too many objects");
  if (b->n + fresh > b->cap) quiesce(lk, b);  // the tables will be reallocated
  std::vector<uint32_t> slots;
  const bool grew = bmsched::add(*b, m, ihs, targets, start, slots, ih_off);
  if (slot_out) std::copy(slots.begin(), slots.end(), slot_out);
  if (grew) {
    b->cap = std::max<size_t>({b->n, 2 * b->cap, 1024});
    batch_free_dev(b);
    const int rc = batch_upload(lk, b);
    if (g_engine) g_engine->notify();
    return rc;
  }
  int rc = sync_vpool(lk, b);  // before the slots that use the new words are handed to the steppers' kernels
  if (rc == 0 && !b->vmoved.empty()) {  // a compaction moved live objects' words (sync_vpool drained)
    rc = init_slots(b, b->vmoved.data(), b->vmoved.size());
    b->vmoved.clear();
  }
  if (rc == 0) rc = init_slots(b, slots.data(), slots.size());
  if (g_engine) g_engine->notify();
  return rc;
}

// Stage the plan's per-shard item lists in the shards' pinned buffers (sized once per step, so
// nothing written is ever reallocated under the copy): the min-trial probe's staging.
int stage_items(const bmsched::StepPlan& p) {
  for (size_t s = 0; s < g_shards.size(); ++s) {
    Shard& sh = g_shards[s];
    const std::vector<bm_item>& items = p.items[s];
    sh.nitems = 0;
    const int rc = ensure_items(sh, std::max<size_t>(items.size(), 1));
    if (rc < 0) return rc;
    if (!items.empty()) std::memcpy(sh.h_items, items.data(), items.size() * sizeof(bm_item));
    sh.nitems = (uint32_t)items.size();
    // the counters after the items, zeroed here so the step's one upload resets them
    std::memset(sh.h_items + sh.nitems, 0, (2 + (size_t)sh.nitems) * sizeof(unsigned long long));
    sh.d_trials = reinterpret_cast<unsigned long long*>(sh.d_items + sh.nitems);
    sh.d_queue = sh.d_trials + 2;
    sh.nchunks = p.nchunks[s];
    sh.nmain = p.nmain.empty() ? sh.nitems : p.nmain[s];
    sh.chmain = p.chmain.empty() ? sh.nchunks : p.chmain[s];
  }
  return 0;
}

// ---- the engine's device side ----

// Stage and enqueue one launch on its shard's stream: items and zeroed counters up (one copy), the
// search kernel(s), the resolve kernel (each item's minimum and its trial value), results home.
int engine_launch(bmsched::Launch& L, std::string& err) {
  Shard& sh = g_shards[L.shard];
  LaunchBuf& lb = sh.lb[L.buf];
  bmpow_batch* b = static_cast<bmpow_batch*>(L.batch);
  const std::vector<bm_item>& items = L.plan.items[0];
  const size_t n = items.size();
  int rc = ensure_launch_buf(sh, lb, std::max<size_t>(n, 1));
  if (rc < 0) {
    err = g_err;
    return rc;
  }
  std::memcpy(lb.h_items, items.data(), n * sizeof(bm_item));
  std::memset(lb.h_items + n, 0, (2 + n) * sizeof(unsigned long long));
  unsigned long long* d_trials = reinterpret_cast<unsigned long long*>(lb.d_items + n);
  unsigned long long* d_queue = d_trials + 2;
  const uint32_t nmain = L.plan.nmain.empty() ? (uint32_t)n : L.plan.nmain[0];
  const uint32_t nch = L.plan.nchunks[0];
  const uint32_t chmain = L.plan.chmain.empty() ? nch : L.plan.chmain[0];
  const bmpow_batch::Dev& d = b->dev[L.shard];
  bm_xbound xb;
  if (L.plan.nx) {
    xb.table = sh.d_xb;
    xb.row = (uint32_t)L.shard;
    xb.rows = (uint32_t)g_shards.size();
  }
  hipError_t e = hipSetDevice(sh.dev);
  if (e == hipSuccess)
    e = hipMemcpyAsync(lb.d_items, lb.h_items, stage_bytes(n), hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = hipEventRecord(lb.ev0, sh.stream);
  if (e == hipSuccess && nmain)
    e = bm_launch_search(sh.stream, chmain, d.d_obj, lb.d_items, nmain, d.d_best, d.d_found, d_trials, d_queue, xb);
  if (e == hipSuccess && n > nmain && nmain && xb.table)  // the var launch's relay counts its own columns
    e = hipMemsetAsync(d_trials + 1, 0, sizeof(unsigned long long), sh.stream);
  if (e == hipSuccess && n > nmain)
    e = bm_launch_search_var(sh.stream, nch - chmain, d.d_obj, lb.d_items + nmain, (uint32_t)n - nmain, d.d_best,
                             d.d_found, d_trials, d_queue + nmain, xb, d.d_vpool);
  if (e == hipSuccess) e = hipEventRecord(lb.ev1, sh.stream);
  if (e == hipSuccess)
    e = bm_launch_resolve(sh.stream, d.d_obj, lb.d_items, (uint32_t)n, d.d_best, d.d_found, lb.d_res, d.d_vpool,
                          d_trials);
  if (e == hipSuccess)
    e = hipMemcpyAsync(lb.h_res, lb.d_res, (n + 1) * sizeof(bm_result), hipMemcpyDeviceToHost, sh.stream);
  if (e == hipSuccess) e = hipEventRecord(lb.evd, sh.stream);
  if (e != hipSuccess) {
    err = std::string("search launch: ") + hipGetErrorString(e);
    return BMPOW_E_HIP;
  }
  return 0;
}

int engine_wait(bmsched::Launch& L, std::string& err) {
  Shard& sh = g_shards[L.shard];
  LaunchBuf& lb = sh.lb[L.buf];
  hipError_t e = hipSetDevice(sh.dev);
  if (e == hipSuccess) {
    if (g_wait == kWaitSleep) {
      const auto t0 = std::chrono::steady_clock::now();
      while ((e = hipEventQuery(lb.evd)) == hipErrorNotReady) {
        const int64_t waited = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
        std::this_thread::sleep_for(std::chrono::microseconds(std::min<int64_t>(1000, std::max<int64_t>(20, waited / 32))));
      }
    } else if (g_wait == kWaitPoll) {
      while ((e = hipEventQuery(lb.evd)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(50));
    } else {
      e = hipEventSynchronize(lb.evd);
    }
  }
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, lb.ev0, lb.ev1);
  if (e != hipSuccess) {
    err = std::string("search wait: ") + hipGetErrorString(e);
    return BMPOW_E_HIP;
  }
  sh.t_prev_done = now_ms();
  const size_t n = L.plan.items[0].size();
  L.res.assign(lb.h_res, lb.h_res + n);
  if (!sh.retired_dev.empty() || !sh.retired_host.empty()) free_retired(sh);
  L.trials = lb.h_res[n].nonce;  // the trials counter rides home after the results
  L.ms = ms;
  return 0;
}

int ensure_parts(Shard& s, size_t n) {
  if (n <= s.parts_cap) return 0;
  const size_t cap = std::max<size_t>(n, 2 * s.parts_cap);
  HIPTRY(hipSetDevice(s.dev));
  if (s.d_parts) HIPTRY(hipFree(s.d_parts));
  if (s.h_parts) HIPTRY(hipHostFree(s.h_parts));
  s.d_parts = nullptr;
  s.h_parts = nullptr;
  s.parts_cap = 0;
  HIPTRY(hipMalloc(&s.d_parts, cap * sizeof(bm_minpart)));
  HIPTRY(hipHostMalloc(&s.h_parts, cap * sizeof(bm_minpart), hipHostMallocDefault));
  s.parts_cap = cap;
  return 0;
}

// Min-trial probe over n (object, range) pairs: min_out[i] = min{trial(m) : m in [start[i],
// start[i] + count[i])} (clipped at 2^64-1) and argmin_out[i] = the first such m reaching it.
// Steps of ~g_step_trials per shard; ranges are covered in ascending order, cut over the shards
// like a search step, and each workgroup's (trial, nonce) minimum is reduced here,
// lexicographically, so ties keep the smaller nonce.
int min_trial_locked(size_t n, const uint8_t* ihs, const uint64_t* start, const uint64_t* count, uint64_t* min_out,
                     uint64_t* argmin_out, const uint64_t* ih_off = nullptr) {
  if (n > 0xffffffffULL) return set_err(BMPOW_E_ARG, "too many objects");
  const size_t S = g_shards.size();
  std::vector<bm_obj> objs(n);
  std::vector<uint64_t> vpool;
  bool any_var = false;
  for (size_t i = 0; i < n; ++i) {
    bmsched::pack_var(bmsched::ih_ptr(ihs, ih_off, i), bmsched::ih_len(ih_off, i), 0, &objs[i], vpool);
    any_var = any_var || objs[i].ihlen != BM_IH_MAIN;
  }
  bmsched::MinTrial mt;
  mt.init(n, start, count, min_out, argmin_out);
  std::vector<bm_obj*> d_obj(S, nullptr);
  std::vector<uint64_t*> d_vpool(S, nullptr);
  auto release = [&]() {
    for (size_t s = 0; s < S; ++s) {
      if (d_obj[s] || d_vpool[s]) (void)hipSetDevice(g_shards[s].dev);
      if (d_obj[s]) (void)hipFree(d_obj[s]);
      if (d_vpool[s]) (void)hipFree(d_vpool[s]);
    }
  };
  int rc = 0;
  for (size_t s = 0; s < S && rc == 0; ++s) {
    Shard& sh = g_shards[s];
    hipError_t e = hipSetDevice(sh.dev);
    if (e == hipSuccess) e = hipMalloc(&d_obj[s], std::max<size_t>(n, 1) * sizeof(bm_obj));
    if (e == hipSuccess && n)
      e = hipMemcpyAsync(d_obj[s], objs.data(), n * sizeof(bm_obj), hipMemcpyHostToDevice, sh.stream);
    if (e == hipSuccess && !vpool.empty()) e = hipMalloc(&d_vpool[s], vpool.size() * sizeof(uint64_t));
    if (e == hipSuccess && !vpool.empty())
      e = hipMemcpyAsync(d_vpool[s], vpool.data(), vpool.size() * sizeof(uint64_t), hipMemcpyHostToDevice, sh.stream);
    if (e != hipSuccess) rc = set_err(BMPOW_E_HIP, std::string("min-trial upload: ") + hipGetErrorString(e));
  }
  const uint64_t total_chunks = std::max<uint64_t>(g_step_trials * S / BM_CHUNK, S);
  bmsched::StepPlan plan;
  while (rc == 0) {
    if (g_abort.load()) {
      rc = set_err(BMPOW_E_ABORTED, "aborted");
      break;
    }
    uint64_t C = 0;
    if (!mt.plan(total_chunks, plan.wins, C)) break;
    bmsched::slice(plan.wins, C, BM_CHUNK, S, plan);
    bmsched::split_kinds(objs, any_var, plan);
    rc = stage_items(plan);
    if (rc < 0) break;
    for (size_t s = 0; s < S && rc == 0; ++s) {
      Shard& sh = g_shards[s];
      if (sh.nitems == 0) continue;
      rc = ensure_parts(sh, sh.nchunks);
      if (rc < 0) break;
      hipError_t e = hipSetDevice(sh.dev);
      if (e == hipSuccess)
        e = hipMemcpyAsync(sh.d_items, sh.h_items, sh.nitems * sizeof(bm_item), hipMemcpyHostToDevice, sh.stream);
      if (e == hipSuccess) e = hipEventRecord(sh.ev0, sh.stream);
      if (e == hipSuccess && sh.nmain)
        e = bm_launch_mintrial(sh.stream, sh.chmain, d_obj[s], sh.d_items, sh.nmain, sh.d_parts);
      if (e == hipSuccess && sh.nitems > sh.nmain)
        e = bm_launch_mintrial_var(sh.stream, sh.nchunks - sh.chmain, d_obj[s], sh.d_items + sh.nmain,
                                   sh.nitems - sh.nmain, sh.d_parts + sh.chmain, d_vpool[s]);
      if (e == hipSuccess) e = hipEventRecord(sh.ev1, sh.stream);
      if (e == hipSuccess)
        e = hipMemcpyAsync(sh.h_parts, sh.d_parts, sh.nchunks * sizeof(bm_minpart), hipMemcpyDeviceToHost,
                           sh.stream);
      if (e != hipSuccess) rc = set_err(BMPOW_E_HIP, std::string("min-trial launch: ") + hipGetErrorString(e));
    }
    for (size_t s = 0; s < S && rc == 0; ++s) {
      Shard& sh = g_shards[s];
      if (sh.nitems == 0) continue;
      hipError_t e = hipSetDevice(sh.dev);
      if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
      float ms = 0;
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, sh.ev0, sh.ev1);
      if (e != hipSuccess) {
        rc = set_err(BMPOW_E_HIP, std::string("min-trial: ") + hipGetErrorString(e));
        break;
      }
      g_stats.probe_kernel_ms += ms;
      const std::vector<bm_item>& its = plan.items[s];
      const std::vector<bm_item> main_items(its.begin(), its.begin() + sh.nmain),
          var_items(its.begin() + sh.nmain, its.end());
      mt.reduce_parts(main_items, sh.h_parts, min_out, argmin_out);
      if (!var_items.empty()) mt.reduce_parts(var_items, sh.h_parts + sh.chmain, min_out, argmin_out);
    }
    if (rc < 0) break;
    for (const bmsched::Win& w : plan.wins) g_stats.probe_trials += w.count;
    mt.advance(plan.wins);
  }
  release();
  return rc;
}


// Library-owned scratch batch reused by the stateless entry points (bmpow_search*, bmpow_search_batch).
bmpow_batch* g_scratch = nullptr;

// Re-initialise the scratch batch with n objects and attach it.  Reused while it is large enough and
// the device set is unchanged: a run() call then writes its 128-B record into slot 0 behind whatever
// is still in flight there (the previous call's lookahead launch, which stops at once on that call's
// hit; its results are stale by the slot's generation), with no allocation and no host wait.
int scratch_batch(std::unique_lock<std::mutex>& lk, size_t n, const uint8_t* ihs, const uint64_t* targets,
                  const uint64_t* start, const uint64_t* ih_off = nullptr) {
  if (g_scratch && g_scratch->dev.size() == g_shards.size() && g_scratch->cap >= n) {
    g_engine->attach(lk, g_scratch);
    const size_t cap = g_scratch->cap;
    bmsched::init(*g_scratch, n, ihs, targets, start, ih_off);
    g_scratch->cap = cap;
    int rc = sync_vpool(lk, g_scratch);
    if (rc < 0) return rc;
    std::vector<uint32_t> slots(n);
    for (size_t i = 0; i < n; ++i) slots[i] = (uint32_t)i;
    return init_slots(g_scratch, slots.data(), n);
  }
  if (g_scratch) {
    if (g_engine->attached() == g_scratch) g_engine->detach(lk);
    batch_free_dev(g_scratch);
    delete g_scratch;
    g_scratch = nullptr;
  }
  g_scratch = new bmpow_batch();
  g_engine->detach(lk);  // nothing may run while the new tables are uploaded synchronously
  const int rc = batch_init(lk, g_scratch, n, ihs, targets, start, ih_off);
  if (rc == 0) g_engine->attach(lk, g_scratch);
  return rc;
}

// ---------------------------------------------------------------------------------------
// run()'s single-object path (bm_search1_kernel, bm_one_* in bmpow_layout.h).  A serial run() call --
// every call site in the reference (class_singleWorker.py:236,1276, api.py:1304,1350) -- needs the
// lowest latency per object: the object rides in the kernel arguments (no upload), each window is one
// launch per piece with the next window queued behind it when it may be needed (it stops at once on
// the call's hit), and each launch's last workgroup writes its result into host-mapped memory that this
// thread polls (no resolve kernel, no copy, no event, no stepper thread in between).
//
// Pieces (round 5).  On several physical devices each window is cut into one interleaved piece per
// device (columns [g0, g0 + nwg) of the window's gn, as the engine's split windows) and the pieces share
// the call's running minimum through the cross-device bound (a host-pinned table, one slot per call in
// the ring, one row per piece; bm_publish / the kernel's relay).  Shards that share a device never split
// a window: their kernels would compete for the same SIMDs (the engine's split windows over 8 streams
// of one MI355X ran C1 at 3.11 GH/s with 46 % of the hashed nonces past the answer, round 4), so such a
// device gets one piece with all its resident workgroups.  bmpow_set_run_split(1) forces one piece per
// shard (the tests' rehearsal of the multi-device path on one GPU).
// ---------------------------------------------------------------------------------------
struct OnePath {
  int dev = -1;
  bm_one_call* d_calls = nullptr;
  bm_one_ctr* d_ctr = nullptr;
  bm_one_out* h_out = nullptr;  // host-mapped ring of results
  bm_one_out* d_out = nullptr;  // the device's address of h_out
  unsigned long long* d_xone = nullptr;  // the cross-device table as this device maps it
  hipStream_t stream = nullptr;  // run_stream (or the shard's), or (a forced piece sharing its device) a masked one
  bool masked = false;           // stream is the CU-masked stream of this piece's slice (masked_stream)
  uint32_t cus = 0;              // CUs of that slice (0: the whole device)
  uint32_t slice = 0, slices = 1;  // this piece's slice of its device, of `slices`
  hipEvent_t ev[8] = {};  // BMPOW_ONE_EVENT: recorded behind launch seq in ev[seq % 8]
  uint64_t seq = 0;
  double rate = 0;  // trials per ms, an exponential average over launches of >= 2^24 trials (0: none yet)
  uint64_t trials = 0;  // since bmpow_reset_stats (bmpow_get_shard_stats)
  double ms = 0;
};
std::vector<OnePath> g_ones;  // per shard; set up for the shards that carry pieces
unsigned long long* g_xone = nullptr;  // the cross-device bound of split run() calls (BM_MAX_SHARDS x BM_XSLOTS)
uint64_t g_one_call = 0;
bool g_run_split = false;  // bmpow_set_run_split: one piece per shard even where shards share a device
// The wait (g_one_wait): "auto" spins when the call's answer is expected within kOneSpinMs (E over
// the pieces' measured rate), and otherwise sleeps between polls of the result word.  The reference's PoW threads run at SCHED_IDLE
// (bitmsghash.cpp:149) and its pool workers at nice 20 (proofofwork.py:72-87): run() happens on the
// caller's own thread here, so it keeps its priority and instead leaves the CPU alone while the GPU
// works, except for the last few ms of a short call.
constexpr double kOneSpinMs = 20.0;
// A run() beside a busy batch expected to take longer than this (one engine launch is ~80 ms) shares the
// device with the batch instead of going first (search_one_calls)
constexpr double kOneShareMs = 100.0;
// a piece's rate before it has a sample: one MI355X's bm_search1_kernel, measured
constexpr double kOneRateGuess = 6.5e6;

// CU-masked streams, one per (device, CU range), created on first use and kept for the life of the
// process.  On this ROCm (7.2) creating a masked stream after masked streams were destroyed hangs inside
// hipExtStreamCreateWithCUMask -- the second creation after three were destroyed, every time
// (tools/diag/cumask_free.hip, profiles/r05/cumask_free/) -- while creating many and destroying none
// does not.  So the library never destroys one; a forced split reuses its slices' streams, and past
// kMaxMasked distinct ranges a piece runs on its shard's stream unmasked.  (Each holds a hardware queue
// and ~190 MiB of host memory in the runtime: tools/diag/rss_layout.py.)
struct MaskedStream {
  int dev;
  uint32_t lo, hi;
  hipStream_t stream;
};
std::vector<MaskedStream> g_masked;
constexpr size_t kMaxMasked = 24;

// The stream of CUs [lo, hi) of device dev (n CUs), or null once kMaxMasked ranges exist.
int masked_stream(int dev, uint32_t n, uint32_t lo, uint32_t hi, hipStream_t* out) {
  *out = nullptr;
  for (const MaskedStream& m : g_masked)
    if (m.dev == dev && m.lo == lo && m.hi == hi) {
      *out = m.stream;
      return 0;
    }
  if (g_masked.size() >= kMaxMasked) return 0;
  std::vector<uint32_t> mask((n + 31) / 32, 0);
  for (uint32_t cu = lo; cu < hi; ++cu) mask[cu / 32] |= 1u << (cu % 32);
  hipStream_t st = nullptr;
  HIPTRY(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
  g_masked.push_back({dev, lo, hi, st});
  BM_TRACE("masked stream %zu: dev %d CUs [%u, %u) stream %p", g_masked.size() - 1, dev, lo, hi, (void*)st);
  *out = st;
  return 0;
}

// run()'s stream on a device: one per device, of the highest priority, kept for the process like the
// masked streams.  On the shard's stream a run() beside a busy batch queued behind the engine's running
// launch and its lookahead (160-240 ms, tools/diag/run_beside_service.py); on its own stream the call's
// workgroups are dispatched as the running launch's retire.  Used only by calls made while the engine
// has work, and created at the first such call: a stream costs the runtime a hardware queue and ~190 MiB
// of host memory (tools/diag/rss_layout.py).  BMPOW_RUN_STREAM=0: always the shard's stream (A/B,
// g_run_stream).
std::vector<std::pair<int, hipStream_t>> g_run_streams;

int run_stream(int dev, hipStream_t* out) {
  for (const auto& r : g_run_streams)
    if (r.first == dev) {
      *out = r.second;
      return 0;
    }
  int least = 0, greatest = 0;
  HIPTRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t st = nullptr;
  HIPTRY(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest));
  g_run_streams.emplace_back(dev, st);
  BM_TRACE("run stream: dev %d priority %d (range %d..%d) stream %p", dev, greatest, least, greatest, (void*)st);
  *out = st;
  return 0;
}

void free_one() {
  // every stream a piece launched on drains before any buffer is freed (hipFree waits for the device)
  for (size_t s = 0; s < g_ones.size(); ++s) {
    OnePath& op = g_ones[s];
    if (op.dev < 0) continue;
    (void)hipSetDevice(op.dev);
    BM_TRACE("free_one: piece %zu dev %d masked %d: stream %s, shard stream %s", s, op.dev, (int)op.masked,
             op.stream ? hipGetErrorName(hipStreamQuery(op.stream)) : "-",
             s < g_shards.size() && g_shards[s].stream ? hipGetErrorName(hipStreamQuery(g_shards[s].stream)) : "-");
    if (s < g_shards.size() && g_shards[s].stream) (void)hipStreamSynchronize(g_shards[s].stream);
    if (op.stream && (s >= g_shards.size() || op.stream != g_shards[s].stream)) (void)hipStreamSynchronize(op.stream);
  }
  BM_TRACE("free_one: streams drained");
  for (size_t s = 0; s < g_ones.size(); ++s) {
    OnePath& op = g_ones[s];
    if (op.dev < 0) continue;
    (void)hipSetDevice(op.dev);
    if (op.d_calls) (void)hipFree(op.d_calls);
    if (op.d_ctr) (void)hipFree(op.d_ctr);
    if (op.h_out) (void)hipHostFree(op.h_out);
    for (hipEvent_t e : op.ev)
      if (e) (void)hipEventDestroy(e);
  }
  g_ones.clear();
  if (g_xone) (void)hipHostFree(g_xone);
  g_xone = nullptr;
  BM_TRACE("free_one: done");
}

int ensure_one(size_t s, uint32_t slice, uint32_t slices) {
  if (g_ones.size() != g_shards.size()) g_ones.resize(g_shards.size());
  OnePath& op = g_ones[s];
  const Shard& sh = g_shards[s];
  if (op.dev == sh.dev && op.d_calls && op.slice == slice && op.slices == slices) return 0;
  HIPTRY(hipSetDevice(sh.dev));
  if (op.stream && op.stream != sh.stream) (void)hipStreamSynchronize(op.stream);  // another slice than before
  if (op.d_calls) (void)hipFree(op.d_calls);
  if (op.d_ctr) (void)hipFree(op.d_ctr);
  if (op.h_out) (void)hipHostFree(op.h_out);
  for (hipEvent_t e : op.ev)
    if (e) (void)hipEventDestroy(e);
  if (!g_xone) {
    HIPTRY(hipHostMalloc(&g_xone, sizeof(unsigned long long) * BM_MAX_SHARDS * BM_XSLOTS,
                         hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent));
    for (size_t i = 0; i < (size_t)BM_MAX_SHARDS * BM_XSLOTS; ++i) g_xone[i] = ~0ULL;
  }
  op = OnePath();
  op.dev = sh.dev;
  op.slice = slice;
  op.slices = slices;
  op.stream = sh.stream;  // search_one_calls moves it to run_stream while a batch is running
  if (slices > 1 && g_split_cumask && sh.cus > 0) {
    const uint32_t n = (uint32_t)sh.cus, lo = slice * n / slices, hi = (slice + 1) * n / slices;
    hipStream_t st = nullptr;
    const int rc = masked_stream(sh.dev, n, lo, hi, &st);
    if (rc < 0) return rc;
    if (st) {
      op.stream = st;
      op.masked = true;
      op.cus = hi - lo;
    }
    BM_TRACE("ensure_one: piece %zu dev %d slice %u/%u: CUs [%u, %u) stream %p", s, sh.dev, slice, slices, lo, hi,
             (void*)op.stream);
  }
  bm_one_call init[BM_ONE_CALLS];
  std::memset(init, 0, sizeof init);
  for (bm_one_call& c : init) c.best = ~0ULL;
  HIPTRY(hipMalloc(&op.d_calls, sizeof init));
  HIPTRY(hipMemcpy(op.d_calls, init, sizeof init, hipMemcpyHostToDevice));
  HIPTRY(hipMalloc(&op.d_ctr, BM_ONE_RING * sizeof(bm_one_ctr)));
  HIPTRY(hipMemset(op.d_ctr, 0, BM_ONE_RING * sizeof(bm_one_ctr)));
  HIPTRY(hipHostMalloc(&op.h_out, BM_ONE_RING * sizeof(bm_one_out), hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(op.h_out, 0, BM_ONE_RING * sizeof(bm_one_out));
  void* dp = nullptr;
  HIPTRY(hipHostGetDevicePointer(&dp, op.h_out, 0));
  op.d_out = (bm_one_out*)dp;
  HIPTRY(hipHostGetDevicePointer(&dp, g_xone, 0));
  op.d_xone = (unsigned long long*)dp;
  if (g_one_event)
    for (hipEvent_t& e : op.ev) HIPTRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return 0;
}

// The shards that carry a run()'s pieces: the first shard of every device (or every shard, forced).
std::vector<size_t> one_pieces() {
  std::vector<size_t> p;
  for (size_t s = 0; s < g_shards.size(); ++s) {
    bool dup = false;
    for (size_t q : p) dup = dup || g_shards[q].dev == g_shards[s].dev;
    if (!dup || g_run_split) p.push_back(s);
  }
  return p;
}

// Wait for launch `seq`'s result word.  spin: poll it with a pause (the answer is due within a few
// ms); else sleep between polls for 1/64 of the time waited so far (20 us .. 250 us) -- a few
// thousand polls per second, each a load of host memory.  The launch's event is queried every few
// polls, so a launch that ended without writing its result (a fault) is caught instead of waited for
// forever.
int wait_one(OnePath& op, uint64_t seq, bool spin, double& spin_ms, double& sleep_ms) {
  bm_one_out* o = &op.h_out[seq % BM_ONE_RING];
  const double t0 = now_ms();
  for (uint32_t k = 1;; ++k) {
    if (__atomic_load_n(&o->seq, __ATOMIC_ACQUIRE) == seq) break;
    if (spin ? k % 1024u == 0 : (g_one_query > 0 && k % (uint32_t)g_one_query == 0)) {
      const hipError_t e = g_one_event ? hipEventQuery(op.ev[seq % 8]) : hipStreamQuery(op.stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(&o->seq, __ATOMIC_ACQUIRE) == seq) break;
        return set_err(BMPOW_E_HIP, "single-object launch completed without its result");
      }
      if (e != hipErrorNotReady) return set_err(BMPOW_E_HIP, std::string("single-object launch: ") + hipGetErrorString(e));
    }
    if (spin) {
      // a spinning wait still gives its CPU to any other runnable thread now and then (the reference's
      // PoW threads run at SCHED_IDLE, bitmsghash.cpp:149: they never hold a CPU another thread wants)
      if (g_spin_yield && (k & 63) == 0) sched_yield();
      else __builtin_ia32_pause();
    } else {
      const double waited_us = (now_ms() - t0) * 1e3;
      std::this_thread::sleep_for(std::chrono::microseconds((int64_t)std::min(250.0, std::max(20.0, waited_us / 64))));
    }
  }
  const double ms = now_ms() - t0;
  (spin ? spin_ms : sleep_ms) += ms;
  return 0;
}

// g: the library's lock (g_mu), held by the caller, who also holds g_one_mu for the whole call.  It is
// released while the call waits for a window's pieces, so the batch service's steps go on between
// run()'s windows (round 6: before, a long run() held it to the end and the batch stalled behind it).
int search_one_calls(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials, uint64_t* nonce_out,
                     uint64_t* trial_out, std::unique_lock<FairMutex>& g) {
  const std::vector<size_t> pieces = one_pieces();
  const size_t P = pieces.size();
  for (size_t p = 0; p < P; ++p) {
    uint32_t slice = 0, slices = 0;  // this piece's place among the pieces on its device
    for (size_t q = 0; q < P; ++q)
      if (g_shards[pieces[q]].dev == g_shards[pieces[p]].dev) {
        if (q < p) ++slice;
        ++slices;
      }
    const int rc = ensure_one(pieces[p], slice, slices);
    if (rc < 0) return rc;
  }
  const uint64_t end = (max_trials - 1 > kU64Max - start) ? kU64Max : start + max_trials - 1;  // last nonce
  const uint64_t call = ++g_one_call;  // every call launches on every piece (it resets call + 2's state)
  const uint32_t xslot = (uint32_t)(call % BM_ONE_CALLS);
  if (P > 1) {
    // the call's slot of every row starts at "no hit": launches still in flight belong to the previous
    // call (each call waits for its first window on every piece), which uses another slot
    for (size_t r = 0; r < P; ++r) __atomic_store_n(&g_xone[r * BM_XSLOTS + xslot], ~0ULL, __ATOMIC_RELAXED);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  // Columns per piece: the device's resident workgroups over the pieces sharing it (at most the
  // hardware queues' worth run at once), less the relay's workgroup of a split call.
  uint32_t hwq = 4;
  if (const char* e = std::getenv("GPU_MAX_HW_QUEUES"))
    if (std::atoi(e) > 0) hwq = (uint32_t)std::atoi(e);
  std::vector<uint32_t> cap(P);
  double rate = 0;
  bool shared = false;  // pieces share a device (bmpow_set_run_split)
  for (size_t p = 0; p < P; ++p) {
    const Shard& sh = g_shards[pieces[p]];
    const OnePath& op = g_ones[pieces[p]];
    uint32_t same = 0;
    for (size_t q : pieces) same += g_shards[q].dev == sh.dev;
    // a piece on its own CU slice owns that slice's resident workgroups; pieces sharing a whole device
    // split its resident workgroups over the kernels that run at once
    const bool sliced = op.cus > 0;
    shared = shared || (same > 1 && !sliced);
    const double part = sliced ? (double)op.cus / (double)std::max(1, sh.cus) : 1.0 / std::min(same, hwq);
    uint32_t c = sliced ? (uint32_t)((uint64_t)sh.resident * op.cus / (uint32_t)std::max(1, sh.cus))
                        : sh.resident / std::min(same, hwq);
    if (P > 1 && c > 1) --c;
    cap[p] = std::max<uint32_t>(1, std::min<uint32_t>(c, BM_ONE_MAX_WG));
    rate += (op.rate > 0 ? op.rate : kOneRateGuess * part);
  }
  // Beside a batch with work (the engine's launches on the shard streams): a call expected to end within
  // kOneShareMs (E, or its budget, over the pieces' rate) takes run()'s own stream of the highest priority
  // -- its windows are dispatched first, and the batch waits at most that long --, a longer one the shard's
  // stream, where its windows and the engine's launches queue in turn and share the device launch by
  // launch (with g_mu released between its windows the service keeps the engine fed).  Round 5 gave every
  // call the priority stream and held g_mu throughout: a C4-difficulty run() stalled the batch for its
  // whole call.  Else the shard's stream.  A piece changing streams first lets the old one drain (a queued
  // window of the previous call stops at its first block), so its launches stay in call order.
  const double expect_ms = std::min(18446744073709551616.0 / ((double)target + 1.0), (double)max_trials) / rate;
  bool busy = false;
  if (g_run_stream && g_engine && expect_ms <= kOneShareMs) {
    std::lock_guard<std::mutex> el(g_engine->mu);
    const bmsched::BatchState* b = g_engine->attached();
    busy = g_engine->in_flight() > 0 || (b && b->pending > 0);
  }
  for (size_t p = 0; p < P; ++p) {
    OnePath& op = g_ones[pieces[p]];
    if (op.masked) continue;
    hipStream_t want = g_shards[pieces[p]].stream;
    if (busy) {
      HIPTRY(hipSetDevice(op.dev));
      const int rc = run_stream(op.dev, &want);
      if (rc < 0) return rc;
    }
    if (op.stream != want) {
      HIPTRY(hipStreamSynchronize(op.stream));
      op.stream = want;
    }
  }
  // A window: one step per piece (a piece hashes ~1/P of it; bm_one_ctr.acc's trial field).  Pieces
  // that share a device do not all run at once (its hardware queues run 4 kernels; the rest start as
  // those finish), so a piece may sweep its whole share of a window before the piece holding the answer
  // starts: there a window is 2E (bmsched::expect_cap), as the engine's split windows.
  uint64_t step = std::min<uint64_t>(g_step_trials.load(), BM_ONE_MAX_WINDOW) * P;
  if (shared) step = std::min(step, bmsched::expect_cap(target, P, BM_CHUNK));
  const uint64_t bpw = bmsched::kBlocksPerWorker;
  uint64_t next = start;
  bool top = false;
  // windows in flight, oldest first: their nonces and each piece's sequence number
  struct Fly {
    uint64_t n;
    uint64_t seq[BM_MAX_SHARDS];
  };
  Fly fly[2];
  int nfly = 0;
  // The next window is queued behind the running one only while the windows in flight may well hold
  // no hit (fewer than kAheadE x E nonces, E = 2^64 / (target + 1): P(no hit) > e^-8): a C1 object
  // (E ~ 1.3e7 against a 2^29 window) then costs one launch per piece, and no idle lookahead launch sits
  // in the next call's way; a hard object (C4) or a sweep (C3) keeps two windows in flight.
  constexpr double kAheadE = 8.0;
  const double expect = 18446744073709551616.0 / ((double)target + 1.0);
  auto want_next = [&]() {
    double n = 0;
    for (int i = 0; i < nfly; ++i) n += (double)fly[i].n;
    return !top && nfly < 2 && (nfly == 0 || n < kAheadE * expect);
  };
  // spin only for a call whose answer is due within kOneSpinMs (at most that much CPU per call); a
  // longer call sleeps between polls, so a wake-up may come up to 250 us late -- 0.2 % of a 120 ms call
  const bool short_call = expect / rate < kOneSpinMs;
  bm_one_args a;
  std::memset(&a, 0, sizeof a);
  for (int i = 0; i < 8; ++i) a.w[i] = bmsched::load_be64(ih + 8 * i);
  a.target = target;
  a.xslot = xslot;
  a.xrows = (uint32_t)P;
  uint32_t nwg[BM_MAX_SHARDS];
  auto launch = [&]() -> int {
    const uint64_t room = end - next;  // nonces after next, up to end
    const uint64_t count = room >= step ? step : room + 1;
    const uint64_t nblk = count / BM_BLOCK + (count % BM_BLOCK ? 1 : 0);
    const uint64_t per = (nblk + P - 1) / P;  // blocks of a piece
    uint32_t gn = 0;
    for (size_t p = 0; p < P; ++p) {
      nwg[p] = (uint32_t)std::min<uint64_t>(cap[p], std::max<uint64_t>(1, (per + bpw - 1) / bpw));
      gn += nwg[p];
    }
    Fly& f = fly[nfly];
    f.n = count;
    a.start = next;
    a.count = count;
    a.gn = gn;
    uint32_t g0 = 0;
    for (size_t p = 0; p < P; ++p) {
      const Shard& sh = g_shards[pieces[p]];
      OnePath& op = g_ones[pieces[p]];
      a.call = op.d_calls + call % BM_ONE_CALLS;
      a.reset = op.d_calls + (call + 2) % BM_ONE_CALLS;
      a.nwg = nwg[p];
      a.g0 = g0;
      g0 += nwg[p];
      a.xb = P > 1 ? op.d_xone : nullptr;
      a.xrow = (uint32_t)p;
      a.seq = ++op.seq;
      const uint32_t r = (uint32_t)(a.seq % BM_ONE_RING);
      a.ctr = op.d_ctr + r;
      a.out = op.d_out + r;
      f.seq[p] = a.seq;
      if (P > 1) HIPTRY(hipSetDevice(sh.dev));
      HIPTRY(bm_launch_search1(op.stream, a));
      if (g_one_event) HIPTRY(hipEventRecord(op.ev[a.seq % 8], op.stream));
    }
    ++nfly;
    if (room < step) top = true;
    else next += count;
    return 0;
  };
  if (P == 1) HIPTRY(hipSetDevice(g_shards[pieces[0]].dev));
  int rc = launch();
  while (rc == 0 && want_next()) rc = launch();  // the next window, queued behind
  while (rc == 0) {
    // the oldest window: every piece's launch, waited for without the library's lock (only this
    // call's pieces are read meanwhile: g_one_mu keeps every other user of them out)
    bool found = false;
    uint64_t best = 0, best_trial = 0;
    double span = 0, spin_ms = 0, sleep_ms = 0;
    const bool spin = g_one_wait == kOneSpin || (g_one_wait == kOneAuto && short_call);
    g.unlock();
    for (size_t p = 0; p < P && rc == 0; ++p) rc = wait_one(g_ones[pieces[p]], fly[0].seq[p], spin, spin_ms, sleep_ms);
    g.lock();
    g_stats.one_wait_spin_ms += spin_ms;
    g_stats.one_wait_sleep_ms += sleep_ms;
    for (size_t p = 0; p < P && rc == 0; ++p) {
      OnePath& op = g_ones[pieces[p]];
      const uint64_t seq = fly[0].seq[p];
      const bm_one_out& o = op.h_out[seq % BM_ONE_RING];
      const double ms = (double)(o.t1 - o.t0) * 1e-5;  // s_memrealtime: 100 MHz
      g_stats.launches++;
      g_stats.trials += o.trials;
      g_stats.cut_trials += o.cut;
      g_stats.kernel_ms += ms;
      span = std::max(span, ms);
      op.trials += o.trials;
      op.ms += ms;
      if (o.trials >= bmsched::kRateMinTrials && ms > 0)
        op.rate = op.rate > 0 ? (1 - bmsched::kRateAlpha) * op.rate + bmsched::kRateAlpha * (double)o.trials / ms
                              : (double)o.trials / ms;
      // a piece's result is its device's running minimum: its own hit, or one the relay folded in (a
      // real hit of the object too); found is its own.  The least found over the pieces is the answer:
      // every piece hashed all of its blocks that start at or below any hit it saw, so the block holding
      // the least hit of the window was hashed by its piece, which then holds that hit
      if (o.found && (!found || o.nonce < best)) {
        found = true;
        best = o.nonce;
        best_trial = o.trial;
      }
    }
    if (rc < 0) break;
    g_stats.steps++;
    g_stats.max_shard_kernel_ms += span;
    if (found) {  // the lowest hit: every earlier window of the call ended without one
      *nonce_out = best;
      *trial_out = best_trial;
      return BMPOW_FOUND;  // a window still queued stops at its first block (the call's best)
    }
    fly[0] = fly[1];
    --nfly;
    if (g_abort.load()) return set_err(BMPOW_E_ABORTED, "aborted");
    while (rc == 0 && want_next()) rc = launch();
    if (nfly == 0) return BMPOW_NOT_FOUND;
  }
  return rc;
}

int search_one(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials, uint64_t* nonce_out,
               uint64_t* trial_out, std::unique_lock<FairMutex>& g) {
  const int rc = search_one_calls(ih, target, start, max_trials, nonce_out, trial_out, g);
  // A call that failed may have launched on only some pieces (or none): the pieces it skipped did not
  // put the state of the call two ahead back to "no hit", which that call would then read.  Start the
  // ring afresh (an abort comes only after every piece's first launch, so it keeps the ring).
  if (rc < 0 && rc != BMPOW_E_ABORTED) free_one();
  return rc;
}

// Drop the scratch batch (device set change, shutdown).  lk: the engine's mutex.
void drop_scratch(std::unique_lock<std::mutex>& lk) {
  if (!g_scratch) return;
  if (g_engine && g_engine->attached() == g_scratch) g_engine->detach(lk);
  batch_free_dev(g_scratch);
  delete g_scratch;
  g_scratch = nullptr;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Receive-side verification session.  Layout per shard, device resident:
//   pool[blocks]  : every payload (object[8:]) SHA-512-padded to whole 128-B blocks, objects
//                   back to back in sorted order (so one lane reads one contiguous run)
//   obj[k]        : {first block, block count, nonce} of the k-th object in sorted order
//   pow[k]        : result
// Objects are sorted by block count (descending) so a wave's lanes iterate alike, and the
// sorted list is cut into per-shard slices of equal block totals.
// ---------------------------------------------------------------------------------------
struct bmpow_vbatch {
  size_t n = 0;
  struct Part : bmsched::VPart {  // shard, sorted order, bv_obj list, blocks (bmpow_sched.h)
    bv_obj* d_obj = nullptr;
    uint4* d_pool = nullptr;
    uint64_t* d_pow = nullptr;
    uint64_t* h_pow = nullptr;  // pinned
    uint32_t* d_bins = nullptr; // plan_bins' offsets + group lists (binned kernel), or null
    bool borrowed = false;      // buffers belong to the shard (one-shot path)
  };
  std::vector<Part> parts;
  uint64_t blocks = 0;
};

namespace {

using bmsched::load_be64;
using bmsched::Span;

void vbatch_free(bmpow_vbatch* vb) {
  for (auto& pt : vb->parts) {
    if (pt.borrowed) continue;
    if (pt.shard < g_shards.size()) (void)hipSetDevice(g_shards[pt.shard].dev);
    if (pt.d_obj) (void)hipFree(pt.d_obj);
    if (pt.d_pool) (void)hipFree(pt.d_pool);
    if (pt.d_pow) (void)hipFree(pt.d_pow);
    if (pt.h_pow) (void)hipHostFree(pt.h_pow);
    if (pt.d_bins) (void)hipFree(pt.d_bins);
  }
  vb->parts.clear();
}

template <typename T>
int grow_device(T*& p, size_t& cap, size_t need) {
  if (need <= cap && p) return 0;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  HIPTRY(hipMalloc(&p, need));
  cap = need;
  return 0;
}

constexpr uint64_t kVStageBytes = 64ull << 20;  // pinned staging chunk (x2 per shard)

// One-shot path: the part's pool goes up through the shard's two pinned staging chunks, padding of
// chunk c+1 overlapping the DMA of chunk c; device buffers are the shard's, reused across calls.
int vbatch_upload_transient(bmpow_vbatch::Part& pt, const std::vector<Span>& objs) {
  const std::vector<bv_obj>& ho = pt.ho;
  Shard& sh = g_shards[pt.shard];
  const size_t m = pt.orig.size();
  if (m > sh.vobj_cap || !sh.d_vobj) {
    if (sh.d_vobj) (void)hipFree(sh.d_vobj);
    if (sh.d_vpow) (void)hipFree(sh.d_vpow);
    if (sh.h_vpow) (void)hipHostFree(sh.h_vpow);
    sh.d_vobj = nullptr;
    sh.d_vpow = nullptr;
    sh.h_vpow = nullptr;
    sh.vobj_cap = 0;
    const size_t cap = std::max<size_t>(m, 4096);
    HIPTRY(hipMalloc(&sh.d_vobj, cap * sizeof(bv_obj)));
    HIPTRY(hipMalloc(&sh.d_vpow, cap * sizeof(uint64_t)));
    HIPTRY(hipHostMalloc(&sh.h_vpow, cap * sizeof(uint64_t), hipHostMallocDefault));
    sh.vobj_cap = cap;
  }
  {
    size_t cap = sh.d_vpool_cap;
    int rc = grow_device(sh.d_vpool, cap, std::max<size_t>(pt.blocks * 128, 16));
    sh.d_vpool_cap = cap;
    if (rc < 0) return rc;
  }
  for (int c = 0; c < 2; ++c) {
    if (!sh.h_vstage[c]) HIPTRY(hipHostMalloc(&sh.h_vstage[c], kVStageBytes, hipHostMallocDefault));
    if (!sh.ev_vstage[c]) HIPTRY(hipEventCreateWithFlags(&sh.ev_vstage[c], hipEventDisableTiming));
  }
  pt.d_obj = sh.d_vobj;
  pt.d_pool = sh.d_vpool;
  pt.d_pow = sh.d_vpow;
  pt.h_pow = sh.h_vpow;
  pt.borrowed = true;
  // chunks of whole objects; an object larger than a chunk is padded in pageable memory on its own
  size_t j = 0;
  int c = 0;
  bool used[2] = {false, false};
  std::unique_ptr<uint8_t[]> big;
  while (j < m) {
    const uint64_t blk0 = ho[j].blk;
    size_t j1 = j;
    uint64_t bytes = 0;
    while (j1 < m && (j1 == j || bytes + (uint64_t)ho[j1].nblk * 128 <= kVStageBytes)) {
      bytes += (uint64_t)ho[j1].nblk * 128;
      ++j1;
    }
    uint8_t* dst;
    if (bytes > kVStageBytes) {
      big.reset(new uint8_t[bytes]);
      dst = big.get();
    } else {
      if (used[c]) HIPTRY(hipEventSynchronize(sh.ev_vstage[c]));  // its previous DMA is done
      dst = sh.h_vstage[c];
    }
    bmsched::pad_range(objs, pt, j, j1, blk0, dst);
    HIPTRY(hipMemcpyAsync((uint8_t*)pt.d_pool + blk0 * 128, dst, bytes, hipMemcpyHostToDevice, sh.stream));
    if (dst == big.get()) {
      HIPTRY(hipStreamSynchronize(sh.stream));
      big.reset();
    } else {
      HIPTRY(hipEventRecord(sh.ev_vstage[c], sh.stream));
      used[c] = true;
      c ^= 1;
    }
    j = j1;
  }
  if (!pt.bins.empty()) {
    size_t cap = sh.vbins_cap;
    const int rc = grow_device(sh.d_vbins, cap, pt.bins.size() * sizeof(uint32_t));
    sh.vbins_cap = cap;
    if (rc < 0) return rc;
    pt.d_bins = sh.d_vbins;
    HIPTRY(hipMemcpyAsync(pt.d_bins, pt.bins.data(), pt.bins.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          sh.stream));
  }
  // the descriptors last: the padding pass filled their nonces (one pass over the objects' memory)
  HIPTRY(hipMemcpyAsync(pt.d_obj, ho.data(), m * sizeof(bv_obj), hipMemcpyHostToDevice, sh.stream));
  HIPTRY(hipStreamSynchronize(sh.stream));
  return 0;
}

// The binned kernel balances the SIMDs of a flood with at least a few waves per SIMD; a smaller
// one runs one wave per group in sorted order.  BMPOW_VBINNED=0/1 forces either (A/B runs).
bool verify_binned(size_t m, size_t nbins) {
  if (nbins == 0) return false;
  if (const char* e = std::getenv("BMPOW_VBINNED")) return std::atoi(e) != 0;
  return (m + BV_BLOCK - 1) / BV_BLOCK >= 2 * nbins;
}

std::vector<bmsched::VPart> g_vplan;  // under g_mu

// Hand a one-shot batch's plan vectors back to g_vplan before the batch is freed.
void vbatch_release_plan(bmpow_vbatch* vb) {
  g_vplan.resize(std::max(g_vplan.size(), vb->parts.size()));
  for (size_t i = 0; i < vb->parts.size(); ++i) std::swap(static_cast<bmsched::VPart&>(vb->parts[i]), g_vplan[i]);
}

int vbatch_build(bmpow_vbatch* vb, const std::vector<Span>& objs, bool transient = false) {
  vb->n = objs.size();
  // the plan's vectors live in g_vplan between calls (swapped into the parts here, back by
  // vbatch_release_plan): a flood's descriptors are tens of MB, and fresh pages cost more than
  // the planning
  std::vector<bmsched::VPart>& plan = g_vplan;
  if (bmsched::plan_verify(objs, g_shards.size(), plan, vb->blocks) < 0)
    return set_err(BMPOW_E_ARG, "too many objects, an object too large, or a payload pool above 2^32 blocks");
  vb->parts.resize(plan.size());
  for (size_t i = 0; i < plan.size(); ++i) {
    bmsched::VPart& pt = vb->parts[i];
    std::swap(pt, plan[i]);
    const size_t nbins = 4 * (size_t)g_shards[pt.shard].cus;
    if (verify_binned(pt.orig.size(), nbins)) bmsched::plan_bins(pt, nbins);
  }
  for (auto& pt : vb->parts) {
    Shard& sh = g_shards[pt.shard];
    HIPTRY(hipSetDevice(sh.dev));
    const size_t m = pt.orig.size();
    if (transient) {
      const int rc = vbatch_upload_transient(pt, objs);
      if (rc < 0) return rc;
      continue;
    }
    // padding is a memory-bound copy of every payload: spread it over host threads
    std::unique_ptr<uint8_t[]> pool(new uint8_t[pt.blocks * 128]);  // pad_into writes every byte
    bmsched::pad_range(objs, pt, 0, m, 0, pool.get());
    HIPTRY(hipMalloc(&pt.d_obj, m * sizeof(bv_obj)));
    HIPTRY(hipMalloc(&pt.d_pool, std::max<size_t>(pt.blocks * 128, 16)));
    HIPTRY(hipMalloc(&pt.d_pow, m * sizeof(uint64_t)));
    HIPTRY(hipHostMalloc(&pt.h_pow, m * sizeof(uint64_t), hipHostMallocDefault));
    HIPTRY(hipMemcpy(pt.d_obj, pt.ho.data(), m * sizeof(bv_obj), hipMemcpyHostToDevice));
    HIPTRY(hipMemcpy(pt.d_pool, pool.get(), pt.blocks * 128, hipMemcpyHostToDevice));
    if (!pt.bins.empty()) {
      HIPTRY(hipMalloc(&pt.d_bins, pt.bins.size() * sizeof(uint32_t)));
      HIPTRY(hipMemcpy(pt.d_bins, pt.bins.data(), pt.bins.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
  }
  return 0;
}

int vbatch_run_locked(bmpow_vbatch* vb, uint64_t* pow_out) {
  for (auto& pt : vb->parts) {
    Shard& sh = g_shards[pt.shard];
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipEventRecord(sh.ev0, sh.stream));
    if (pt.d_bins)
      HIPTRY(bv_launch_pow_binned(sh.stream, pt.d_obj, (uint32_t)pt.orig.size(), pt.d_pool, pt.d_pow, pt.d_bins,
                                  (uint32_t)pt.nbins));
    else
      HIPTRY(bv_launch_pow(sh.stream, pt.d_obj, (uint32_t)pt.orig.size(), pt.d_pool, pt.d_pow));
    HIPTRY(hipEventRecord(sh.ev1, sh.stream));
    HIPTRY(hipMemcpyAsync(pt.h_pow, pt.d_pow, pt.orig.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, sh.stream));
  }
  double mx = 0;
  for (auto& pt : vb->parts) {
    Shard& sh = g_shards[pt.shard];
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipStreamSynchronize(sh.stream));
    float ms = 0;
    HIPTRY(hipEventElapsedTime(&ms, sh.ev0, sh.ev1));
    mx = std::max<double>(mx, ms);
    g_stats.verify_launches++;
    if (pow_out)
      for (size_t j = 0; j < pt.orig.size(); ++j) pow_out[pt.orig[j]] = pt.h_pow[j];
  }
  g_stats.verify_kernel_ms += mx;
  g_stats.verify_objects += vb->n;
  g_stats.verify_blocks += vb->blocks;
  return 0;
}

int spans_from(size_t n, const uint8_t* objs, const uint64_t* offsets, std::vector<Span>& out) {
  if (n && (!objs || !offsets)) return set_err(BMPOW_E_ARG, "null pointer");
  out.resize(n);
  for (size_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i] + 8) return set_err(BMPOW_E_ARG, "object shorter than its 8-byte nonce");
    out[i] = {objs + offsets[i], offsets[i + 1] - offsets[i]};
  }
  return 0;
}

using bmsched::pow_sufficient;

}  // namespace

// ---------------------------------------------------------------------------------------
// RIPE-prefix address search (bmpow_addr.hip).  Steps cover contiguous ranges of try indices
// [next, next + S*step), one slice per shard; a hit is reported only after the step that
// covers every smaller try has completed, so the answer is the first k, as the reference's
// sequential loop finds it.  Step sizes ramp up from about the expected number of tries
// (256^null_bytes) so a 1-byte search costs one small launch.
// ---------------------------------------------------------------------------------------
namespace {

constexpr uint64_t kAddrMaxStep = 1ULL << 22;  // tries per shard per launch (~10 ms)

// Shards are only ever freed all together (reset / re-init), so a borrowed table never outlives
// its owner.  The allocation holds ec::kWindows extra entries: ar_launch_table's base points.
// c = 0: the 16-bit comb (64 MB), c = 1: the 24-bit comb (10.7 GB).
constexpr int kCombBits[2] = {ec::kCombSmall, ec::kCombLarge};

int ensure_table(Shard& sh, int c = 0) {
  if (sh.d_table[c]) return 0;
  for (const Shard& o : g_shards)
    if (&o != &sh && o.dev == sh.dev && o.d_table[c] && o.owns_table[c]) {
      sh.d_table[c] = o.d_table[c];
      return 0;
    }
  HIPTRY(hipSetDevice(sh.dev));
  const size_t bytes = ar_table_entries(kCombBits[c]) * sizeof(ec::ge);
  ec::ge* t = nullptr;
  const hipError_t e = hipMalloc(&t, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // an out-of-memory here is reported, not sticky
    return set_err(BMPOW_E_HIP, std::string("comb table allocation: ") + hipGetErrorString(e));
  }
  sh.d_table[c] = t;
  sh.owns_table[c] = true;
  HIPTRY(hipMemsetAsync(t, 0, bytes, sh.stream));
  HIPTRY(ar_launch_table(sh.stream, t, kCombBits[c]));
  HIPTRY(hipStreamSynchronize(sh.stream));
  return 0;
}

// Comb choice for one search: the 24-bit comb when forced (bmpow_addr_set_comb(24)), or in auto
// mode when it is already built on every shard or the search is expected to take >= 2^32 tries
// (4+ null bytes: seconds of work, against ~0.4 s to build the table once per device; judged from
// null_bytes alone, since callers cut long searches into bounded calls); else the 16-bit one.  An
// auto-mode allocation failure falls back to the small comb.
int g_addr_comb = 0;       // 0 auto, 16, 24
int g_addr_last_comb = 0;  // width used by the last search

int addr_pick_comb(int null_bytes) {
  if (g_addr_comb == ec::kCombSmall) return 0;
  bool built = true;
  for (const Shard& sh : g_shards) built = built && sh.d_table[1] != nullptr;
  const uint64_t expected = null_bytes >= 8 ? kU64Max : (1ULL << (8 * null_bytes));
  const bool want = g_addr_comb == ec::kCombLarge || built || expected >= (1ULL << 32);
  if (!want) return 0;
  for (Shard& sh : g_shards) {
    const int rc = ensure_table(sh, 1);
    if (rc < 0) {
      if (g_addr_comb == ec::kCombLarge) return rc;
      return 0;
    }
  }
  return 1;
}

void be_words_from_bytes(const uint8_t* b, uint64_t (&w)[4]) {
  for (int i = 0; i < 4; ++i) w[i] = load_be64(b + 8 * i);
}

void bytes_from_be_words(const uint64_t* w, int n, uint8_t* out) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(w[i] >> (56 - 8 * j));
}

void point_bytes(const ec::ge& p, uint8_t* out) {  // 04 || X || Y, big-endian
  out[0] = 0x04;
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) {
      out[1 + 4 * i + j] = (uint8_t)(p.x.d[7 - i] >> (24 - 8 * j));
      out[33 + 4 * i + j] = (uint8_t)(p.y.d[7 - i] >> (24 - 8 * j));
    }
}

struct AddrShard {
  ar_params* d_prm = nullptr;
  uint8_t* d_seed = nullptr;
  unsigned long long* d_best = nullptr;
  ar_result* d_res = nullptr;
  uint64_t* d_priv = nullptr;
  uint32_t* d_ok = nullptr;
};

void addr_free(std::vector<AddrShard>& v) {
  for (size_t s = 0; s < v.size() && s < g_shards.size(); ++s) {
    (void)hipSetDevice(g_shards[s].dev);
    if (v[s].d_prm) (void)hipFree(v[s].d_prm);
    if (v[s].d_seed) (void)hipFree(v[s].d_seed);
    if (v[s].d_best) (void)hipFree(v[s].d_best);
    if (v[s].d_res) (void)hipFree(v[s].d_res);
    if (v[s].d_priv) (void)hipFree(v[s].d_priv);
    if (v[s].d_ok) (void)hipFree(v[s].d_ok);
  }
  v.clear();
}

int addr_search_locked(uint32_t mode, const uint8_t* seed, size_t len, const uint8_t* priv_s, uint64_t start,
                       uint64_t max_tries, int null_bytes, bmpow_address* out, std::vector<AddrShard>& as) {
  if (null_bytes < 0 || null_bytes > 20) return set_err(BMPOW_E_ARG, "null_bytes must be in [0, 20]");
  if (!out || (len && !seed) || (mode == 1 && !priv_s)) return set_err(BMPOW_E_ARG, "null pointer");
  if (max_tries == 0) return BMPOW_NOT_FOUND;
  if (mode == 0 && start > (kU64Max >> 1)) return set_err(BMPOW_E_ARG, "try index above 2^63 (nonce 2k overflows)");
  ar_params hp;
  std::memset(&hp, 0, sizeof hp);
  hp.total_len = len;
  hp.tail_len = (uint32_t)(len % 128);
  hp.null_bytes = (uint32_t)null_bytes;
  hp.mode = mode;
  const uint64_t nfull = len / 128;
  for (uint32_t i = 0; i < hp.tail_len; ++i) {
    const uint64_t byte = seed[nfull * 128 + i];
    hp.tmpl[i >> 3] |= byte << (56 - 8 * (i & 7));
  }
  uint64_t pw[4] = {0, 0, 0, 0};
  if (mode == 1) be_words_from_bytes(priv_s, pw);
  const size_t S = g_shards.size();
  as.assign(S, AddrShard());
  for (size_t s = 0; s < S; ++s) {
    Shard& sh = g_shards[s];
    int rc = ensure_table(sh, 0);
    if (rc < 0) return rc;
    AddrShard& a = as[s];
    HIPTRY(hipMalloc(&a.d_prm, sizeof(ar_params)));
    HIPTRY(hipMalloc(&a.d_seed, std::max<size_t>(len, 1)));
    HIPTRY(hipMalloc(&a.d_best, sizeof(unsigned long long)));
    HIPTRY(hipMalloc(&a.d_res, sizeof(ar_result)));
    HIPTRY(hipMalloc(&a.d_priv, 4 * sizeof(uint64_t)));
    HIPTRY(hipMalloc(&a.d_ok, sizeof(uint32_t)));
    HIPTRY(hipMemcpyAsync(a.d_prm, &hp, sizeof hp, hipMemcpyHostToDevice, sh.stream));
    if (len) HIPTRY(hipMemcpyAsync(a.d_seed, seed, len, hipMemcpyHostToDevice, sh.stream));
    HIPTRY(hipMemsetAsync(a.d_best, 0xFF, sizeof(unsigned long long), sh.stream));
    HIPTRY(ar_launch_midstate(sh.stream, a.d_seed, nfull, (uint64_t*)a.d_prm));  // mid[] is at offset 0
    if (mode == 1) {
      HIPTRY(hipMemcpyAsync(a.d_priv, pw, sizeof pw, hipMemcpyHostToDevice, sh.stream));
      HIPTRY(ar_launch_pubkeys(sh.stream, a.d_priv, 1, sh.d_table[0], &a.d_prm->pub_s, a.d_ok));
    }
  }
  for (auto& sh : g_shards) {
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipStreamSynchronize(sh.stream));
  }
  if (mode == 1) {
    uint32_t ok = 0;
    HIPTRY(hipSetDevice(g_shards[0].dev));
    HIPTRY(hipMemcpy(&ok, as[0].d_ok, sizeof ok, hipMemcpyDeviceToHost));
    if (!ok) return set_err(BMPOW_E_ARG, "signing private key is zero");
  }
  const uint64_t end = (kU64Max - start < max_tries) ? kU64Max : start + max_tries;
  const int comb = addr_pick_comb(null_bytes);
  if (comb < 0) return comb;
  g_addr_last_comb = kCombBits[comb];
  uint64_t step = 4096;
  for (int b = 0; b < null_bytes && step < kAddrMaxStep; ++b) step = std::min<uint64_t>(step * 256, kAddrMaxStep);
  step = std::max<uint64_t>(step / 4, 4096);
  uint64_t next = start;
  while (next < end) {
    if (g_abort.load()) return set_err(BMPOW_E_ABORTED, "aborted");
    uint64_t lo[64], cnt[64];
    for (size_t s = 0; s < S && s < 64; ++s) {
      lo[s] = next + s * step;
      cnt[s] = lo[s] >= end ? 0 : std::min<uint64_t>(step, end - lo[s]);
      if (lo[s] < next) cnt[s] = 0;  // wrapped
      Shard& sh = g_shards[s];
      HIPTRY(hipSetDevice(sh.dev));
      HIPTRY(hipEventRecord(sh.ev0, sh.stream));
      HIPTRY(ar_launch_search(sh.stream, as[s].d_prm, mode, sh.d_table[comb], kCombBits[comb], lo[s],
                              (uint32_t)cnt[s], as[s].d_best));
      HIPTRY(hipEventRecord(sh.ev1, sh.stream));
    }
    uint64_t best = kU64Max;
    size_t best_s = 0;
    double mx = 0;
    for (size_t s = 0; s < S && s < 64; ++s) {
      Shard& sh = g_shards[s];
      HIPTRY(hipSetDevice(sh.dev));
      HIPTRY(hipStreamSynchronize(sh.stream));
      float ms = 0;
      HIPTRY(hipEventElapsedTime(&ms, sh.ev0, sh.ev1));
      mx = std::max<double>(mx, ms);
      unsigned long long b = 0;
      HIPTRY(hipMemcpy(&b, as[s].d_best, sizeof b, hipMemcpyDeviceToHost));
      g_stats.addr_tries += cnt[s];
      if (b < best) {
        best = b;
        best_s = s;
      }
    }
    g_stats.addr_kernel_ms += mx;
    g_stats.addr_launches++;
    if (best != kU64Max) {
      Shard& sh = g_shards[best_s];
      HIPTRY(hipSetDevice(sh.dev));
      HIPTRY(ar_launch_resolve(sh.stream, as[best_s].d_prm, sh.d_table[comb], kCombBits[comb], best,
                               as[best_s].d_res));
      ar_result r;
      HIPTRY(hipMemcpyAsync(&r, as[best_s].d_res, sizeof r, hipMemcpyDeviceToHost, sh.stream));
      HIPTRY(hipStreamSynchronize(sh.stream));
      if (!r.ok) return set_err(BMPOW_E_HIP, "resolve of the found try failed");
      std::memset(out, 0, sizeof *out);
      out->k = r.k;
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) out->ripe[4 * i + j] = (uint8_t)(r.ripe[i] >> (8 * j));
      if (mode == 0) bytes_from_be_words(r.priv_s, 4, out->priv_signing);
      else std::memcpy(out->priv_signing, priv_s, 32);
      bytes_from_be_words(r.priv_e, 4, out->priv_encryption);
      point_bytes(r.pub_s, out->pub_signing);
      point_bytes(r.pub_e, out->pub_encryption);
      return BMPOW_FOUND;
    }
    const uint64_t span = step * std::min<size_t>(S, 64);
    next = (kU64Max - next < span) ? end : next + span;
    step = std::min<uint64_t>(step * 2, kAddrMaxStep);
  }
  return BMPOW_NOT_FOUND;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Continuous-batching service (bmpow_service_*): bmsched::Service's stepper thread over a resident
// session, so no caller thread -- and no Python GIL -- sits between two steps.  Its ops take g_mu
// one at a time; the service's own mutex is never held with it.
// ---------------------------------------------------------------------------------------
struct bmpow_service {
  bmpow_batch* b = nullptr;  // resident session (ops run on the stepper thread, under g_mu)
  uint64_t budget = 0;       // trials per step (0 = library default)
  std::unique_ptr<bmsched::Service> svc;
};

namespace {

// Services not yet destroyed: bmpow_atexit stops their threads before it releases the devices.
std::mutex g_svc_mu;
std::vector<bmpow_service*> g_live_services;

// A service op finds the library shut down (bmpow_shutdown / resetPoW under a live service): an error
// the service reports through its poll, never a step on released devices.
int engine_gone(std::string& err) {
  err = "the library was shut down under this service";
  return BMPOW_E_STATE;
}

bmsched::ServiceOps service_ops(bmpow_service* s) {
  bmsched::ServiceOps ops;
  ops.add = [s](size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* tg, uint32_t* slots,
                std::string& err) {
    std::lock_guard<FairMutex> g(g_mu);
    if (!g_engine || s->b->dev.size() != g_shards.size()) return engine_gone(err);
    std::unique_lock<std::mutex> lk(g_engine->mu);
    const int rc = batch_add_locked(lk, s->b, n, ihs, tg, nullptr, slots, ih_off);
    if (rc < 0) err = g_err;
    return rc;
  };
  // let the steppers claim one round of launches (and keep one queued behind it) and return as soon
  // as an object finished, so the service hands it out while the devices go on
  ops.step = [s](std::string& err) {
    std::lock_guard<FairMutex> g(g_mu);
    if (!g_engine || s->b->dev.size() != g_shards.size()) return engine_gone(err);
    std::unique_lock<std::mutex> lk(g_engine->mu);
    g_engine->attach(lk, s->b);
    bmpow_batch* b = s->b;
    const uint64_t budget = (s->budget ? s->budget : g_step_trials.load()) * g_shards.size();
    // ... or as soon as a launch completes while another caller waits for the library (a serial run())
    return g_engine->run(lk, budget, true,
                         [b] { return b->finished_head < b->finished.size() || b->pending == 0 || g_mu.waiting() > 0; },
                         err);
  };
  ops.take = [s](size_t cap, uint32_t* slot, uint64_t* nonce, uint64_t* trial, uint8_t* done) -> size_t {
    std::lock_guard<FairMutex> g(g_mu);
    if (!g_engine) return 0;
    std::lock_guard<std::mutex> lk(g_engine->mu);
    return bmsched::take_done(*s->b, cap, slot, nonce, trial, done);
  };
  ops.reset = [s](std::string& err) {
    std::lock_guard<FairMutex> g(g_mu);
    if (!g_engine) return engine_gone(err);
    std::unique_lock<std::mutex> lk(g_engine->mu);
    if (g_engine->attached() == s->b) g_engine->detach(lk);
    batch_free_dev(s->b);
    delete s->b;
    s->b = new bmpow_batch();
    const int rc = batch_init(lk, s->b, 0, nullptr, nullptr, nullptr);
    if (rc < 0) err = g_err;
    return rc;
  };
  return ops;
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

int bmpow_init(void) {
  std::lock_guard<FairMutex> lk(g_mu);
  return init_locked();
}

int bmpow_device_count(void) { return (int)visible_gfx950().size(); }

int bmpow_set_devices(const int* ids, int n) {
  std::lock_guard<std::timed_mutex> one(g_one_mu);
  std::lock_guard<FairMutex> lk(g_mu);
  if (n < 0) return set_err(BMPOW_E_ARG, "bad device list");
  std::vector<int> v;
  if (n == 0) {
    v = visible_gfx950();
  } else if (!ids) {  // the first n visible devices (int bmpow_set_devices(int ndev))
    v = visible_gfx950();
    if ((size_t)n > v.size())
      return set_err(BMPOW_E_ARG, std::to_string(n) + " devices asked for, " + std::to_string(v.size()) + " visible");
    v.resize((size_t)n);
  } else {
    v.assign(ids, ids + n);
  }
  if (g_engine) {
    std::unique_lock<std::mutex> el(g_engine->mu);
    drop_scratch(el);
    g_engine->detach(el);
  }
  if (v.empty()) return set_err(BMPOW_E_NODEV, "no gfx950 (MI355X) device visible to the HIP runtime");
  int rc = select_devices(v);
  g_inited = rc > 0;
  return rc;
}

int bmpow_set_device_count(int ndev) {
  if (ndev < 1) return set_err(BMPOW_E_ARG, "device count must be >= 1");
  return bmpow_set_devices(nullptr, ndev);
}

int bmpow_get_devices(int* ids, int cap) {
  std::lock_guard<FairMutex> lk(g_mu);
  for (int i = 0; i < (int)g_shards.size() && i < cap; ++i) ids[i] = g_shards[i].dev;
  return (int)g_shards.size();
}

int bmpow_device_pci_bus_id(int device, char* out, int len) {
  if (!out || len < 13) return set_err(BMPOW_E_ARG, "buffer too small");
  const hipError_t e = hipDeviceGetPCIBusId(out, len, device);
  if (e != hipSuccess) return set_err(BMPOW_E_ARG, std::string("hipDeviceGetPCIBusId: ") + hipGetErrorString(e));
  return 0;
}

int bmpow_get_shard_rates(double* rates, int cap) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!rates && cap > 0) return set_err(BMPOW_E_ARG, "null pointer");
  if (!g_engine) return 0;
  std::lock_guard<std::mutex> el(g_engine->mu);
  const std::vector<double>& ema = g_engine->rates.ema;
  for (int i = 0; i < (int)g_shards.size() && i < cap; ++i) rates[i] = i < (int)ema.size() ? ema[i] : 0.0;
  return (int)g_shards.size();
}

static void shutdown_locked() {
  if (g_engine) {
    std::unique_lock<std::mutex> el(g_engine->mu);
    drop_scratch(el);
    g_engine->detach(el);
  }
  g_engine.reset();
  free_one();
  for (auto& s : g_shards) free_shard(s);
  g_shards.clear();
  if (g_xb) (void)hipHostFree(g_xb);
  g_xb = nullptr;
  g_inited = false;
}

void bmpow_shutdown(void) {
  std::lock_guard<std::timed_mutex> one(g_one_mu);
  std::lock_guard<FairMutex> lk(g_mu);
  shutdown_locked();
}

void bmpow_atexit(void) {
  // the services' threads step the engine: stopped (joined after their current op) first
  std::vector<bmpow_service*> live;
  {
    std::lock_guard<std::mutex> g(g_svc_mu);
    live = g_live_services;
  }
  for (bmpow_service* s : live) s->svc->stop();
  // a call still running in another thread (a daemon thread at interpreter exit) keeps the library
  std::unique_lock<std::timed_mutex> one(g_one_mu, std::chrono::milliseconds(5000));
  if (!one.owns_lock() || !g_mu.try_lock_for(std::chrono::milliseconds(5000))) return;
  if (!g_exited) {
    g_exited = true;
    shutdown_locked();
    // the streams kept for the life of the process (no stream is created after this: init refuses)
    for (const MaskedStream& m : g_masked) {
      (void)hipSetDevice(m.dev);
      (void)hipStreamSynchronize(m.stream);
      (void)hipStreamDestroy(m.stream);
    }
    g_masked.clear();
    for (const auto& r : g_run_streams) {
      (void)hipSetDevice(r.first);
      (void)hipStreamSynchronize(r.second);
      (void)hipStreamDestroy(r.second);
    }
    g_run_streams.clear();
  }
  g_mu.unlock();
}

const char* bmpow_last_error(void) { return g_err.c_str(); }

const char* bmpow_version(void) {
  static char buf[160];
  // BM_SRC_ID (the Makefile: an md5 of every source and header the library is built from) identifies
  // the library a bench line or profile came from; no build time, so a rebuild of the same sources in
  // the same tree gives the same file (bench.py compares the PMC passes' library md5 with the benched one)
#ifndef BM_SRC_ID
#define BM_SRC_ID "unknown"
#endif
  std::snprintf(buf, sizeof buf, "bmpow %d gfx950 block=%d iters=%d src %s", BMPOW_ABI_VERSION, BM_BLOCK, BM_ITERS,
                BM_SRC_ID);
  return buf;
}

void bmpow_abort(void) { g_abort.store(1); }
void bmpow_clear_abort(void) { g_abort.store(0); }

int bmpow_trials_len(const uint8_t* ih, size_t ih_len, const uint64_t* nonces, size_t n, uint64_t* trials_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if ((!ih && ih_len) || (n && (!nonces || !trials_out))) return set_err(BMPOW_E_ARG, "null pointer");
  if (ih_len > BMPOW_MAX_IH_LEN) return set_err(BMPOW_E_ARG, "initialHash longer than BMPOW_MAX_IH_LEN");
  if (n == 0) return 0;
  Shard& sh = g_shards[0];
  HIPTRY(hipSetDevice(sh.dev));
  bm_obj o;
  std::vector<uint64_t> vpool;
  const uint8_t zero = 0;
  bmsched::pack_var(ih ? ih : &zero, ih_len, 0, &o, vpool);
  bm_obj* d_o = nullptr;
  uint64_t *d_n = nullptr, *d_t = nullptr, *d_v = nullptr;
  HIPTRY(hipMalloc(&d_o, sizeof(bm_obj)));
  HIPTRY(hipMalloc(&d_n, n * sizeof(uint64_t)));
  HIPTRY(hipMalloc(&d_t, n * sizeof(uint64_t)));
  if (!vpool.empty()) HIPTRY(hipMalloc(&d_v, vpool.size() * sizeof(uint64_t)));
  hipError_t e = hipMemcpyAsync(d_o, &o, sizeof o, hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess && d_v)
    e = hipMemcpyAsync(d_v, vpool.data(), vpool.size() * sizeof(uint64_t), hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_n, nonces, n * sizeof(uint64_t), hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = bm_launch_trials(sh.stream, d_o, d_n, n, d_t, d_v);
  if (e == hipSuccess) e = hipMemcpyAsync(trials_out, d_t, n * sizeof(uint64_t), hipMemcpyDeviceToHost, sh.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
  (void)hipFree(d_o);
  (void)hipFree(d_n);
  (void)hipFree(d_t);
  if (d_v) (void)hipFree(d_v);
  if (e != hipSuccess) return set_err(BMPOW_E_HIP, std::string("bmpow_trials: ") + hipGetErrorString(e));
  return 0;
}

int bmpow_trials(const uint8_t ih[64], const uint64_t* nonces, size_t n, uint64_t* trials_out) {
  if (!ih) return set_err(BMPOW_E_ARG, "null pointer");
  return bmpow_trials_len(ih, 64, nonces, n, trials_out);
}

int bmpow_search(const uint8_t ih[64], uint64_t target, uint64_t start, uint64_t max_trials,
                 uint64_t* nonce_out, uint64_t* trial_out) {
  if (!ih) return set_err(BMPOW_E_ARG, "null pointer");
  return bmpow_search_len(ih, 64, target, start, max_trials, nonce_out, trial_out);
}

int bmpow_search_len(const uint8_t* ih, size_t ih_len, uint64_t target, uint64_t start, uint64_t max_trials,
                     uint64_t* nonce_out, uint64_t* trial_out) {
  std::lock_guard<std::timed_mutex> one(g_one_mu);
  std::unique_lock<FairMutex> g(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if ((!ih && ih_len) || !nonce_out || !trial_out) return set_err(BMPOW_E_ARG, "null pointer");
  if (ih_len > BMPOW_MAX_IH_LEN) return set_err(BMPOW_E_ARG, "initialHash longer than BMPOW_MAX_IH_LEN");
  if (max_trials == 0) return BMPOW_NOT_FOUND;
  if (g_abort.load()) return set_err(BMPOW_E_ABORTED, "aborted");
  // every 64-byte object takes the single-object path, on any number of devices (round 5; before, only
  // one shard did and several took the engine's split windows)
  if (ih_len == 64 && g_one_enabled) return search_one(ih, target, start, max_trials, nonce_out, trial_out, g);
  const uint8_t zero = 0;
  const uint64_t off[2] = {0, ih_len};
  std::unique_lock<std::mutex> lk(g_engine->mu);
  rc = scratch_batch(lk, 1, ih ? ih : &zero, &target, &start, ih_len == 64 ? nullptr : off);
  if (rc < 0) return rc;
  bmpow_batch* b = g_scratch;
  // the search's last nonce: windows are cut there, so a hit past the caller's budget is never
  // reported (it resumes at start + max_trials and finds it again)
  b->lim[0] = (max_trials - 1 > kU64Max - start) ? kU64Max : start + max_trials - 1;
  std::string err;
  rc = g_engine->run(lk, kU64Max, false, [b] { return b->done[0] != BMPOW_PENDING; }, err);
  if (rc < 0) return set_err(rc, err);
  if (b->done[0] == BMPOW_DONE_FOUND) {
    *nonce_out = b->nonce[0];
    *trial_out = b->trial[0];
    return BMPOW_FOUND;
  }
  return BMPOW_NOT_FOUND;
}

int bmpow_min_trial(const uint8_t ih[64], uint64_t start, uint64_t count, uint64_t* min_out, uint64_t* argmin_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (!ih || !min_out || !argmin_out) return set_err(BMPOW_E_ARG, "null pointer");
  return min_trial_locked(1, ih, &start, &count, min_out, argmin_out);
}

int bmpow_min_trial_batch(size_t n, const uint8_t* ihs, const uint64_t* start, const uint64_t* count,
                          uint64_t* min_out, uint64_t* argmin_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!ihs || !start || !count || !min_out || !argmin_out) return set_err(BMPOW_E_ARG, "null pointer");
  return min_trial_locked(n, ihs, start, count, min_out, argmin_out);
}

// shared argument check of the *_var entry points: n + 1 ascending offsets, lengths in range
static int check_ih_offsets(size_t n, const uint8_t* ihs, const uint64_t* ih_off) {
  if (!ih_off || (!ihs && ih_off[n] > ih_off[0])) return set_err(BMPOW_E_ARG, "null pointer");
  for (size_t i = 0; i < n; ++i) {
    if (ih_off[i + 1] < ih_off[i]) return set_err(BMPOW_E_ARG, "initialHash offsets are not ascending");
    if (ih_off[i + 1] - ih_off[i] > BMPOW_MAX_IH_LEN)
      return set_err(BMPOW_E_ARG, "initialHash longer than BMPOW_MAX_IH_LEN");
  }
  return 0;
}

int bmpow_min_trial_var(size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* start,
                        const uint64_t* count, uint64_t* min_out, uint64_t* argmin_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!start || !count || !min_out || !argmin_out) return set_err(BMPOW_E_ARG, "null pointer");
  rc = check_ih_offsets(n, ihs, ih_off);
  if (rc < 0) return rc;
  const uint8_t zero = 0;
  return min_trial_locked(n, ihs ? ihs : &zero, start, count, min_out, argmin_out, ih_off);
}

int bmpow_search_batch(size_t n, const uint8_t* ihs, const uint64_t* targets, uint64_t* next_start,
                       uint64_t budget, uint64_t* nonce_out, uint64_t* trial_out, uint8_t* done) {
  std::lock_guard<FairMutex> g(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!ihs || !targets || !next_start || !nonce_out || !trial_out || !done)
    return set_err(BMPOW_E_ARG, "null pointer");
  if (g_abort.load()) return set_err(BMPOW_E_ABORTED, "aborted");
  std::unique_lock<std::mutex> lk(g_engine->mu);
  rc = scratch_batch(lk, n, ihs, targets, next_start);
  if (rc < 0) return rc;
  bmpow_batch* b = g_scratch;
  for (size_t i = 0; i < n; ++i) {
    if (done[i] != BMPOW_PENDING) {
      b->done[i] = done[i];
      b->pending--;
    }
  }
  if (budget == 0) budget = g_step_trials * g_shards.size();
  // no lookahead: every claim is applied when the call returns, so next_start is where the batch stands
  std::string err;
  rc = g_engine->run(lk, budget, false, [b] { return b->pending == 0; }, err);
  if (rc < 0) return set_err(rc, err);
  for (size_t i = 0; i < n; ++i) {
    if (done[i] != BMPOW_PENDING) continue;
    done[i] = b->done[i];
    next_start[i] = bmsched::resume_point(*b, i);
    if (b->done[i] == BMPOW_DONE_FOUND) {
      nonce_out[i] = b->nonce[i];
      trial_out[i] = b->trial[i];
    }
  }
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

bmpow_batch* bmpow_batch_create(size_t n, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start) {
  std::lock_guard<FairMutex> g(g_mu);
  if (init_locked() < 0) return nullptr;
  if (n && (!ihs || !targets)) {
    set_err(BMPOW_E_ARG, "null pointer");
    return nullptr;
  }
  if (n > 0xffffffffULL) {
    set_err(BMPOW_E_ARG, "too many objects");
    return nullptr;
  }
  std::unique_lock<std::mutex> lk(g_engine->mu);
  bmpow_batch* b = new bmpow_batch();
  if (batch_init(lk, b, n, ihs, targets, start) < 0) {
    batch_free_dev(b);
    delete b;
    return nullptr;
  }
  return b;
}

// Let the steppers claim ~budget trials of the batch (and one more launch per shard, which stays
// queued behind the running one when this returns, so consecutive calls keep every device busy).
int bmpow_batch_step(bmpow_batch* b, uint64_t budget) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (!g_engine) return set_err(BMPOW_E_STATE, "library not initialised");
  if (b->dev.size() != g_shards.size()) return set_err(BMPOW_E_STATE, "device set changed under a live batch");
  if (g_abort.load()) return set_err(BMPOW_E_ABORTED, "aborted");
  std::unique_lock<std::mutex> lk(g_engine->mu);
  g_engine->attach(lk, b);
  if (budget == 0) budget = g_step_trials.load() * g_shards.size();
  std::string err;
  const int rc = g_engine->run(lk, budget, true, [b] { return b->pending == 0; }, err);
  if (rc < 0) return set_err(rc, err);
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_results(const bmpow_batch* b, uint64_t* nonce_out, uint64_t* trial_out, uint8_t* done,
                        uint64_t* next_start) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  std::unique_lock<std::mutex> lk;
  if (g_engine) lk = std::unique_lock<std::mutex>(g_engine->mu);
  for (size_t i = 0; i < b->n; ++i) {
    if (nonce_out) nonce_out[i] = b->nonce[i];
    if (trial_out) trial_out[i] = b->trial[i];
    if (done) done[i] = b->done[i];
    if (next_start) next_start[i] = bmsched::resume_point(*b, i);
  }
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_reset(bmpow_batch* b, const uint64_t* start) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (b->dev.size() != g_shards.size() || !g_engine) return set_err(BMPOW_E_STATE, "device set changed under a live batch");
  std::unique_lock<std::mutex> lk(g_engine->mu);
  quiesce(lk, b);
  bmsched::reset(*b, start);
  for (size_t s = 0; s < g_shards.size(); ++s) {
    Shard& sh = g_shards[s];
    HIPTRY(hipSetDevice(sh.dev));
    if (b->n) HIPTRY(hipMemsetAsync(b->dev[s].d_best, 0xFF, b->n * sizeof(unsigned long long), sh.stream));
    if (b->n) HIPTRY(hipMemsetAsync(b->dev[s].d_found, 0, b->n * sizeof(uint32_t), sh.stream));
  }
  for (auto& sh : g_shards) {
    HIPTRY(hipSetDevice(sh.dev));
    HIPTRY(hipStreamSynchronize(sh.stream));
  }
  g_engine->notify();
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_set_pending(bmpow_batch* b, size_t first, size_t count, int pending) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (first > b->n || count > b->n - first) return set_err(BMPOW_E_ARG, "range outside the batch");
  std::unique_lock<std::mutex> lk;
  if (g_engine) lk = std::unique_lock<std::mutex>(g_engine->mu);
  bmsched::set_pending(*b, first, count, pending != 0);
  if (g_engine) g_engine->notify();
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_add(bmpow_batch* b, size_t n, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
                    uint32_t* slot_out) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (n == 0) return (int)std::min<size_t>(b->pending, 0x7fffffff);
  if (!ihs || !targets) return set_err(BMPOW_E_ARG, "null pointer");
  if (!g_engine) return set_err(BMPOW_E_STATE, "library not initialised");
  std::unique_lock<std::mutex> lk(g_engine->mu);
  const int rc = batch_add_locked(lk, b, n, ihs, targets, start, slot_out);
  if (rc < 0) return rc;
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_add_var(bmpow_batch* b, size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* targets,
                        const uint64_t* start, uint32_t* slot_out) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (n == 0) return (int)std::min<size_t>(b->pending, 0x7fffffff);
  if (!targets) return set_err(BMPOW_E_ARG, "null pointer");
  if (!g_engine) return set_err(BMPOW_E_STATE, "library not initialised");
  int rc = check_ih_offsets(n, ihs, ih_off);
  if (rc < 0) return rc;
  const uint8_t zero = 0;
  std::unique_lock<std::mutex> lk(g_engine->mu);
  rc = batch_add_locked(lk, b, n, ihs ? ihs : &zero, targets, start, slot_out, ih_off);
  if (rc < 0) return rc;
  return (int)std::min<size_t>(b->pending, 0x7fffffff);
}

int bmpow_batch_take_done(bmpow_batch* b, size_t cap, uint32_t* slot_out, uint64_t* nonce_out, uint64_t* trial_out,
                          uint8_t* done_out) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return set_err(BMPOW_E_STATE, "null batch");
  if (cap && !slot_out) return set_err(BMPOW_E_ARG, "null pointer");
  std::unique_lock<std::mutex> lk;
  if (g_engine) lk = std::unique_lock<std::mutex>(g_engine->mu);
  const size_t k = bmsched::take_done(*b, std::min<size_t>(cap, 0x7fffffff), slot_out, nonce_out, trial_out, done_out);
  return (int)k;
}

void bmpow_batch_destroy(bmpow_batch* b) {
  std::lock_guard<FairMutex> g(g_mu);
  if (!b) return;
  if (g_engine) {
    std::unique_lock<std::mutex> lk(g_engine->mu);
    if (g_engine->attached() == b) g_engine->detach(lk);
  }
  batch_free_dev(b);
  delete b;
}

bmpow_service* bmpow_service_create(uint64_t step_budget, uint32_t flags) {
  bmpow_service* s = new bmpow_service();
  {
    std::lock_guard<FairMutex> g(g_mu);
    s->b = new bmpow_batch();
    if (init_locked() < 0) {
      delete s->b;
      delete s;
      return nullptr;
    }
    std::unique_lock<std::mutex> lk(g_engine->mu);
    if (batch_init(lk, s->b, 0, nullptr, nullptr, nullptr) < 0) {
      batch_free_dev(s->b);
      delete s->b;
      delete s;
      return nullptr;
    }
    s->budget = step_budget;
  }
  s->svc.reset(new bmsched::Service(service_ops(s), (flags & BMPOW_SERVICE_VERIFY) != 0));
  std::lock_guard<std::mutex> g(g_svc_mu);
  g_live_services.push_back(s);
  return s;
}

int bmpow_service_submit(bmpow_service* s, size_t n, const uint8_t* ihs, const uint64_t* targets,
                         uint64_t* tickets_out) {
  if (!s) return set_err(BMPOW_E_STATE, "null service");
  if (n && (!ihs || !targets)) return set_err(BMPOW_E_ARG, "null pointer");
  const int rc = s->svc->submit(n, ihs, targets, tickets_out);
  return rc < 0 ? set_err(rc, "service stopping") : rc;
}

int bmpow_service_submit_var(bmpow_service* s, size_t n, const uint8_t* ihs, const uint64_t* ih_off,
                             const uint64_t* targets, uint64_t* tickets_out) {
  if (!s) return set_err(BMPOW_E_STATE, "null service");
  if (n == 0) return 0;
  if (!targets) return set_err(BMPOW_E_ARG, "null pointer");
  int rc = check_ih_offsets(n, ihs, ih_off);
  if (rc < 0) return rc;
  const uint8_t zero = 0;
  rc = s->svc->submit(n, ihs ? ihs : &zero, targets, tickets_out, ih_off);
  return rc < 0 ? set_err(rc, "service stopping") : rc;
}

int bmpow_service_poll(bmpow_service* s, size_t cap, int timeout_ms, uint64_t* tickets, uint64_t* nonce_out,
                       uint64_t* trial_out, uint8_t* done_out) {
  if (!s) return set_err(BMPOW_E_STATE, "null service");
  if (cap && !tickets) return set_err(BMPOW_E_ARG, "null pointer");
  std::string err;
  const int rc = s->svc->poll(cap, timeout_ms, tickets, nonce_out, trial_out, done_out, err);
  if (rc < 0) g_err = err;
  return rc;
}

int bmpow_service_cancel(bmpow_service* s) {
  if (!s) return set_err(BMPOW_E_STATE, "null service");
  s->svc->cancel();
  return 0;
}

int bmpow_service_outstanding(bmpow_service* s) {
  if (!s) return set_err(BMPOW_E_STATE, "null service");
  return (int)std::min<size_t>(s->svc->outstanding(), 0x7fffffff);
}

void bmpow_service_stop(bmpow_service* s) {
  if (s) s->svc->stop();
}

void bmpow_service_destroy(bmpow_service* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(g_svc_mu);
    g_live_services.erase(std::remove(g_live_services.begin(), g_live_services.end(), s), g_live_services.end());
  }
  s->svc.reset();  // joins the service thread after its current op
  std::lock_guard<FairMutex> g(g_mu);
  if (g_engine) {
    std::unique_lock<std::mutex> lk(g_engine->mu);
    if (g_engine->attached() == s->b) g_engine->detach(lk);
  }
  batch_free_dev(s->b);
  delete s->b;
  delete s;
}

bmpow_vbatch* bmpow_vbatch_create(size_t n, const uint8_t* objs, const uint64_t* offsets) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (init_locked() < 0) return nullptr;
  std::vector<Span> spans;
  if (spans_from(n, objs, offsets, spans) < 0) return nullptr;
  bmpow_vbatch* vb = new bmpow_vbatch();
  if (vbatch_build(vb, spans) < 0) {
    vbatch_free(vb);
    delete vb;
    return nullptr;
  }
  return vb;
}

int bmpow_vbatch_run(bmpow_vbatch* vb, uint64_t* pow_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!vb) return set_err(BMPOW_E_STATE, "null verification batch");
  for (auto& pt : vb->parts)
    if (pt.shard >= g_shards.size()) return set_err(BMPOW_E_STATE, "device set changed under a live batch");
  return vbatch_run_locked(vb, pow_out);
}

void bmpow_vbatch_destroy(bmpow_vbatch* vb) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!vb) return;
  vbatch_free(vb);
  delete vb;
}

int bmpow_pow_values(size_t n, const uint8_t* objs, const uint64_t* offsets, uint64_t* pow_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!pow_out) return set_err(BMPOW_E_ARG, "null pointer");
  std::vector<Span> spans;
  rc = spans_from(n, objs, offsets, spans);
  if (rc < 0) return rc;
  bmpow_vbatch vb;
  rc = vbatch_build(&vb, spans, true);
  if (rc == 0) rc = vbatch_run_locked(&vb, pow_out);
  vbatch_release_plan(&vb);
  vbatch_free(&vb);
  return rc;
}

// shared by both verify entry points (internal linkage despite the extern "C" block)
static int verify_spans_locked(size_t n, const uint8_t* const* ptrs, const uint64_t* lens, const uint64_t* ntpb,
                               const uint64_t* extra, const int64_t* recv_time, uint8_t* ok_out) {
  // scratch kept across calls under g_mu (a flood's worth of fresh pages costs several ms)
  static std::vector<Span> spans;
  static std::vector<size_t> idx;
  static std::vector<uint64_t> pow, eol;
  spans.clear();
  idx.clear();
  spans.reserve(n);
  idx.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if ((ntpb && ntpb[i] >= (1ULL << 62)) || (extra && extra[i] >= (1ULL << 62)))
      return set_err(BMPOW_E_ARG, "nonceTrialsPerByte / payloadLengthExtraBytes above 2^62");
    if (lens[i] < 16) {
      ok_out[i] = 2;  // the reference's unpack('>Q', data[8:16]) raises struct.error
      continue;
    }
    if (!ptrs[i]) return set_err(BMPOW_E_ARG, "null object pointer");
    spans.push_back({ptrs[i], lens[i]});
    idx.push_back(i);
  }
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const clk::time_point t0 = clk::now();
  pow.resize(spans.size());
  eol.resize(spans.size());
  if (!spans.empty()) {
    bmpow_vbatch vb;
    int rc = vbatch_build(&vb, spans, true);
    const clk::time_point t1 = clk::now();
    if (rc == 0) rc = vbatch_run_locked(&vb, pow.data());
    g_stats.verify_host_build_ms += ms(t0, t1);
    g_stats.verify_host_run_ms += ms(t1, clk::now());
    for (const auto& pt : vb.parts)  // expiresTime, read by the padding pass
      for (size_t j = 0; j < pt.orig.size(); ++j) eol[pt.orig[j]] = pt.eol[j];
    vbatch_release_plan(&vb);
    vbatch_free(&vb);
    if (rc < 0) return rc;
  }
  const clk::time_point t2 = clk::now();
  const int64_t now = (int64_t)std::time(nullptr);
  bmsched::parallel_for(spans.size(), 32768, [&](size_t a, size_t b) {
    for (size_t j = a; j < b; ++j) {
      const size_t i = idx[j];
      const int64_t recv = (recv_time && recv_time[i]) ? recv_time[i] : now;
      ok_out[i] = (uint8_t)pow_sufficient(pow[j], spans[j].len, ntpb ? ntpb[i] : 0, extra ? extra[i] : 0, recv, eol[j]);
    }
  });
  g_stats.verify_host_verdict_ms += ms(t2, clk::now());
  return 0;
}

int bmpow_verify_batch(size_t n, const uint8_t* objs, const uint64_t* offsets, const uint64_t* ntpb,
                       const uint64_t* extra, const int64_t* recv_time, uint8_t* ok_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!objs || !offsets || !ok_out) return set_err(BMPOW_E_ARG, "null pointer");
  std::vector<const uint8_t*> ptrs(n);
  std::vector<uint64_t> lens(n);
  for (size_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) return set_err(BMPOW_E_ARG, "offsets are not ascending");
    ptrs[i] = objs + offsets[i];
    lens[i] = offsets[i + 1] - offsets[i];
  }
  return verify_spans_locked(n, ptrs.data(), lens.data(), ntpb, extra, recv_time, ok_out);
}

int bmpow_verify_batch_ptrs(size_t n, const uint8_t* const* objs, const uint64_t* lens, const uint64_t* ntpb,
                            const uint64_t* extra, const int64_t* recv_time, uint8_t* ok_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!objs || !lens || !ok_out) return set_err(BMPOW_E_ARG, "null pointer");
  return verify_spans_locked(n, objs, lens, ntpb, extra, recv_time, ok_out);
}

int bmpow_pow_sufficient(uint64_t pow, uint64_t len, uint64_t ntpb, uint64_t extra, int64_t recv_time,
                         uint64_t expires) {
  if (ntpb >= (1ULL << 62) || extra >= (1ULL << 62)) return set_err(BMPOW_E_ARG, "difficulty above 2^62");
  return pow_sufficient(pow, len, ntpb, extra, recv_time ? recv_time : (int64_t)std::time(nullptr), expires);
}

int bmpow_pubkeys(size_t n, const uint8_t* privkeys, uint8_t* pubkeys_out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!privkeys || !pubkeys_out) return set_err(BMPOW_E_ARG, "null pointer");
  if (n > 0xffffffffULL) return set_err(BMPOW_E_ARG, "too many keys");
  Shard& sh = g_shards[0];
  rc = ensure_table(sh, 0);
  if (rc < 0) return rc;
  std::vector<uint64_t> w(4 * n);
  for (size_t i = 0; i < n; ++i) {
    uint64_t k[4];
    be_words_from_bytes(privkeys + 32 * i, k);
    for (int j = 0; j < 4; ++j) w[4 * i + j] = k[j];
  }
  std::vector<ec::ge> pubs(n);
  std::vector<uint32_t> ok(n);
  uint64_t* d_w = nullptr;
  ec::ge* d_p = nullptr;
  uint32_t* d_ok = nullptr;
  HIPTRY(hipSetDevice(sh.dev));
  hipError_t e = hipMalloc(&d_w, w.size() * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&d_p, n * sizeof(ec::ge));
  if (e == hipSuccess) e = hipMalloc(&d_ok, n * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpyAsync(d_w, w.data(), w.size() * sizeof(uint64_t), hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = ar_launch_pubkeys(sh.stream, d_w, (uint32_t)n, sh.d_table[0], d_p, d_ok);
  if (e == hipSuccess) e = hipMemcpyAsync(pubs.data(), d_p, n * sizeof(ec::ge), hipMemcpyDeviceToHost, sh.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(ok.data(), d_ok, n * sizeof(uint32_t), hipMemcpyDeviceToHost, sh.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
  (void)hipFree(d_w);
  (void)hipFree(d_p);
  (void)hipFree(d_ok);
  if (e != hipSuccess) return set_err(BMPOW_E_HIP, std::string("bmpow_pubkeys: ") + hipGetErrorString(e));
  for (size_t i = 0; i < n; ++i) {
    if (ok[i]) point_bytes(pubs[i], pubkeys_out + 65 * i);
    else std::memset(pubkeys_out + 65 * i, 0, 65);
  }
  return 0;
}

int bmpow_fe_probe(int op, size_t n, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  if (n == 0) return 0;
  if (!a || !b || !out) return set_err(BMPOW_E_ARG, "null pointer");
  if (op < 0 || op > 6) return set_err(BMPOW_E_ARG, "fe probe op must be 0..6");
  if (n > (1u << 24)) return set_err(BMPOW_E_ARG, "too many operands");
  Shard& sh = g_shards[0];
  const size_t bytes = n * sizeof(ec::fe);
  ec::fe *d_a = nullptr, *d_b = nullptr, *d_o = nullptr;
  HIPTRY(hipSetDevice(sh.dev));
  hipError_t e = hipMalloc(&d_a, bytes);
  if (e == hipSuccess) e = hipMalloc(&d_b, bytes);
  if (e == hipSuccess) e = hipMalloc(&d_o, bytes);
  if (e == hipSuccess) e = hipMemcpyAsync(d_a, a, bytes, hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d_b, b, bytes, hipMemcpyHostToDevice, sh.stream);
  if (e == hipSuccess) e = ar_launch_fe_probe(sh.stream, op, d_a, d_b, d_o, (uint32_t)n);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_o, bytes, hipMemcpyDeviceToHost, sh.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
  (void)hipFree(d_a);
  (void)hipFree(d_b);
  (void)hipFree(d_o);
  if (e != hipSuccess) return set_err(BMPOW_E_HIP, std::string("bmpow_fe_probe: ") + hipGetErrorString(e));
  return 0;
}

int bmpow_address_search(const uint8_t* passphrase, size_t len, uint64_t start, uint64_t max_tries, int null_bytes,
                         bmpow_address* out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  std::vector<AddrShard> as;
  rc = addr_search_locked(0, passphrase, len, nullptr, start, max_tries, null_bytes, out, as);
  addr_free(as);
  return rc;
}

int bmpow_address_search_random(const uint8_t priv_signing[32], const uint8_t* seed, size_t seed_len, uint64_t start,
                                uint64_t max_tries, int null_bytes, bmpow_address* out) {
  std::lock_guard<FairMutex> lk(g_mu);
  int rc = init_locked();
  if (rc < 0) return rc;
  std::vector<AddrShard> as;
  rc = addr_search_locked(1, seed, seed_len, priv_signing, start, max_tries, null_bytes, out, as);
  addr_free(as);
  return rc;
}

int bmpow_addr_set_comb(int wbits) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (wbits != 0 && wbits != ec::kCombSmall && wbits != ec::kCombLarge)
    return set_err(BMPOW_E_ARG, "comb width must be 0 (auto), 16 or 24");
  const int prev = g_addr_comb;
  g_addr_comb = wbits;
  return prev;
}

int bmpow_addr_last_comb(void) {
  std::lock_guard<FairMutex> lk(g_mu);
  return g_addr_last_comb;
}

int bmpow_get_stats(bmpow_stats* out) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!out) return BMPOW_E_ARG;
  *out = g_stats;
  out->masked_streams = g_masked.size();
  out->run_streams = g_run_streams.size();
  if (g_engine) {  // the searches: the engine's launches
    std::lock_guard<std::mutex> el(g_engine->mu);
    const bmsched::EngineStats& es = g_engine->stats;
    out->launches += es.launches;
    out->trials += es.trials;
    out->kernel_ms += es.kernel_ms;
    out->steps += es.launches;
    double mx = 0;
    for (double ms : es.shard_ms) mx = std::max(mx, ms);
    out->max_shard_kernel_ms += mx;
    out->past_window += es.waste.window;
    out->past_later += es.waste.later;
    out->past_split += es.waste.split;
    out->engine_hashed_est += es.waste.hashed;
  }
  return 0;
}

void bmpow_reset_stats(void) {
  std::lock_guard<FairMutex> lk(g_mu);
  g_stats = bmpow_stats{};
  for (OnePath& op : g_ones) {
    op.trials = 0;
    op.ms = 0;
  }
  if (g_engine) {
    std::lock_guard<std::mutex> el(g_engine->mu);
    bmsched::EngineStats& es = g_engine->stats;
    const size_t S = es.shard_ms.size();
    es = bmsched::EngineStats();
    es.shard_ms.assign(S, 0.0);
    es.shard_trials.assign(S, 0);
  }
}

int bmpow_get_shard_stats(uint64_t* trials, double* kernel_ms, int cap) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!g_engine) return 0;
  std::lock_guard<std::mutex> el(g_engine->mu);
  const bmsched::EngineStats& es = g_engine->stats;
  for (int i = 0; i < (int)es.shard_ms.size() && i < cap; ++i) {
    // the engine's launches and run()'s single-object pieces on the shard
    const bool one = i < (int)g_ones.size();
    if (trials) trials[i] = es.shard_trials[i] + (one ? g_ones[i].trials : 0);
    if (kernel_ms) kernel_ms[i] = es.shard_ms[i] + (one ? g_ones[i].ms : 0);
  }
  return (int)g_shards.size();
}

int bmpow_set_run_split(int per_shard) {
  std::lock_guard<std::timed_mutex> one(g_one_mu);
  std::lock_guard<FairMutex> lk(g_mu);
  const int prev = g_run_split ? 1 : 0;
  if (per_shard < 0) return prev;
  if ((per_shard != 0) != g_run_split) {
    // a shard that carries no piece misses the ring resets of the calls it sits out: start afresh
    free_one();
    g_run_split = per_shard != 0;
  }
  return prev;
}

int bmpow_set_engine_split(int per_shard) {
  std::lock_guard<FairMutex> lk(g_mu);
  const int prev = g_engine_split ? 1 : 0;
  if (per_shard < 0) return prev;
  if ((per_shard != 0) != g_engine_split) {
    g_engine_split = per_shard != 0;
    apply_engine_groups();
  }
  return prev;
}

int bmpow_get_run_pieces(int* shards, int cap) {
  std::lock_guard<FairMutex> lk(g_mu);
  const int rc = init_locked();
  if (rc < 0) return rc;
  const std::vector<size_t> p = one_pieces();
  for (int i = 0; i < (int)p.size() && i < cap; ++i)
    if (shards) shards[i] = (int)p[i];
  return (int)p.size();
}

int bmpow_get_thread_info(double* cpu_s, int* policy, int cap) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!g_engine) return 0;
  std::vector<double> c;
  std::vector<int> p;
  {
    std::lock_guard<std::mutex> el(g_engine->mu);
    g_engine->thread_info(c, p);
  }
  for (int i = 0; i < (int)c.size() && i < cap; ++i) {
    if (cpu_s) cpu_s[i] = c[i];
    if (policy) policy[i] = p[i];
  }
  return (int)c.size();
}

int bmpow_set_shard_throttle(int shard, double ms) {
  std::lock_guard<FairMutex> lk(g_mu);
  if (!g_engine) return set_err(BMPOW_E_STATE, "library not initialised");
  if (shard < 0 || shard >= (int)g_shards.size() || !(ms >= 0)) return set_err(BMPOW_E_ARG, "bad shard or delay");
  g_engine->set_throttle((size_t)shard, ms);
  return 0;
}

uint64_t bmpow_get_step_trials(void) { return g_step_trials.load(); }

void bmpow_set_step_trials(uint64_t t) {
  std::lock_guard<FairMutex> lk(g_mu);
  g_step_trials.store(t ? std::max<uint64_t>(t, BM_CHUNK) : kDefaultStepTrials);
  if (g_engine) {
    std::lock_guard<std::mutex> el(g_engine->mu);
    g_engine->set_step_trials(g_step_trials.load());
  }
}

unsigned long long BitmessagePOW(unsigned char* starthash, unsigned long long target) {
  uint64_t start = 1, nonce = 0, tv = 0;
  for (;;) {
    const uint64_t budget = 1ULL << 34;
    int rc = bmpow_search(starthash, target, start, budget, &nonce, &tv);
    if (rc == BMPOW_FOUND) return nonce;
    if (rc < 0) return 0;
    if (start > kU64Max - budget) return 0;
    start += budget;
  }
}

}  // extern "C"
