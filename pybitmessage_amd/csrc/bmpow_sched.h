// bmpow_sched.h -- the host-only half of libbmpow_hip.so's scheduler: everything between the C ABI
// and the HIP calls that needs no device.  bmpow_host.hip drives the devices with it; the same
// source builds with g++ for the sanitizer tests (tests/native/: ThreadSanitizer, ASan/UBSan),
// which run it against a CPU stand-in for the kernels.
//
//   search         Engine: one stepper thread per shard claiming windows from the objects'
//                  frontiers (plan_launch -> launch -> wait -> apply_launch), no lockstep
//                  (bmpow_search*, bmpow_batch_step, the service)
//   sessions       init / add / take_done / reset / set_pending          (bmpow_batch_*)
//   min-trial      MinTrial::plan -> (launch) -> reduce_parts -> advance (bmpow_min_trial*)
//   verification   plan_verify, pad_range, pow_sufficient                (bmpow_verify*, bmpow_pow_values)
//   service        Service: stepper thread, submit / poll / cancel         (bmpow_service_*)
//
// Semantics reproduced: the reference's _doSafePoW first nonce (src/proofofwork.py:100-111) over
// contiguous windows per object, and protocol.isProofOfWorkSufficient (src/protocol.py:258-286).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <time.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bmpow.h"
#include "bmpow_layout.h"

namespace bmsched {

constexpr uint64_t kU64Max = ~0ULL;

uint64_t load_be64(const uint8_t* p);
// trial(nonce, ih) on the host (OpenSSL SHA-512): the re-check of device answers, never a search
uint64_t host_trial(const uint8_t ih[64], uint64_t nonce);
// the same for an initialHash of any length (src/proofofwork.py:106-107 hashes it as given)
uint64_t host_trial_len(const uint8_t* ih, size_t len, uint64_t nonce);
void pack_obj(const uint8_t* ih, uint64_t target, bm_obj* o);
// An object of any initialHash length: 64 bytes -> pack_obj; otherwise the var form, its message words
// appended to pool (block 0's 16 words, then K[t] + W[t] for t < 80 of every further block).
void pack_var(const uint8_t* ih, size_t len, uint64_t target, bm_obj* o, std::vector<uint64_t>& pool);
// Object i of a list given as concatenated bytes: 64 bytes each when off is null, else bytes
// [off[i], off[i+1]).
inline const uint8_t* ih_ptr(const uint8_t* ihs, const uint64_t* off, size_t i) { return ihs + (off ? off[i] : 64 * i); }
inline size_t ih_len(const uint64_t* off, size_t i) { return off ? (size_t)(off[i + 1] - off[i]) : 64; }

// A window of an object's nonce space [start, start + count), handed out in P interleaved pieces:
// piece p is columns [p G, (p + 1) G) of the window's P G columns (bmpow_layout.h: column c takes
// blocks c, c + P G, ...).  P = 1: one shard sweeps the whole window (an object owned by one
// device); P > 1: a window split over the shards, each piece claimed by whichever shard plans next,
// so every device sweeps the same rows of it.  Pieces are claimed in order; the window stays open
// until every piece has been applied.
struct OpenWin {
  uint64_t start, count;
  uint32_t G;                 // columns per piece
  uint16_t P, claimed, done;  // pieces: in all, handed out, applied
  uint16_t seq;               // the object's window number (BatchState::wseq; claimable's cap)
};

// One applied item whose share of the trials past the object's answer is not known yet (the answer
// was not final when it was applied): kept per object until it settles (BatchState::wrec).
struct WasteRec {
  uint64_t start, count;  // the window
  uint32_t g0, gn, nwg;   // the item's columns (bmpow_layout.h)
  uint32_t taken;         // units its block queue handed out (bm_result.pad, from the resolve kernel)
  uint16_t P;
};

// Trials hashed past the objects' answers, by where they were hashed (EngineStats; estimates from the
// block queues: every workgroup ends on one unit it takes and does not hash, so of the `taken` units
// handed out the first taken - nwg are counted as hashed).
struct WasteStats {
  uint64_t window = 0;  // unsplit windows holding the answer: blocks above it
  uint64_t later = 0;   // unsplit windows starting above the answer (the lookahead queued behind)
  uint64_t split = 0;   // pieces of split windows: blocks above the answer
  uint64_t hashed = 0;  // every item's estimated hashed nonces (checks the estimate against trials)
};

// Holder of an object's in-flight windows (BatchState::holder): none, one shard (its index), or
// several shards at once.
constexpr int16_t kNoHolder = -1, kShared = -2;

// Host mirror of a device-resident batch (one slot per object; slots of finished objects are
// released by take_done and reused by add).
struct BatchState {
  size_t n = 0;    // slots in the table (objects, finished ones and free slots included)
  size_t cap = 0;  // device allocation, in objects (set by the device side; add() reports growth)
  std::vector<bm_obj> objs;
  // next: the claim frontier (the first nonce no window covers yet); nonce/trial: the least hit
  // applied so far (the answer once done = FOUND)
  std::vector<uint64_t> next, nonce, trial;
  std::vector<uint8_t> done;
  size_t first_pending = 0;
  size_t pending = 0;
  std::vector<uint32_t> finished;  // slots finished since the last take_done, in finishing order
  size_t finished_head = 0;
  std::vector<uint32_t> free_slots;  // slots released by take_done, reused by add (LIFO)
  // var-form objects (initialHash length != 64): their words, appended by add; emptied by add when
  // no slot holds a var object any more (vpool_epoch then counts up, so the device copy restarts)
  std::vector<uint64_t> vpool;
  size_t nvar_slots = 0;  // non-free slots holding a var-form object
  size_t vlive = 0;       // words of vpool those slots use (the rest belong to released slots)
  uint64_t vpool_epoch = 0;
  // slots whose var-form words add() moved (a compaction of vpool, which also starts a new epoch):
  // their device records (vword) must be rewritten before the next launch
  std::vector<uint32_t> vmoved;
  // ---- the claim frontier of per-device stepping (Engine, plan_launch / apply_launch) ----
  std::vector<uint32_t> gen;     // bumped whenever the slot's search restarts: older launches are stale
  std::vector<uint64_t> lim;     // last nonce a window may reach (inclusive): a bounded search's end
  std::vector<uint8_t> hit;      // an applied window reported a hit (nonce/trial hold the least)
  std::vector<uint8_t> top;      // the frontier passed lim: no window left to create
  std::vector<int16_t> holder;   // shard holding the object's in-flight items, kNoHolder or kShared
  std::vector<uint32_t> nfly;    // the object's items in flight
  std::vector<uint8_t> xs;       // cross-shard bound slot + 1 while the object is shared, 0 none
  // shards with items of the object in flight (a shard has at most two: its running and staged
  // launch): bit s of fly1 = at least one, of fly2 = two
  std::vector<uint64_t> fly1, fly2;
  std::vector<std::vector<OpenWin>> open;  // windows not yet fully applied, ascending start
  std::vector<uint16_t> wseq;    // the number the object's next window gets (wraps; only differences count)
  std::vector<std::vector<WasteRec>> wrec;  // applied items not yet priced against the final answer
  bool broken = false;           // a launch was lost to a device error: only reset() continues it
};

// ih_off: null (n x 64-byte initialHashes) or n + 1 byte offsets into ihs (any lengths)
void init(BatchState& b, size_t n, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
          const uint64_t* ih_off = nullptr);

// Append m objects (slots reused first).  slots[i] = object i's slot.  Returns true when the table
// outgrew b.cap (the caller reallocates and re-uploads); false when only `slots` need uploading.
// Var-form words of released slots are reclaimed: once they outnumber the live ones (and 64 Ki
// words), the pool is repacked -- live objects' words moved down, their vword updated and their
// slots listed in b.vmoved, a new vpool_epoch -- so a service fed steady non-64-byte objects keeps
// a pool of about twice its live words.
bool add(BatchState& b, size_t m, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
         std::vector<uint32_t>& slots, const uint64_t* ih_off = nullptr);

// Pop up to cap finished slots (any output but slot_out may be null); they become BMPOW_FREE.
size_t take_done(BatchState& b, size_t cap, uint32_t* slot_out, uint64_t* nonce_out, uint64_t* trial_out,
                 uint8_t* done_out);

void reset(BatchState& b, const uint64_t* start);  // released slots stay free
void set_pending(BatchState& b, size_t first, size_t count, bool pending);

// One object's contiguous nonce window in a step: `chunks` chunks from chunk index `chunk0` of the
// step's flattened chunk list.
struct Win {
  uint32_t obj;
  uint64_t start, count, chunks, chunk0;
};

struct StepPlan {
  uint32_t iters = 0;   // planning unit: chunk = BM_BLOCK x iters nonces (a window is whole chunks)
  uint64_t chunk = 0;
  uint64_t C = 0;       // chunks planned in the step
  std::vector<Win> wins;                    // ascending object order
  std::vector<std::vector<bm_item>> items;  // per shard, ascending chunk_base
  std::vector<uint32_t> nchunks;            // per shard: workgroups of its launch(es)
  // after split_kinds: per shard, items[s][0, nmain[s]) are 64-byte objects (bm_search_kernel, chunk_base
  // from 0, chmain[s] workgroups) and the rest var-form objects (bm_search_var_kernel, chunk_base again
  // from 0)
  std::vector<uint32_t> nmain, chmain;
  uint32_t nx = 0;  // windows split over the shards: cross-shard bound slots [0, nx) (bmpow_layout.h)
};

// Reorder each shard's items into the two kernels' launches (see StepPlan); with any_var false every
// item is 64-byte and nothing moves.
void split_kinds(const std::vector<bm_obj>& objs, bool any_var, StepPlan& p);

// Deal windows (C chunks, ascending chunk0) to S shards as work items (bmpow_layout.h): the flattened
// chunk list is cut into S contiguous slices and each (window, shard) piece is one item whose
// workgroups take its blocks in order; a piece gets one workgroup per g_blocks_per_worker blocks, at
// most `resident` (0 = no cap), the workgroups its shard keeps on the chip at once.  chunk_base of each
// item is relative to its shard's launch.  (The min-trial probe's layout; searches use plan_launch.)
void slice(const std::vector<Win>& wins, uint64_t C, uint64_t chunk, size_t S, StepPlan& p, uint32_t resident = 0);
// Blocks of a piece per workgroup: a window of n blocks gets ceil(n / this) workgroups, at most
// `resident`.  Each workgroup takes about that many blocks from the item's queue before the item
// runs dry, so this sets how long the workgroups live, and the launch's tail with it.  Same box,
// twice each (profiles/r03/waves_queue_ab/blocks_per_worker_ab.txt): 16 blocks 6.644 / 6.654 GH/s on
// the C5 sample and 6.656 / 6.661 on C2, against 6.633 / 6.634 and 6.648 / 6.649 at 32 (one workgroup
// per chunk) and 6.633 / 6.642, 6.648 / 6.646 at 8; 128 and 512 were 2 % and 9 % slower.
// g_blocks_per_worker (0 = kBlocksPerWorker, at most a chunk) is set once by the library
// (bmpow_host.hip, BMPOW_BLOCKS_PER_WORKER for A/B runs).
constexpr uint64_t kBlocksPerWorker = 16;
extern uint32_t g_blocks_per_worker;

// Per-shard throughput: an exponential average of trials per ms over its launches of at least
// kRateMinTrials trials (short launches measure launch latency, not rate).  An object-sharded
// shard's fair share of the claimable objects is proportional to its rate (plan_launch), and a
// stepper estimates from it when its launch will end (the wait's sleep, bmpow_host.hip).  Weights are
// 1 until every shard has a sample and are clamped to [1/2, 2] x the mean.
constexpr uint64_t kRateMinTrials = (uint64_t)1 << 24;
constexpr double kRateAlpha = 0.25;
struct ShardRates {
  std::vector<double> ema;  // trials per ms; 0 = no sample yet
  uint64_t min_trials = kRateMinTrials;  // (the CPU stand-in's launches are small)
  void reset(size_t S) { ema.assign(S, 0.0); }
  void sample(size_t s, uint64_t trials, double ms);
  // w[s] with mean 1; false (w all 1) until every shard has a sample
  bool weights(std::vector<double>& w) const;
};

// A window split over the device groups (P = D pieces) covers kExpectWindows x E nonces (E = 2^64 /
// (target + 1), the expected trials to a hit; at least one chunk per piece): a split object then
// takes about one round of pieces, and with the cross-shard bound the pieces above a hit stop within
// a block row of it.  An object owned by one shard is not capped: its own early exit stops at its hit.
constexpr double kExpectWindows = 2.0;
uint64_t expect_cap(uint64_t target, size_t S, uint64_t chunk);

// ---------------------------------------------------------------------------------------
// Per-device stepping (round 4): one stepper thread and stream per shard,
// each claiming windows from the objects' frontiers under the engine's mutex whenever it is ready
// to launch, with its next launch staged behind the running one.  No shard waits for another.
//
// Exactness (the _doSafePoW answer, src/proofofwork.py:100-111, at any number of shards):
//   * an object's windows are created in ascending order at its frontier (next), and a launch's
//     result for an item is its device's running minimum hit of the object: every nonce of the
//     item's columns below that minimum was hashed (an early exit only skips nonces above a real
//     hit: the device's own, one folded in from the cross-shard bound, or one a previous launch on
//     the same stream left in best[]);
//   * an object is final once it has a hit h and every open window starts above h: every window
//     below h, and every piece of the window holding h, has been applied, whichever shard ran it;
//   * results of launches planned for an earlier occupant of a slot (its generation) are ignored.
// ---------------------------------------------------------------------------------------

// One item of a launch: piece `piece` of window [start, start + count) of object obj.
struct Claim {
  uint32_t obj, gen;
  uint64_t start, count;
  uint32_t G;
  uint16_t P, piece;
};

// One launch of one shard: planned under the engine's mutex, enqueued and waited for without it.
struct Launch {
  size_t shard = 0;
  int buf = 0;                  // the shard's launch buffer (two per shard: running + staged)
  BatchState* batch = nullptr;  // the batch it was planned from (the device side's bmpow_batch)
  std::vector<Claim> claims;
  StepPlan plan;                // items[0]: one per claim (bm_item.pad = its claim index), split_kinds order
  uint64_t planned = 0;         // nonces the launch covers (the engine's budget accounting)
  std::vector<uint32_t> xslots; // cross-shard bound slots its items carry (one count each)
  std::vector<bm_result> res;   // filled by EngineOps::wait, per item
  uint64_t trials = 0;          // hashed (the device counter)
  double ms = 0;                // search kernels' time (HIP events)
  double t_launch = 0;          // steady-clock ms at enqueue (the wait's sleep estimate)
};

// The cross-shard bound slots (BM_XSLOTS; bmpow_layout.h) of the objects that have items on more
// than one shard: an object keeps its slot while it has items in flight or open windows, and a
// slot is reused only once no in-flight item carries it (a stale launch still publishes there).
struct XPool {
  uint32_t ref[BM_XSLOTS] = {};    // in-flight items carrying the slot
  uint32_t owner[BM_XSLOTS] = {};  // object + 1, 0 = unowned
  // -1 when every slot is needed (the items then go without one); with b, a slot whose owner no
  // longer needs it (needed) is reclaimed first
  int alloc(uint32_t obj, BatchState* b = nullptr);
  bool needed(uint32_t x, const BatchState* b) const;
  size_t owned() const;
};

// What plan_launch needs to know about the shard it plans for.
struct PlanCtx {
  size_t s = 0, S = 1;
  // Device groups: group[s] = the physical device of shard s (ids 0 .. D-1), null = every shard its own.
  // Shards of one group share a device's SIMDs, where the kernel launched first holds the older waves:
  // two of them on one object would race each other's columns, so they never hold one object at once
  // and a split window has one piece per group (round 6; run()'s pieces follow the same rule).  A group
  // of one shard is the round-5 engine exactly.
  const std::vector<uint16_t>* group = nullptr;
  size_t D = 0;              // groups (0: S)
  uint64_t budget = 0;       // nonces this launch may claim (at least one chunk is claimed)
  uint32_t resident = 0;     // columns a piece may get on this shard (0 = no cap)
  double weight = 1.0;       // the shard's rate over the mean (ShardRates)
  XPool* xp = nullptr;       // null: no cross-shard bound
  // a slot was allocated: set it in every row to v (UINT64_MAX, or the object's least hit so far)
  std::function<void(uint32_t, uint64_t)> xreset;
};

// Objects a launch may take a window or a piece from.
// A new window of an object only while it is fewer than kMaxOpen windows past the object's oldest
// open one (claimable): the running window and the one staged behind it.
constexpr uint16_t kMaxOpen = 2;
bool claimable(const BatchState& b, size_t o);

// Plan the next launch of shard c.s from the claimable objects (slot order):
//   * object mode (at least D claimable objects, or one group): the shard takes its fair share q =
//     ceil(C x weight / S) of them -- those it already holds first, then ones no shard holds, then
//     (only if it found none) ones other shards hold -- each a window of budget / taken nonces;
//   * split mode (fewer claimable objects than groups): every object, one piece each of windows of
//     P = D pieces, expect_cap nonces per window;
//   * an object whose latest window still has pieces to hand out gets the next piece first;
//   * never an object another shard of the shard's group has in flight (with one group: no split, and
//     each object on one shard at a time, its windows in order on that shard's stream).
// Objects with items on several shards get a cross-shard bound slot (c.xp).  Returns false (L
// untouched) when nothing is claimable.
bool plan_launch(BatchState& b, const PlanCtx& c, Launch& L);

// Fold a completed launch into the state (results L.res[k] for L.plan.items[0][k]); an object that
// becomes final is queued for take_done.  publish(xslot, nonce): a new least hit of a shared object,
// for the other shards' relays.  waste (may be null): trials past the answers, priced once an object's
// answer is final (L.res[k].pad = the units item k's block queue handed out).  Returns the objects
// finished by it.
size_t apply_launch(BatchState& b, const Launch& L, XPool* xp,
                    const std::function<void(uint32_t, uint64_t)>& publish, WasteStats* waste = nullptr);
// Nonces of an item hashed above nonce h (all of them when h lies below its window), and the nonces it
// hashed in all: the first taken - nwg units its queue handed out, clipped to its blocks (WasteStats).
void waste_of(const WasteRec& r, uint64_t h, uint64_t& above, uint64_t& hashed);
// A launch that was never enqueued (an error before its kernels): its items are no longer in flight,
// and its windows never complete (the batch is broken).
void drop_launch(BatchState& b, const Launch& L, XPool* xp);
// The first nonce not known to be hashed: the lowest open window's start, else the frontier.
uint64_t resume_point(const BatchState& b, size_t o);

// The device side of the engine (bmpow_host.hip; tests/native/sched_sim.cpp runs a CPU stand-in).
struct EngineOps {
  std::function<int(Launch& L, std::string& err)> launch;  // stage + enqueue on shard L.shard, buffer L.buf
  std::function<int(Launch& L, std::string& err)> wait;    // block until it completed; fill res, trials, ms
  std::function<void(uint32_t xslot, uint64_t v)> xstore;  // store v in the slot of every shard's row
  std::function<bool()> aborted;
  std::function<void(size_t shard)> thread_init;           // first thing each stepper thread runs
};

struct EngineStats {
  uint64_t launches = 0, trials = 0, planned = 0, stale_items = 0;
  double kernel_ms = 0;
  std::vector<double> shard_ms;      // per shard: summed kernel time
  std::vector<uint64_t> shard_trials;
  WasteStats waste;                  // trials past the answers, by phase (apply_launch)
};

class Engine {
 public:
  Engine(EngineOps ops, size_t S, uint32_t resident, uint64_t step_trials);
  ~Engine();  // drains and joins the steppers
  // the attached batch's state and everything below; held across a launch's enqueue (plan and enqueue
  // are one step, so a slot's reuse cannot fall between them), never across a wait for the device
  std::mutex mu;
  // Make b the batch the steppers work on; a different attached batch is drained first.  lk holds mu.
  void attach(std::unique_lock<std::mutex>& lk, BatchState* b);
  // No new claims; wait until no launch is in flight (results applied); the batch stays attached.
  void drain(std::unique_lock<std::mutex>& lk);
  void detach(std::unique_lock<std::mutex>& lk);  // drain, then no batch
  BatchState* attached() const { return b_; }
  // Let the steppers claim `budget` more nonces beyond what has been applied (kU64Max: no bound) --
  // plus, with lookahead, one more launch per shard, which stays queued behind the running one when
  // run returns -- and wait until `budget` nonces have been applied since the call, done() holds
  // (checked after every applied launch), nothing is left to claim or in flight, or an error / abort.
  // Returns 0 or < 0 (err).
  int run(std::unique_lock<std::mutex>& lk, uint64_t budget, bool lookahead, const std::function<bool()>& done,
          std::string& err);
  void notify() { cv_.notify_all(); }  // after changing the attached batch's state (add, set_pending)
  void set_step_trials(uint64_t t) { step_ = t; }
  void set_throttle(size_t s, double ms);  // A/B knob: a shard sleeps this long before each launch
  // Device groups (PlanCtx::group; empty = every shard its own) and the columns an item may get, after
  // draining what is in flight.  lk holds mu.
  void set_groups(std::unique_lock<std::mutex>& lk, const std::vector<uint16_t>& group, uint32_t resident);
  size_t groups() const { return D_; }
  size_t shards() const { return S_; }
  size_t in_flight() const { return inflight_; }
  // Cross-shard bound slots with an owner (under mu); gc: first give back those no object needs.  After
  // a drain with every object settled, 0 (sched_sim checks it).
  size_t xslots_owned(bool gc = false);
  ShardRates rates;  // under mu
  EngineStats stats; // under mu
  int error() const { return error_; }
  void clear_error() { error_ = 0; err_.clear(); }
  // Each stepper thread's CPU seconds so far (CLOCK_THREAD_CPUTIME_ID) and scheduling policy
  // (sched_getscheduler as the thread set it; -2 before it ran).
  void thread_info(std::vector<double>& cpu_s, std::vector<int>& policy);

 private:
  struct EShard {
    std::deque<Launch*> q;  // in flight, oldest first
    Launch buf[2];
    int next = 0;
    double throttle_ms = 0;
    bool throttled = false;  // the throttle's delay before this shard's next plan has been served
    int policy = -2;       // the stepper's scheduling policy
    clockid_t cpu_clock{}; // its CPU-time clock
    bool have_clock = false;
  };
  void stepper(size_t s);
  bool can_plan() const;
  EngineOps ops_;
  const size_t S_;
  uint32_t resident_;
  std::vector<uint16_t> group_;  // empty: every shard its own group
  size_t D_;
  uint64_t step_;
  std::vector<EShard> sh_;
  BatchState* b_ = nullptr;
  XPool xp_;
  uint64_t claimed_ = 0, applied_ = 0, limit_ = 0;  // nonces (planned), monotonic
  size_t inflight_ = 0;
  int error_ = 0;
  std::string err_;
  bool stop_ = false;
  std::condition_variable cv_;
  std::vector<std::thread> th_;
};

// Scheduling class of the library's PoW threads (the steppers): the reference runs its PoW threads at
// SCHED_IDLE (src/bitmsghash/bitmsghash.cpp:149) and its pool workers at nice 20
// (src/proofofwork.py:72-87), so the PoW never takes a CPU from the application.  `policy` "idle"
// (SCHED_IDLE, the default), "batch" (SCHED_BATCH, nice 19) or "normal"; BMPOW_THREAD_POLICY overrides
// it.  Returns the sched_getscheduler() value in effect, or -1.
int set_thread_background(const char* policy = nullptr);

// Min-trial probe over n (object, range) pairs, in steps.
struct MinTrial {
  std::vector<uint64_t> cur, left;
  std::vector<uint8_t> any;
  size_t first = 0;
  void init(size_t n, const uint64_t* start, const uint64_t* count, uint64_t* min_out, uint64_t* argmin_out);
  // windows of the next step (<= total_chunks chunks of BM_CHUNK); false when every range is done
  bool plan(uint64_t total_chunks, std::vector<Win>& wins, uint64_t& C);
  // fold one shard's workgroup minima (parts[c] for the chunks of `items`) into min/argmin,
  // lexicographically on (trial, nonce) so ties keep the smaller nonce
  void reduce_parts(const std::vector<bm_item>& items, const bm_minpart* parts, uint64_t* min_out,
                    uint64_t* argmin_out);
  void advance(const std::vector<Win>& wins);
};

// ---- receive-side verification ----
struct Span {
  const uint8_t* p;
  uint64_t len;  // >= 8 (nonce || payload)
};

// blocks of SHA-512 padding for an m-byte message: m + 1 (0x80) + 16 (bit length) rounded up
uint64_t padded_blocks(uint64_t m);
void pad_into(const uint8_t* msg, uint64_t m, uint8_t* dst, uint64_t nblk);
// the same with non-temporal stores (dst 16-B aligned); stream_fence() before the device reads it
void pad_into_stream(const uint8_t* msg, uint64_t m, uint8_t* dst, uint64_t nblk);
void stream_fence();

struct VPart {
  size_t shard = 0;
  std::vector<uint32_t> orig;  // sorted position -> input index
  std::vector<bv_obj> ho;      // per sorted position: first block (part-relative), blocks, nonce
  std::vector<uint64_t> eol;   // per sorted position: expiresTime (object[8:16]; 0 if shorter), set by pad_range
  uint64_t blocks = 0;
  // work bins of bv_pow_binned_kernel (plan_bins): bins[0..nbins] are offsets into the group list
  // that follows them at bins[nbins + 1 ..]; empty when the part is not binned
  std::vector<uint32_t> bins;
  size_t nbins = 0;
};

// Sort objects by padded block count (descending, stable) and cut them into per-shard parts of
// equal block totals.  Reads only the lengths: the objects' bytes are first touched by pad_range,
// which also fills each descriptor's nonce and expiresTime (one pass over memory, in parallel).
// Returns BMPOW_E_ARG on size limits, else 0.
int plan_verify(const std::vector<Span>& objs, size_t S, std::vector<VPart>& parts, uint64_t& total_blocks,
                size_t nbins = 0);

// Deal a part's waves to nbins work bins, one per SIMD of its device (nbins a multiple of 4: four
// per workgroup of bv_pow_binned_kernel, one workgroup per CU).  A wave is BV_BLOCK consecutive
// objects of the sorted order (group g = objects [g * BV_BLOCK, (g + 1) * BV_BLOCK)); it costs its
// first object's block count + 2 (the trial's two compressions), since a wave runs as long as its
// longest lane.  Longest first, each to the least-loaded bin (LPT), so every SIMD's total is the
// average to within about one wave, whatever the objects' size mix.  The bins' group lists keep
// that order (a SIMD's waves take its longest groups first).
void plan_bins(VPart& pt, size_t nbins);

// Pad objects [j0, j1) of a part (sorted order) into dst (their blocks from blk0 on) and fill their
// nonce / expiresTime, over up to 16 host threads: a memory-bound copy of every payload.
void pad_range(const std::vector<Span>& objs, VPart& pt, size_t j0, size_t j1, uint64_t blk0, uint8_t* dst);

// The same thread fan-out for an index range (a thread per >= `grain` indices, at most 16).
void parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& body);

// protocol.isProofOfWorkSufficient's comparison (src/protocol.py:272-286) in the reference's
// arithmetic.  1 sufficient, 0 not.
int pow_sufficient(uint64_t pow, uint64_t len, uint64_t ntpb, uint64_t extra, int64_t recv, uint64_t eol);

// ---- continuous-batching service (bmpow_service_*) ----
// The service's threading, independent of the device: one stepper thread folds what producers
// submitted into the session (ops.add), steps it (ops.step) and queues the finished objects
// (ops.take) for poll().  The ops run on the stepper thread only and never under the service's
// mutex, so a caller of submit/poll/cancel waits at most for a queue operation, never for a step.
struct ServiceOps {
  // append n objects (initialHashes: 64 bytes each, or by ih_off as in init; targets; searches start at
  // nonce 1); slots[i] = object i's slot
  std::function<int(size_t n, const uint8_t* ihs, const uint64_t* ih_off, const uint64_t* targets, uint32_t* slots,
                    std::string& err)>
      add;
  std::function<int(std::string& err)> step;  // one step over the pending objects
  std::function<size_t(size_t cap, uint32_t* slot, uint64_t* nonce, uint64_t* trial, uint8_t* done)> take;
  std::function<int(std::string& err)> reset;  // drop every object of the session
};

class Service {
 public:
  struct Done {
    uint64_t ticket, nonce, trial;
    uint8_t done;
  };
  // verify: poll() re-hashes every found nonce on the host (host_trial) and reports a wrong trial or
  // one above the target as BMPOW_DONE_BADHASH
  explicit Service(ServiceOps ops, bool verify = false);
  ~Service();  // stop()
  // Queue n objects; tickets_out[i] (may be null) = object i's ticket, ascending over the service's
  // life.  BMPOW_E_STATE once stopping.
  // ih_off: null (64-byte initialHashes) or n + 1 offsets into ihs (any lengths)
  int submit(size_t n, const uint8_t* ihs, const uint64_t* targets, uint64_t* tickets_out,
             const uint64_t* ih_off = nullptr);
  // Pop up to cap finished objects, waiting up to timeout_ms (< 0: forever) for the first.  Returns
  // the count, 0 on timeout, or the error a step hit (err = its text) once everything before it was
  // popped; nothing is stepped after an error until cancel().
  int poll(size_t cap, int timeout_ms, uint64_t* tickets, uint64_t* nonce, uint64_t* trial, uint8_t* done,
           std::string& err);
  void cancel();  // drop queued, live and unpolled objects and a pending error
  size_t outstanding();  // submitted and not yet popped
  void stop();  // after the current step; idempotent, thread-safe

 private:
  void loop();
  struct Out {
    Done d;
    uint64_t target;
    uint8_t ih[64];
    std::vector<uint8_t> ihv;  // an initialHash of another length (ih unused), else empty
    bool var = false;
  };
  ServiceOps ops_;
  const bool verify_;
  std::mutex mu_;  // guards every member below
  std::condition_variable cv_in_, cv_out_;
  std::vector<uint8_t> in_ih_;
  std::vector<uint64_t> in_off_;  // n + 1 offsets into in_ih_ once any queued object is not 64 bytes, else empty
  std::vector<uint64_t> in_target_, in_ticket_;
  std::deque<Out> out_;
  uint64_t next_ticket_ = 0;
  size_t outstanding_ = 0;
  bool stopping_ = false, cancel_ = false;
  int error_ = 0;
  std::string err_;
  std::mutex join_mu_;
  std::thread th_;
};

}  // namespace bmsched
