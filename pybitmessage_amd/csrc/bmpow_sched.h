// bmpow_sched.h -- the host-only half of libbmpow_hip.so's scheduler: everything between the C ABI
// and the HIP calls that needs no device.  bmpow_host.hip drives the devices with it; the same
// source builds with g++ for the sanitizer tests (tests/native/: ThreadSanitizer, ASan/UBSan),
// which run it against a CPU stand-in for the kernels.
//
//   search steps   plan_step -> (launch per shard) -> apply_step        (bmpow_batch_step)
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

// Host mirror of a device-resident batch (one slot per object; slots of finished objects are
// released by take_done and reused by add).
struct BatchState {
  size_t n = 0;    // slots in the table (objects, finished ones and free slots included)
  size_t cap = 0;  // device allocation, in objects (set by the device side; add() reports growth)
  std::vector<bm_obj> objs;
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
  uint64_t vpool_epoch = 0;
};

// ih_off: null (n x 64-byte initialHashes) or n + 1 byte offsets into ihs (any lengths)
void init(BatchState& b, size_t n, const uint8_t* ihs, const uint64_t* targets, const uint64_t* start,
          const uint64_t* ih_off = nullptr);

// Append m objects (slots reused first).  slots[i] = object i's slot.  Returns true when the table
// outgrew b.cap (the caller reallocates and re-uploads); false when only `slots` need uploading.
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

// Deal the step's windows (C chunks, ascending chunk0) to S shards as work items (bmpow_layout.h).
//   * default: the flattened chunk list is cut into S contiguous slices -- big windows are
//     nonce-sharded, small ones object-sharded -- and each (window, shard) piece is one item whose
//     workgroups take its blocks in order; a piece gets one workgroup per g_blocks_per_worker blocks,
//     at most `resident` (0 = no cap), the workgroups its shard keeps on the chip at once;
//   * split (fewer pending objects than shards, S > 1): every shard gets an item over each whole
//     window, interleaved column by column (shard s runs columns [g0_s, g0_s + G) of S x G), so all
//     devices sweep the same front, and the window's cross-shard bound slot (p.nx of them) lets a hit
//     on one device stop the columns above it on every other.
// chunk_base of each item is relative to its shard's launch.
//   * weights (null = equal): the default mode's slices are cut in proportion to w[s] (ShardRates), so a
//     slower shard gets fewer chunks; split mode keeps equal columns (every shard sweeps the same rows).
void slice(const std::vector<Win>& wins, uint64_t C, uint64_t chunk, size_t S, StepPlan& p, uint32_t resident = 0,
           bool split = false, const double* weights = nullptr);
// Blocks of a piece per workgroup in the default mode: a piece of n blocks gets ceil(n / this)
// workgroups, at most `resident`.  Each workgroup takes about that many blocks from the item's queue
// before the item runs dry, so this sets how long the workgroups live, and the launch's tail with it.
// Same box, twice each (profiles/r03/waves_queue_ab/blocks_per_worker_ab.txt): 16 blocks 6.644 /
// 6.654 GH/s on the C5 sample and 6.656 / 6.661 on C2, against 6.633 / 6.634 and 6.648 / 6.649 at 32
// (one workgroup per chunk) and 6.633 / 6.642, 6.648 / 6.646 at 8; 128 and 512 were 2 % and 9 %
// slower.  g_blocks_per_worker (0 = kBlocksPerWorker, at most a chunk) is set once by the library
// (bmpow_host.hip, BMPOW_BLOCKS_PER_WORKER for A/B runs).
constexpr uint64_t kBlocksPerWorker = 16;
extern uint32_t g_blocks_per_worker;

// Per-shard throughput, to weight a step's slices.  The in-process multi-device step is lockstep
// (launch on every shard, wait for all, plan the next), so the slowest shard sets its length; a
// shard's share of the next step is made proportional to its measured rate instead of 1/S: an
// exponential average of trials per ms over its launches of at least kRateMinTrials trials (short
// launches measure launch latency, not rate).  Weights are 1 until every shard has a sample and are
// clamped to [1/2, 2] x the mean.
constexpr uint64_t kRateMinTrials = (uint64_t)1 << 24;
constexpr double kRateAlpha = 0.25;
struct ShardRates {
  std::vector<double> ema;  // trials per ms; 0 = no sample yet
  void reset(size_t S) { ema.assign(S, 0.0); }
  void sample(size_t s, uint64_t trials, double ms);
  // w[s] with mean 1; false (w all 1) until every shard has a sample
  bool weights(std::vector<double>& w) const;
};

// A window split over the shards is capped at kExpectWindows x E nonces (E = 2^64 / (target + 1), the
// expected trials to a hit; at least one chunk per shard): a step then lasts about as long as the
// object, and with the cross-shard bound the shards above a hit stop within a block row of it.  With
// as many objects as shards or more, objects are object-sharded and a shard's own early exit stops at
// its object's hit: no cap (it would only add steps).
constexpr double kExpectWindows = 2.0;
uint64_t expect_cap(uint64_t target, size_t S, uint64_t chunk);

// Windows for the next step over S shards with about `budget` trials (0 = step_trials x S): pending
// objects in slot order, k chunks each (capped by expect_cap when fewer than S are pending), dealt by
// slice (split mode when fewer than S objects are pending).  resident, weights: as slice.  Returns false (p
// untouched) when nothing is pending.
bool plan_step(BatchState& b, uint64_t budget, uint64_t step_trials, size_t S, StepPlan& p, uint32_t resident = 0,
               const double* weights = nullptr);

// Fold the step's per-shard results (res[s][k] for p.items[s][k]) into the state: the min over
// shards of each object's hits is final (every lower nonce of its window was hashed); no hit moves
// next past the window; a window ending at 2^64-1 without a hit exhausts the object.
void apply_step(BatchState& b, const StepPlan& p, const std::vector<const bm_result*>& res);

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
