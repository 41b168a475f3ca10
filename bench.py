#!/usr/bin/env python3
"""Benchmark of the Bitmessage double-SHA-512 PoW hot path on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5]

Default workload (N=1): BASELINE config C2 -- a batch of 1,024 pending msg objects,
payload sizes L ~ U[512, 16384] drawn with payloads from random.Random(20250216 + rank),
default difficulty (ntpb = extra = 1000), TTL = 345600 s, solved to the exact
_doSafePoW answer through the batch session of libbmpow_hip.so (the engine behind
proofofwork.run_batch).  One "step" = solving the whole batch from nonce 1.  The object
table is uploaded before the timed region (inputs resident in HBM); each step resets the
per-object state on the device (bmpow_batch_reset) and runs scheduler steps to completion.

Multi-GPU (torch.distributed.run, one process per GPU): each rank drives its own GPU
(LOCAL_RANK); the global batch is 1,024 objects per GPU, resident on every rank, and ranks
claim pieces of it on demand through the process group's TCP store (run_batch_bench), so all
GPUs finish together.  Units are independent: no data-path collective ("scaling": "weak");
gloo carries only the timing barrier and the max-over-ranks / sum-over-ranks reductions.

value = useful double-SHA-512 trials per second over the whole job (sum over objects of the
found nonce, i.e. the trials the sequential _doSafePoW would need -- the reference's own
nonce/time convention -- divided by the max-over-ranks wall time), in GH/s.  Trials the
kernels actually hashed (incl. the work past a hit that the early exit did not cancel) are
reported beside it.
"""
import argparse
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "double-SHA512 PoW trials/sec (GH/s, node) at 1/2/4/8 GPUs; objects PoW'd/sec"
SEED = 20250216
#: algorithmic int32 lane-ops per trial: 2 blocks x (80 x 34 + 64 x 22 + 16)
OPS_PER_TRIAL = 8288
#: vector-ALU peak, T int32 lane-ops/s: 256 CUs x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz -- the rate
#: behind MI355X_MICROARCH.md's 157.3 TFLOPS FP32 vector peak (one wave64 VALU op per 2 cycles).
PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12
#: The VALU issue model behind the roofline (profiles/r02): a wave64 VALU
#: instruction occupies its SIMD for one quad-cycle (4 clocks) unless two waves' full-rate 32-bit ops
#: pair in it (SQ_ACTIVE_INST_VALU2); bm_search_kernel's mix is 73 % half-rate VOP3 (v_alignbit_b32,
#: v_lshl_add_u64, v_lshrrev_b64), so its ceiling is one instruction per SIMD per quad-cycle.
SIMDS = 256 * 4
#: v_bitop3_b32 per trial in bm_search_kernel's nonce loop (tools/isa_census.py): the pairable share
BITOP3_PER_TRIAL = 1716


def object_target(L, ttl, ntpb=1000, extra=1000):
    from pybitmessage_amd.targets import object_target as f
    return int(f(L, ttl, ntpb, extra))


def make_objects(config, rank, n_override=None, test_mode=False):
    """-> (objects [(target, ih)], workload description).  test_mode: the reference's -t /
    extralowdifficulty difficulty (ntpb and extra divided by 100, bitmessagemain.py:167-172)."""
    rng = random.Random(SEED + rank)
    div = 100 if test_mode else 1
    objs = []
    if config == 'c2':
        n = n_override or 1024
        for _ in range(n):
            L = rng.randrange(512, 16385)
            payload = rng.randbytes(L)
            objs.append((object_target(L, 345600), hashlib.sha512(payload).digest()))
        desc = ('C2: %d pending msg objects, L~U[512,16384], ntpb=extra=1000, TTL=345600 s, '
                'exact first nonce via the batch session' % n)
    elif config == 'c4':
        n = n_override or 64
        for _ in range(n):
            payload = rng.randbytes(1024)
            objs.append((object_target(1024, 2419200, 20000, 1000), hashlib.sha512(payload).digest()))
        desc = 'C4: %d objects L=1024 at 20x ntpb (20000), TTL=28 d' % n
    elif config == 'c5':
        n = n_override or 100000
        for i in range(n):
            if i % 2 == 0:
                payload = rng.randbytes(46)
                objs.append((object_target(46, 2419200, 1000 // div, 1000 // div), hashlib.sha512(payload).digest()))
            else:
                payload = rng.randbytes(200)
                objs.append((object_target(200, 345600, 1000 // div, 1000 // div), hashlib.sha512(payload).digest()))
        desc = 'C5: %d objects, 50%% acks (L=46, TTL=28 d) + 50%% pubkey-size (L=200, TTL=4 d)%s' % (
            n, ', test-mode difficulty (ntpb = extra = 10)' if test_mode else '')
    else:
        raise ValueError(config)
    return objs, desc


# ----------------------------------------------------------------------------------------
# distributed plumbing (timing only; no data-path collective)
# ----------------------------------------------------------------------------------------
class Dist(object):
    def __init__(self):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local_rank = int(os.environ.get('LOCAL_RANK', '0'))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            # gloo prints "[Gloo] Rank r is connected to ..." on fd 1 from C++ while it builds its
            # mesh: send that to stderr so rank 0's stdout holds only the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group('gloo', rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def reduce(self, value, op):
        if not self.dist:
            return value
        import torch
        t = torch.tensor([float(value)], dtype=torch.float64)
        self.dist.all_reduce(t, op={'max': self.dist.ReduceOp.MAX, 'sum': self.dist.ReduceOp.SUM}[op])
        return float(t.item())

    def gather(self, obj):
        """Every rank's obj, in rank order (gloo all_gather_object; host-side, outside the timed region)."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def store(self):
        """The process group's TCP store (host-side key/value; used for work claiming)."""
        from torch.distributed import distributed_c10d
        return distributed_c10d._get_default_store()

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


# ----------------------------------------------------------------------------------------
# GPU legs
# ----------------------------------------------------------------------------------------
def solve_batch(lib, h, budget=0):
    from pybitmessage_amd import _lib
    _lib.check(lib, lib.bmpow_batch_reset(h, None), 'bmpow_batch_reset')
    pending = 1
    while pending > 0:
        pending = _lib.check(lib, lib.bmpow_batch_step(h, budget), 'bmpow_batch_step')


class Claimer(object):
    """Hands out pieces of the global batch to ranks on demand: a shared counter in the
    torch.distributed TCP store (host-side coordination only; no data moves).  With one rank it
    is a local counter that hands out everything at once."""

    def __init__(self, dist, n, chunk):
        self.n, self.chunk = n, chunk
        self.store = dist.store() if dist.world > 1 else None
        self.key, self.local = None, 0

    def start(self, tag):
        self.key, self.local = 'bmpow_claim_%s' % tag, 0

    def claim(self):
        if self.store is not None:
            lo = int(self.store.add(self.key, self.chunk)) - self.chunk
        else:
            lo, self.local = self.local, self.local + self.chunk
        return None if lo >= self.n else (lo, min(lo + self.chunk, self.n))


def cpu_snapshot(lib):
    """(process CPU seconds, per-stepper CPU seconds, per-stepper scheduling policy): getrusage of the
    whole process (every thread: this interpreter, the library's steppers and service thread) and the
    library's own account of its stepper threads (bmpow_get_thread_info)."""
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (ctypes.c_double * 64)()
    pol = (ctypes.c_int * 64)()
    n = lib.bmpow_get_thread_info(cpu, pol, 64) if hasattr(lib, 'bmpow_get_thread_info') else 0  # (older A/B builds)
    return ru.ru_utime + ru.ru_stime, [cpu[i] for i in range(min(n, 64))], [pol[i] for i in range(min(n, 64))]


def cpu_delta(c0, c1, elapsed):
    """Host CPU the PoW took while the GPU worked: CPU-seconds per wall-second of the timed region."""
    names = {0: 'SCHED_OTHER', 3: 'SCHED_BATCH', 5: 'SCHED_IDLE'}
    steppers = [round((b - a) / elapsed, 5) for a, b in zip(c0[1], c1[1])] if len(c0[1]) == len(c1[1]) else []
    return {'process_cpu_per_s': round((c1[0] - c0[0]) / elapsed, 5), 'stepper_cpu_per_s': steppers,
            'stepper_policy': sorted({names.get(p, str(p)) for p in c1[2]}),
            'wait': {'steppers': os.environ.get('BMPOW_WAIT', 'sleep')},
            'what': 'getrusage(RUSAGE_SELF) over the timed region (every thread of this process) and each '
                    'stepper thread\'s CLOCK_THREAD_CPUTIME_ID (bmpow_get_thread_info), per wall-second'}


def one_wait(st, elapsed):
    """How run()'s single-object path waited (bmpow_stats.one_wait_*): wall time the calling thread spun
    on a result word (a short call's last window) and slept between polls, per wall-second."""
    spin, sleep = getattr(st, 'one_wait_spin_ms', 0.0), getattr(st, 'one_wait_sleep_ms', 0.0)
    if spin + sleep <= 0:
        return None
    return {'mode': os.environ.get('BMPOW_WAIT1', 'auto'), 'spin_s_per_s': round(spin * 1e-3 / elapsed, 5),
            'sleep_poll_s_per_s': round(sleep * 1e-3 / elapsed, 5),
            'spin_share': round(spin / (spin + sleep), 5)}


def past_answers(st):
    """Where the engine hashed past the objects' answers (bmpow_stats.past_*, round 6): the window
    holding an answer (blocks above it), windows above it (the lookahead), and pieces of windows split
    over device groups -- estimates from each item's block queue (include/bmpow.h), with the estimated
    hashed total beside the device's count.  None when no batch ran."""
    est = int(getattr(st, 'engine_hashed_est', 0) or 0)
    if not est:
        return None
    return {'window': int(st.past_window), 'later': int(st.past_later), 'split': int(st.past_split),
            'hashed_est': est, 'trials': int(st.trials),
            'what': 'nonces hashed above the objects\' answers by where: the window holding the answer, '
                    'unsplit windows above it, split pieces (block-queue estimates, bmsched::WasteStats)'}


def prove_sample(lib, objs, nonce, idx, k, seed):
    """Exactness of k answers (a seeded sample of idx) at any size: each nonce n is the _doSafePoW
    answer (src/proofofwork.py:100-111) iff trial(n) <= target (re-checked with hashlib by the
    caller) and min{trial(m) : 1 <= m < n} > target -- the min-trial probe (bmpow_min_trial_batch), a
    kernel apart from the search's hit logic, hashes every nonce below each answer.  Outside the
    timed region."""
    import numpy as np
    from pybitmessage_amd import _lib
    pick = sorted(random.Random(seed).sample(idx, min(k, len(idx))))
    if not pick:
        return None
    n = len(pick)
    p64 = ctypes.POINTER(ctypes.c_uint64)
    st = np.ones(n, dtype=np.uint64)
    ct = np.array([int(nonce[i]) - 1 for i in pick], dtype=np.uint64)
    mn, arg = np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint64)
    t0 = time.perf_counter()
    _lib.check(lib, lib.bmpow_min_trial_batch(n, b''.join(objs[i][1] for i in pick), st.ctypes.data_as(p64),
                                              ct.ctypes.data_as(p64), mn.ctypes.data_as(p64),
                                              arg.ctypes.data_as(p64)), 'bmpow_min_trial_batch')
    ok = sum(1 for j, i in enumerate(pick) if int(mn[j]) > objs[i][0])
    return {'exact': ok, 'of': n, 'trials_rehashed': int(ct.sum()), 'seconds': round(time.perf_counter() - t0, 2),
            'how': 'bmpow_min_trial_batch over [1, nonce) of each sampled answer: min > target'}


def solve_claimed(lib, h, claimer, tag, low_water):
    """Solve the pieces of the global batch this rank claims: the whole table is resident and
    parked; pieces are scheduled (bmpow_batch_set_pending) whenever fewer than low_water objects
    are pending, so every rank keeps its GPU busy until the global batch runs out."""
    from pybitmessage_amd import _lib
    _lib.check(lib, lib.bmpow_batch_reset(h, None), 'bmpow_batch_reset')
    _lib.check(lib, lib.bmpow_batch_set_pending(h, 0, claimer.n, 0), 'bmpow_batch_set_pending')
    claimer.start(tag)
    mine, pending, exhausted = [], 0, False
    t_last = time.perf_counter()
    while True:
        if time.perf_counter() - t_last > 30:  # a progress line for long steps (C5 at full size)
            t_last = time.perf_counter()
            print('bench: %s: %d objects pending on this rank' % (tag, pending), file=sys.stderr, flush=True)
        while not exhausted and pending < low_water:
            r = claimer.claim()
            if r is None:
                exhausted = True
                break
            pending = _lib.check(lib, lib.bmpow_batch_set_pending(h, r[0], r[1] - r[0], 1), 'set_pending')
            mine.append(r)
        if pending == 0:
            return mine
        pending = _lib.check(lib, lib.bmpow_batch_step(h, 0), 'bmpow_batch_step')


def run_batch_bench(args, dist):
    """C2/C4/C5 over one global batch of objects-per-GPU x world objects.  Every rank holds the
    whole table in HBM (128 B/object) and claims pieces of it on demand, so all GPUs finish
    together (weak scaling without the max-over-ranks penalty of a fixed random split)."""
    import ctypes

    import numpy as np

    from pybitmessage_amd import _lib, proofofwork
    per_gpu = args.objects or {'c2': 1024, 'c4': 64, 'c5': 100000}[args.config]
    units = dist.world * max(1, args.devices)
    if args.config == 'c4' and args.devices and not args.objects:
        units = 1  # BASELINE C4: 64 objects in all, nonce-sharded over the in-process devices
    objs, desc = make_objects(args.config, 0, per_gpu * units, test_mode=args.test_mode)
    lib = _lib.get()
    n = len(objs)
    ihs = b''.join(ih for _, ih in objs)
    tg = np.array([t for t, _ in objs], dtype=np.uint64)
    p64 = ctypes.POINTER(ctypes.c_uint64)
    chunk = n if dist.world == 1 else max(1, min(8, per_gpu // 8))
    # Objects a rank keeps pending (N > 1).  When the global batch runs out each rank still has these
    # to finish, and an object's remaining work is ~E whatever it has hashed (the hit is memoryless),
    # so the spread between ranks' tails grows as the square root of this count: 32 (C2: ~0.8 % of a
    # step at 8 GPUs by that estimate, against ~1.7 % at 128) still gives one GPU thousands of
    # workgroups per step, since a single window already fills the chip (the block queue).
    low_water = max(chunk, min(32, per_gpu // 4))
    claimer = Claimer(dist, n, chunk)
    h = lib.bmpow_batch_create(n, ihs, tg.ctypes.data_as(p64), None)
    if not h:
        raise RuntimeError('bmpow_batch_create: %s' % lib.bmpow_last_error().decode())
    try:
        for w in range(args.warmup):
            solve_claimed(lib, h, claimer, 'w%d' % w, low_water)
        dist.barrier()
        lib.bmpow_reset_stats()
        c0 = cpu_snapshot(lib)
        t0 = time.perf_counter()
        mine = []
        for k in range(args.steps):
            mine = solve_claimed(lib, h, claimer, 's%d' % k, low_water)
        dist.barrier()
        elapsed = time.perf_counter() - t0
        host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
        st = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(st))
        nonce = np.zeros(n, dtype=np.uint64)
        trial = np.zeros(n, dtype=np.uint64)
        done = np.zeros(n, dtype=np.uint8)
        lib.bmpow_batch_results(h, nonce.ctypes.data_as(p64), trial.ctypes.data_as(p64),
                                done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), None)
    finally:
        lib.bmpow_batch_destroy(h)
    # every answer of the last step re-checked on the host: trial(nonce) <= target with hashlib
    idx = [i for lo, hi in mine for i in range(lo, hi)]
    assert all(done[i] == _lib.DONE_FOUND for i in idx)
    for i in idx:
        proofofwork._verify(int(tg[i]), objs[i][1], int(trial[i]), int(nonce[i]))
    useful = float(sum(int(nonce[i]) for i in idx)) * args.steps
    if dist.world > 1:
        desc += ' (global batch of %d, pieces of %d claimed on demand)' % (n, chunk)
    # exactness of a seeded sample of the answers, proven at full size outside the timed region
    # (1,000 of C5's 100k; 64 elsewhere)
    exact = None if args.no_exact else prove_sample(lib, objs, nonce, idx, 1000 if args.config == 'c5' else 64,
                                                   SEED + dist.rank)
    return {'desc': desc, 'objects': len(idx) * args.steps, 'useful': useful, 'elapsed': elapsed, 'stats': st,
            'nonces_sum': int(sum(int(nonce[i]) for i in idx)), 'host_cpu': host_cpu, 'exact_sample': exact}


def run_service_bench(args, dist):
    """C2/C5 through worker.PowService: every object submitted to the service (the library's stepping
    thread over a resident device session, bmpow_service_submit / bmpow_service_poll), all futures
    awaited; the same objects and answers as the batch leg, so the two objects/s figures compare
    directly."""
    from pybitmessage_amd import _lib, worker
    per_gpu = args.objects or {'c2': 1024, 'c5': 4096}[args.config]
    objs, desc = make_objects(args.config, dist.rank, per_gpu, test_mode=args.test_mode)
    lib = _lib.get()

    def once():
        svc = worker.PowService().start()
        stop = threading.Event()

        def progress():  # a line every 30 s, so a long run (C5 at full size) shows it is alive
            while not stop.wait(30):
                print('bench: service: %d of %d objects solved' % (svc.solved, len(objs)), file=sys.stderr, flush=True)
        th = threading.Thread(target=progress, daemon=True)
        th.start()
        try:
            futs = svc.submit_many(objs)
            return [f.result() for f in futs]
        finally:
            stop.set()
            th.join()
            svc.stop(30)
    for _ in range(args.warmup):
        once()
    dist.barrier()
    lib.bmpow_reset_stats()
    c0 = cpu_snapshot(lib)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = once()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    useful = float(sum(n for _, n in res)) * args.steps
    nonce = [n for _, n in res]
    exact = None if args.no_exact else prove_sample(lib, objs, nonce, list(range(len(objs))),
                                                   1000 if args.config == 'c5' else 64, SEED + dist.rank)
    return {'desc': desc + ' via worker.PowService (native stepping thread)', 'objects': len(objs) * args.steps,
            'useful': useful, 'elapsed': elapsed, 'stats': st,
            'host_cpu': host_cpu, 'exact_sample': exact}


def run_runbatch_bench(args, dist):
    """C2/C5 through the product entry point proofofwork.run_batch (session + stepping thread +
    per-object hashlib re-check, each answer the _doSafePoW nonce)."""
    from pybitmessage_amd import _lib, proofofwork
    per_gpu = args.objects or {'c2': 1024, 'c5': 4096}[args.config]
    objs, desc = make_objects(args.config, dist.rank, per_gpu, test_mode=args.test_mode)
    lib = _lib.get()
    for _ in range(args.warmup):
        proofofwork.run_batch(objs)
    dist.barrier()
    lib.bmpow_reset_stats()
    c0 = cpu_snapshot(lib)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = proofofwork.run_batch(objs)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    useful = float(sum(n for _, n in res)) * args.steps
    return {'desc': desc + ' via proofofwork.run_batch', 'objects': len(objs) * args.steps,
            'useful': useful, 'elapsed': elapsed, 'stats': st,
            'host_cpu': host_cpu}


def run_serial_bench(args, dist):
    """C2/C4/C5 objects solved ONE AFTER ANOTHER through proofofwork.run -- every call site of the
    reference is such a serial call (class_singleWorker.py:236,1276, api.py:1304,1350) -- on the
    single-object path (pieces over the devices); the host CPU the calls take is in host_cpu."""
    from pybitmessage_amd import _lib, proofofwork
    per_gpu = args.objects or {'c2': 64, 'c4': 8, 'c5': 256}[args.config]
    objs, desc = make_objects(args.config, dist.rank, per_gpu, test_mode=args.test_mode)
    lib = _lib.get()
    for t, ih in objs[:args.warmup]:
        proofofwork.run(t, ih)
    dist.barrier()
    lib.bmpow_reset_stats()
    c0 = cpu_snapshot(lib)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = [proofofwork.run(t, ih) for t, ih in objs]
    dist.barrier()
    elapsed = time.perf_counter() - t0
    host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    nonce = [n for _, n in res]
    exact = None if args.no_exact else prove_sample(lib, objs, nonce, list(range(len(objs))), 64, SEED + dist.rank)
    return {'desc': desc + ', one proofofwork.run call after another', 'objects': len(objs) * args.steps,
            'useful': float(sum(nonce)) * args.steps, 'elapsed': elapsed, 'stats': st, 'host_cpu': host_cpu,
            'exact_sample': exact, 'path': one_path_desc(args, lib), 'call_ms': round(elapsed * 1e3 / len(objs) / args.steps, 3),
            'kernel': 'bm_search1_kernel' if single_object_path(args) else 'bm_search_kernel'}


def run_c3_bench(args, dist):
    """C3: fixed initialHash, target 0 (no hit), 2^log2 nonces split contiguously over ranks."""
    import ctypes

    from pybitmessage_amd import _lib
    lib = _lib.get()
    ih = hashlib.sha512(b'bmpow-sweep').digest()
    total = 1 << args.c3_log2
    share = total // dist.world
    start = 1 + dist.rank * share
    n, t = ctypes.c_uint64(), ctypes.c_uint64()

    def sweep():
        rc = _lib.check(lib, lib.bmpow_search(ih, 0, start, share, ctypes.byref(n), ctypes.byref(t)), 'search')
        assert rc == _lib.NOT_FOUND
    for _ in range(args.warmup):
        sweep()
    dist.barrier()
    lib.bmpow_reset_stats()
    c0 = cpu_snapshot(lib)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sweep()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    desc = 'C3: fixed initialHash, target=0, 2^%d nonces split over %d GPU(s)' % (args.c3_log2, dist.world)
    return {'desc': desc, 'objects': 0, 'useful': float(share) * args.steps, 'elapsed': elapsed, 'stats': st,
            'scaling': 'strong', 'host_cpu': host_cpu, 'path': one_path_desc(args, lib),
            'kernel': 'bm_search1_kernel' if single_object_path(args) else 'bm_search_kernel'}


def single_object_path(args):
    """run()/bmpow_search take the single-object kernel (bmpow_host.hip search_one) on any number of
    shards unless BMPOW_ONE=0 (round 5: several devices each run one interleaved piece of a window)."""
    return os.environ.get('BMPOW_ONE') != '0'


def run_pieces(lib):
    """The shards carrying run()'s pieces (bmpow_get_run_pieces) and the devices they are on."""
    ids = (ctypes.c_int * 64)()
    n = lib.bmpow_get_run_pieces(ids, 64) if hasattr(lib, 'bmpow_get_run_pieces') else 1
    dev = (ctypes.c_int * 64)()
    lib.bmpow_get_devices(dev, 64)
    return [{'shard': ids[i], 'device': dev[ids[i]]} for i in range(max(0, min(n, 64)))]


def one_path_desc(args, lib):
    if not single_object_path(args):
        return 'engine (bm_search_kernel)'
    p = run_pieces(lib)
    if len(p) <= 1:
        return 'single-object (bm_search1_kernel)'
    return ('single-object split into %d pieces, one per %s (bm_search1_kernel + relay, cross-device bound)'
            % (len(p), 'shard (forced, bmpow_set_run_split; pieces sharing a GPU each on their own CU slice)'
               if getattr(args, 'run_split', False) else 'device'))


def run_c1_bench(args, dist):
    import ctypes

    from pybitmessage_amd import _lib, proofofwork
    lib = _lib.get()
    payload = random.Random(SEED).randbytes(1024)
    ih = hashlib.sha512(payload).digest()
    target = object_target(1024, 345600)
    for _ in range(args.warmup):
        proofofwork.run(target, ih)
    lib.bmpow_reset_stats()
    c0 = cpu_snapshot(lib)
    # per call: wall time and trials hashed (the stats counters are read between calls, outside the
    # call, so the distribution shows a slow or wasteful call without slowing the others)
    per_ms, per_trials, prev = [], [], 0
    cst = _lib.BmpowStats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        c = time.perf_counter()
        tv, nonce = proofofwork.run(target, ih)
        per_ms.append((time.perf_counter() - c) * 1e3)
        lib.bmpow_get_stats(ctypes.byref(cst))
        per_trials.append(cst.trials - prev)
        prev = cst.trials
    elapsed = time.perf_counter() - t0
    host_cpu = cpu_delta(c0, cpu_snapshot(lib), elapsed)
    assert nonce == 10909138, nonce
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))

    def dist(xs, nd):
        xs = sorted(xs)
        return {'min': round(xs[0], nd), 'median': round(xs[len(xs) // 2], nd), 'p90': round(xs[int(0.9 * (len(xs) - 1))], nd),
                'max': round(xs[-1], nd)}
    return {'desc': 'C1: one 1 KB msg at defaults via proofofwork.run (golden nonce 10909138)',
            'objects': args.steps, 'useful': float(nonce) * args.steps, 'elapsed': elapsed, 'stats': st,
            'host_cpu': host_cpu, 'call_ms': round(elapsed * 1e3 / args.steps, 4),
            'per_call': {'ms': dist(per_ms, 4), 'trials': dist(per_trials, 0),
                         'past_answer_frac': dist([(x - nonce) / x for x in per_trials], 5),
                         'calls_by_past_answer': {k: sum(1 for x in per_trials if lo <= (x - nonce) / x < hi)
                                                  for k, lo, hi in (('<1%', -1, 0.01), ('1-5%', 0.01, 0.05),
                                                                    ('5-20%', 0.05, 0.2), ('>=20%', 0.2, 2))}},
            'path': one_path_desc(args, lib),
            'kernel': 'bm_search1_kernel' if single_object_path(args) else 'bm_search_kernel'}


def verify_objects(n, rank):
    """Receive-side flood: finished objects as they arrive from the network,
    half acks (54 B), a quarter pubkey-size (208 B), a quarter msgs (L ~ U[512, 16384])."""
    rng = random.Random(SEED + 1000 + rank)
    objs = []
    for i in range(n):
        r = i % 4
        L = 46 if r in (0, 1) else (200 if r == 2 else rng.randrange(512, 16385))
        objs.append(rng.randbytes(8) + (1700000000 + 345600).to_bytes(8, 'big') + rng.randbytes(L - 8))
    return objs


def run_verify_bench(args, dist):
    """POW values of a resident flood, one bv_pow_kernel pass per step (bmpow_vbatch_run)."""
    import ctypes

    from pybitmessage_amd import _lib, targets, verify
    n = args.objects or 500000  # an inventory sync's worth of objects (--objects to change)
    objs = verify_objects(n, dist.rank)
    payload_bytes = sum(len(o) - 8 for o in objs)
    lib = _lib.get()
    with verify.VerifyBatch(objs) as vb:
        first = vb.run()
        for i in range(0, n, max(1, n // 500)):  # spot-check against hashlib
            assert int(first[i]) == targets.pow_value(objs[i]), i
        for _ in range(args.warmup):
            vb.run(want=False)
        dist.barrier()
        lib.bmpow_reset_stats()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            vb.run(want=False)
        dist.barrier()
        elapsed = time.perf_counter() - t0
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    # end to end, the way a caller uses it: host buffers in, verdicts out (padding and sorting on
    # the host, PCIe upload, kernel, IEEE-double verdicts) -- reported beside, never as `value`
    # (first call: allocates the library's staging and device buffers; later floods reuse them)
    e2e, parts = [], []
    for _ in range(3):
        lib.bmpow_reset_stats()
        t1 = time.perf_counter()
        ok = verify.isProofOfWorkSufficient_batch(objs, recvTime=1700000000)
        e2e.append(time.perf_counter() - t1)
        s2 = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(s2))
        parts.append({'build_ms': round(s2.verify_host_build_ms, 2), 'run_ms': round(s2.verify_host_run_ms, 2),
                      'verdict_ms': round(s2.verify_host_verdict_ms, 2), 'kernel_ms': round(s2.verify_kernel_ms, 3),
                      'marshal_ms': round(e2e[-1] * 1e3 - s2.verify_host_build_ms - s2.verify_host_run_ms
                                          - s2.verify_host_verdict_ms, 2)})
        assert len(ok) == n
    best = 1 + min(range(2), key=lambda i: e2e[1 + i])
    return {'e2e_objects_per_s': n / e2e[best], 'e2e_s': e2e[best], 'e2e_first_s': e2e[0], 'e2e_parts': parts[best],
            'e2e_fast_marshalling': verify._fast() is not None,
            'desc': 'verify: %d received objects (50%% acks, 25%% pubkeys, 25%% msgs 0.5-16 KB), POW of each '
                    '(protocol.isProofOfWorkSufficient hashing) resident in HBM' % n,
            'objects': n * args.steps, 'elapsed': elapsed, 'stats': st, 'payload_bytes': payload_bytes * args.steps}


def summarize_verify(args, dist, r, lib_version):
    st = r['stats']
    el_max = dist.reduce(r['elapsed'], 'max')
    objects = dist.reduce(r['objects'], 'sum')
    nbytes = dist.reduce(r['payload_bytes'], 'sum')
    line = {
        'metric': 'received objects verified/sec (protocol.isProofOfWorkSufficient POW, GPU batch)',
        'value': round(objects / el_max, 1), 'unit': 'objects/s', 'n_gpus': dist.world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(el_max * 1e3 / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u64', 'data': 'synthetic',
        'config': {'workload': r['desc'], 'parallelism': 'object-sharded dp%d' % dist.world, 'lib': lib_version},
        'payload_GBps': round(nbytes / el_max / 1e9, 3),
        'e2e_host_buffers': {'objects_per_s': round(r['e2e_objects_per_s'], 1), 'seconds': round(r['e2e_s'], 3),
                             'first_call_seconds': round(r['e2e_first_s'], 3), 'parts': r['e2e_parts'],
                             'c_marshalling': r['e2e_fast_marshalling'],
                             'what': 'bmpow_verify_batch_ptrs from host buffers: sort + pad into pinned staging '
                                     'overlapped with the PCIe upload + kernel + verdicts (rank 0; best of 2 '
                                     'calls after the first, which allocates the reused buffers)'},
    }
    if st.verify_kernel_ms > 0:
        # algorithmic ops: 4,144 per 128-B payload block (SURVEY 8(d) per-block count) + 8,288 for
        # the outer double hash of each object
        ops = 4144 * st.verify_blocks + OPS_PER_TRIAL * st.verify_objects
        achieved = ops / (st.verify_kernel_ms * 1e-3) / 1e12
        # the library bins floods of >= 2 waves per SIMD (bmpow_host.hip verify_binned)
        binned = r['objects'] // max(args.steps, 1) >= 2 * 64 * 4 * 256
        line['roofline'] = {'bound': 'valu', 'kernel': 'bv_pow_binned_kernel' if binned else 'bv_pow_kernel',
                            'achieved': round(achieved, 3),
                            'peak': round(PEAK_TOPS, 3), 'unit': 'T int32 lane-ops/s', 'frac': round(achieved / PEAK_TOPS, 4),
                            'traffic': None, 'blocks_per_s': round(st.verify_blocks / (st.verify_kernel_ms * 1e-3), 1),
                            'avg_launch_ms': round(st.verify_kernel_ms / max(args.steps, 1), 3),
                            'kernel_busy_frac': round(st.verify_kernel_ms * 1e-3 / r['elapsed'], 4)}
        pmc = kernel_pmc('verify_binned.json') if binned else None
        if pmc:
            line['roofline']['traffic'] = pmc.pop('hbm_bytes_per_launch', None)
            line['roofline']['counters'] = pmc
    return line


def kernel_pmc(name):
    """Counters of a kernel from the committed rocprofv3 PMC passes (profiles/r02/scripts/r02_pmc_verify_addr.sh ->
    tools/pmc_kernel.py -> profiles/r02/pmc/<name>): per-launch HBM bytes (2 x FETCH_SIZE + WRITE_SIZE)
    and the VALU issue figures."""
    path = os.path.join(ROOT, 'profiles', 'r02', 'pmc', name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)['derived']
    out = {'source': 'profiles/r02/pmc/' + name}
    for k in ('hbm_bytes_per_launch', 'valu_issue_util', 'valu_instr_per_simd_quad_cycle', 'dual_issue_share',
              'simd_busy_frac', 'eff_clock_ghz'):
        if d.get(k) is not None:
            out[k] = round(d[k], 4) if k != 'hbm_bytes_per_launch' else round(d[k])
    return out


def _verify_pool_worker(seconds):
    from pybitmessage_amd import targets
    objs = verify_objects(4000, 0)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        targets.pow_value(objs[k % len(objs)])
        k += 1
    return k, time.perf_counter() - t0


def _verify_pool(seconds, p):
    """In a fresh child process (cpu_baseline_worker, mode 'verify'): a pool of p processes, each
    hashing the flood for `seconds`."""
    import multiprocessing
    with multiprocessing.get_context('fork').Pool(p) as pool:
        t0 = time.perf_counter()
        res = pool.map(_verify_pool_worker, [seconds] * p)
        wall = time.perf_counter() - t0
    return {'objects': sum(r[0] for r in res), 'wall': wall}


def cpu_verify_baseline(seconds):
    """The reference's per-object check (protocol.py:280-282, targets.pow_value: hashlib, i.e.
    OpenSSL) on the same flood, one process per CPU of the box's share, each hashing for
    `seconds` (no pickling of objects: every worker builds the flood itself).  The pool runs in a
    fresh child process that never touches the GPU (HIP_VISIBLE_DEVICES=''), like the PoW legs: this
    process has initialised HIP and the library's padding threads, which a fork must not inherit."""
    info = host_cpu_info()
    p = info['share']
    cmd = [sys.executable, os.path.abspath(__file__), '--cpu-baseline-worker', '--cpu-seconds', str(seconds),
           '--cpu-threads', str(p), '--cpu-mode', 'verify']
    env = dict(os.environ)
    env['HIP_VISIBLE_DEVICES'] = ''
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 20 + 120, env=env)
    line = [l for l in out.stdout.splitlines() if l.startswith('{')]
    if out.returncode != 0 or not line:
        return {'error': (out.stderr or out.stdout)[-400:], 'host': info}
    r = json.loads(line[-1])
    k, wall = r['objects'], r['wall']
    return {'value': round(k / wall, 1), 'unit': 'objects/s', 'cores': p, 'kind': 'port',
            'sample': '%d objects of the same flood hashed by hashlib (OpenSSL) in %.1f s wall on a pool of %d '
                      'processes' % (k, wall, p), 'host': info}


ADDR_PASSPHRASE = b'bmpow address-search benchmark'


def run_addr_bench(args, dist):
    """Deterministic address search (class_addressGenerator.py:238-271) at --null-bytes
    (default 3: ~16.7M expected tries, a "vanity" request the reference would take hours on),
    repeated from try 0 each step; useful tries = found k + 1 (the sequential loop's count)."""
    import ctypes

    from pybitmessage_amd import _lib, addressgen
    lib = _lib.get()
    pp = ADDR_PASSPHRASE + b' rank %d' % dist.rank
    nb = args.null_bytes
    lib.bmpow_addr_set_comb(args.addr_comb)
    t0 = time.perf_counter()
    addressgen.search_deterministic(b'comb table build', 1)  # builds the comb table(s) once per device
    table_s = time.perf_counter() - t0
    if args.addr_mode == 'random':  # createRandomAddress: fixed signing key, fresh encryption keys
        priv_s = hashlib.sha256(pp).digest()
        seed = hashlib.sha512(pp).digest()

        def one():
            r = addressgen.random_address(null_bytes=nb, priv_signing=priv_s, seed=seed)
            return r['k'], r['ripe']
        what = 'random address search (class_addressGenerator.py:130-148), %d null bytes, fixed signing key' % nb
    else:
        def one():
            f = addressgen.search_deterministic(pp, nb)
            return f.k, f.ripe
        what = 'deterministic address search, %d null bytes, passphrase %r' % (nb, pp)
    for _ in range(args.warmup):
        one()
    dist.barrier()
    lib.bmpow_reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k, ripe = one()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    assert ripe[:nb] == b'\x00' * nb
    comb = lib.bmpow_addr_last_comb()
    return {'desc': 'addrgen: %s, found k=%d, %d-bit comb' % (what, k, comb),
            'tries': float(k + 1) * args.steps, 'elapsed': elapsed, 'stats': st, 'k': k,
            'comb_bits': comb, 'table_build_s': table_s}


def summarize_addr(args, dist, r, lib_version):
    st = r['stats']
    el_max = dist.reduce(r['elapsed'], 'max')
    tries = dist.reduce(r['tries'], 'sum')
    launched = dist.reduce(st.addr_tries, 'sum')
    line = {
        'metric': 'address-search tries/sec (%s secp256k1 k*G + SHA-512 + RIPEMD-160 per try)'
                  % ('1 x' if args.addr_mode == 'random' else '2 x'),
        'value': round(tries / el_max, 1), 'unit': 'tries/s', 'n_gpus': dist.world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(el_max * 1e3 / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32', 'data': 'synthetic',
        'config': {'workload': r['desc'], 'parallelism': 'dp%d' % dist.world, 'lib': lib_version},
        'launched_tries_per_s': round(launched / el_max, 1),
        'comb_bits': r['comb_bits'],
        'table_build_s': round(r['table_build_s'], 3),  # one-time per device, before the timed region
    }
    if st.addr_kernel_ms > 0:
        line['kernel'] = {'name': 'ar_search_kernel', 'tries_per_s': round(st.addr_tries / (st.addr_kernel_ms * 1e-3), 1),
                          'launches': int(st.addr_launches), 'kernel_ms': round(st.addr_kernel_ms, 3),
                          'kernel_busy_frac': round(st.addr_kernel_ms * 1e-3 / r['elapsed'], 4)}
    pmc = kernel_pmc('addrgen_%s.json' % args.addr_mode)
    if pmc and pmc.get('valu_instr_per_simd_quad_cycle'):
        # k*G has no implementation-independent op count like SHA-512's 8,288, so this roofline is
        # in issued VALU lane-instructions: the measured instructions per SIMD quad-cycle against two
        # (the 78.64 T dual-issue peak); one per quad-cycle is the single-issue ceiling
        ipq = pmc['valu_instr_per_simd_quad_cycle']
        clk = pmc.get('eff_clock_ghz') or 2.4
        line['roofline'] = {'bound': 'valu', 'kernel': 'ar_search_kernel',
                            'achieved': round(ipq * 1024 * clk * 1e9 / 4 * 64 / 1e12, 3), 'peak': round(PEAK_TOPS, 3),
                            'unit': 'T VALU lane-instructions/s issued (no implementation-independent op count)',
                            'frac': round(ipq / 2, 4), 'single_issue_frac': round(ipq, 4),
                            'traffic': pmc.pop('hbm_bytes_per_launch', None), 'counters': pmc}
    return line


def cpu_addr_baseline(seconds, mode='det'):
    """One core: the reference's per-try work with the same compiled library calls it makes --
    OpenSSL EC_POINT_mul for both keys (random mode: the encryption key only, the signing key is
    fixed; oracle.addrgen_oracle.OpenSSLPointMult), hashlib SHA-512, and libcrypto's RIPEMD160()
    (oracle.addrgen_oracle.OpenSSLRipemd160; hashlib's ripemd160 needs OpenSSL's legacy provider).
    The per-call Python overhead is the reference's too (its loop is Python)."""
    import hashlib as hl

    from oracle import addrgen_oracle as ao
    pm = ao.OpenSSLPointMult()
    rmd = ao.OpenSSLRipemd160()
    pub_s = pm(hl.sha256(ADDR_PASSPHRASE).digest())
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        ps, pe = ao.try_keys(ADDR_PASSPHRASE, k)
        rmd(hl.sha512((pub_s if mode == 'random' else pm(ps)) + pm(pe)).digest())
        k += 1
    el = time.perf_counter() - t0
    return {'value': round(k / el, 1), 'unit': 'tries/s', 'cores': 1, 'kind': 'port',
            'sample': '%d tries in %.1f s: OpenSSL EC_POINT_mul x%d (system libcrypto, as pyelliptic calls it), '
                      'hashlib SHA-512, libcrypto RIPEMD160(); 1 thread' % (k, el, 1 if mode == 'random' else 2)}


# ----------------------------------------------------------------------------------------
# CPU baseline (rank 0, N=1): the reference's own BitmessagePOW built from its source (the C
# path, _doCPoW) and its hashlib + multiprocessing path (_doFastPoW), on the host's cores
# ----------------------------------------------------------------------------------------
def host_cpu_info():
    """CPU model, CPU count, this process's affinity and the cgroup CPU quota (the box's share:
    a one-GPU box may show the whole machine's CPUs while its quota is far smaller)."""
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    for path in ('/sys/fs/cgroup/cpu.max',):
        try:
            q, per = open(path).read().split()[:2]
            if q != 'max':
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
            per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    aff = len(os.sched_getaffinity(0))
    share = max(1, int(min(aff, quota))) if quota else aff
    return {'model': model, 'nproc': os.cpu_count(), 'affinity': aff,
            'cgroup_quota_cpus': round(quota, 2) if quota else None, 'share': share}


def cpu_baseline_worker(seconds, threads, mode):
    """Child process, never touches the GPU.  Solves C2 objects (the first of the rank-0 batch) in
    order until `seconds` elapse; rate = sum(nonce) / time, the reference's nonce/time convention.
    mode 'c': the reference's BitmessagePOW (oracle/_ref) on `threads` CPUs of the affinity mask
    (it sizes its pthread pool from that mask, bitmsghash.cpp:96,109-121); mode 'fast': the
    _doFastPoW mechanism (oracle/fastpow.py) with a pool of `threads` processes."""
    if mode == 'verify':
        print(json.dumps(_verify_pool(seconds, threads)), flush=True)
        return
    cpus = sorted(os.sched_getaffinity(0))
    if mode == 'c':
        os.sched_setaffinity(0, cpus[:threads])
    from oracle import oracle
    objs, _ = make_objects('c2', 0, 64)
    if mode == 'fast':
        from oracle import fastpow
        kind = 'reference-mechanism'
        solve = lambda t, ih: fastpow.fast_pow(t, ih, threads)[1]  # noqa: E731
    elif oracle.have_ref():
        ref = oracle.RefBitmsghash()
        kind = 'reference'
        solve = lambda t, ih: ref.pow(t, ih)[1]  # noqa: E731
    else:
        co = oracle.COracle()
        kind = 'port'
        solve = lambda t, ih: co.search_mt(ih, t, 1, 1 << 40, threads=threads)[0][1]  # noqa: E731
    t0 = time.perf_counter()
    total, k = 0, 0
    for t, ih in objs:
        total += solve(t, ih)
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    print(json.dumps({'kind': kind, 'mode': mode, 'cores': threads, 'objects': k, 'nonce_sum': total,
                      'seconds': el}))


def _cpu_leg(seconds, threads, mode):
    cmd = [sys.executable, os.path.abspath(__file__), '--cpu-baseline-worker', '--cpu-seconds', str(seconds),
           '--cpu-threads', str(threads), '--cpu-mode', mode]
    env = dict(os.environ)
    env['HIP_VISIBLE_DEVICES'] = ''  # the baseline never touches the GPU
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=seconds * 20 + 120, env=env)
    line = [l for l in out.stdout.splitlines() if l.startswith('{')]
    if out.returncode != 0 or not line:
        return {'error': (out.stderr or out.stdout)[-400:]}
    r = json.loads(line[-1])
    r['ghs'] = r['nonce_sum'] / r['seconds'] / 1e9
    r['objects_per_s'] = r['objects'] / r['seconds']
    return r


def cpu_baseline(seconds, threads=None):
    """The C path (reference BitmessagePOW) at the box's CPU share and, when the process may run
    on more CPUs than that, at every CPU of its affinity mask too; the Fast path (_doFastPoW
    mechanism) at the share.  `value` = the best rate; every leg is reported."""
    info = host_cpu_info()
    share = threads or info['share']
    legs = {'c_share': _cpu_leg(seconds, share, 'c')}
    if info['affinity'] > share:
        legs['c_all_cpus'] = _cpu_leg(max(4.0, seconds / 2), info['affinity'], 'c')
    legs['fast_share'] = _cpu_leg(seconds, share, 'fast')
    ok = {k: v for k, v in legs.items() if 'ghs' in v}
    if not ok:
        return {'error': legs, 'host': info}
    best_key = max(ok, key=lambda k: ok[k]['ghs'])
    best = ok[best_key]
    what = {'c': 'oracle/_ref/bitmsghash.so (reference BitmessagePOW compiled from its source, OpenSSL SHA512, '
                 'pthreads)' if best['kind'] == 'reference' else 'oracle/liboracle.so bmo_search_mt (port)',
            'fast': 'the _doFastPoW mechanism (oracle/fastpow.py: hashlib, multiprocessing Pool, 0.2 s polling)'}
    return {'value': round(best['ghs'], 6), 'unit': 'GH/s', 'cores': best['cores'],
            'kind': 'reference' if best['kind'] in ('reference', 'reference-mechanism') else 'port',
            'objects_per_s': round(best['objects_per_s'], 4), 'best_leg': best_key,
            'sample': '%d C2 objects (the first of the rank-0 batch) solved in %.1f s by %s on %d host CPUs; '
                      'rate = sum(nonce)/time' % (best['objects'], best['seconds'], what[best['mode']], best['cores']),
            'host': info,
            'legs': {k: ({'ghs': round(v['ghs'], 6), 'cores': v['cores'], 'objects': v['objects'],
                          'seconds': round(v['seconds'], 2), 'kind': v['kind']} if 'ghs' in v else v)
                     for k, v in legs.items()}}


# ----------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='c2', choices=['c1', 'c2', 'c3', 'c4', 'c5', 'verify', 'addrgen'])
    ap.add_argument('--null-bytes', type=int, default=3, help='addrgen: leading zero bytes of the ripe')
    ap.add_argument('--addr-mode', default='det', choices=['det', 'random'],
                    help='addrgen: deterministic (passphrase) or random (fixed signing key) keys')
    ap.add_argument('--addr-comb', type=int, default=24, choices=[0, 16, 24],
                    help='addrgen: comb window bits (0 = the library\'s automatic choice)')
    ap.add_argument('--objects', type=int, default=None, help='override the object count (c2/c4/c5)')
    ap.add_argument('--c3-log2', type=int, default=36)
    ap.add_argument('--step-trials', type=int, default=0, help='per-launch trial budget per GPU (0 = lib default)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--cpu-threads', type=int, default=0, help='CPU-baseline threads (0 = the box\'s CPU share)')
    ap.add_argument('--cpu-mode', default='c', choices=['c', 'fast', 'verify'], help=argparse.SUPPRESS)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--share-device', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--devices', type=int, default=0,
                    help='one process driving this many GPUs in-process (bmpow_set_devices: one stepper thread '
                         'per device claiming windows of the objects, host min-reduction); 0 = one GPU per rank')
    ap.add_argument('--shards-per-device', type=int, default=1,
                    help='--devices: this many shards (streams, each with its own stepper) per device -- on a '
                         'one-GPU box, a rehearsal of the multi-device path, not a scaling number')
    ap.add_argument('--test-mode', action='store_true',
                    help='c5: the reference\'s test-mode difficulty (ntpb and extra / 100): 100k objects of '
                         '~2e4 trials each, so per-object host and launch costs dominate')
    ap.add_argument('--run-batch', action='store_true',
                    help='c2/c5: through proofofwork.run_batch (the product entry point, host re-check included)')
    ap.add_argument('--service', action='store_true',
                    help='c2/c5: feed the objects through worker.PowService (the library\'s continuous-batching '
                         'service, bmpow_service_submit/poll) instead of one batch')
    ap.add_argument('--no-exact', action='store_true',
                    help='skip the min-trial proof of a seeded sample of the answers (after the timed region)')
    ap.add_argument('--run-split', action='store_true',
                    help='run() legs (c1, c3, --serial): one piece per shard even where shards share a device '
                         '(bmpow_set_run_split; the multi-device path rehearsed on one GPU)')
    ap.add_argument('--engine-split', action='store_true',
                    help='--devices: every shard its own device group (bmpow_set_engine_split), so windows split '
                         'over shards that share a GPU -- the multi-device split rehearsed on one GPU')
    ap.add_argument('--no-nonce-sharded', action='store_true',
                    help='N > 1: skip the in-process nonce-sharded C3/C4 leg after the timed region')
    ap.add_argument('--serial', action='store_true',
                    help='c2/c4/c5: the objects one after another through proofofwork.run (the reference\'s '
                         'serial call sites), not as one batch')
    ap.add_argument('--throttle', default=None,
                    help='--devices A/B: "shard:ms" -- that shard\'s stepper sleeps ms before each launch')
    ap.add_argument('--cpu-baseline-worker', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--nonce-sharded-child', type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_worker:
        cpu_baseline_worker(args.cpu_seconds, args.cpu_threads, args.cpu_mode)
        return
    if args.nonce_sharded_child:
        os.environ['BMPOW_DEVICES'] = '0'
        from pybitmessage_amd import _lib
        print(json.dumps(nonce_sharded(_lib.get(), args.nonce_sharded_child, args.share_device)), flush=True)
        return

    dist = Dist()
    # one process per GPU; --share-device puts every rank on GPU 0 (rehearsing the multi-rank
    # path on a one-GPU box: the ranks then split one GPU, so the value is not a scaling number)
    if args.devices:
        if dist.world > 1:
            raise SystemExit('--devices drives several GPUs from one process: run it without torch.distributed')
        os.environ['BMPOW_DEVICES'] = ','.join(str(i) for i in range(args.devices) for _ in range(args.shards_per_device))
    else:
        os.environ['BMPOW_DEVICES'] = str(rank_device(dist, args.share_device))
    from pybitmessage_amd import _lib
    lib = _lib.get()
    if args.step_trials:
        lib.bmpow_set_step_trials(args.step_trials)
    if args.run_split:
        lib.bmpow_set_run_split(1)
    if args.engine_split:
        lib.bmpow_set_engine_split(1)
    if args.throttle:
        shard, ms = args.throttle.split(':')
        _lib.check(lib, lib.bmpow_set_shard_throttle(int(shard), float(ms)), 'bmpow_set_shard_throttle')

    if args.config == 'addrgen':
        r = run_addr_bench(args, dist)
        line = summarize_addr(args, dist, r, lib.bmpow_version().decode())
        if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_addr_baseline(min(args.cpu_seconds, 10.0), args.addr_mode)
        if dist.rank == 0:
            print(json.dumps(line), flush=True)
        dist.close()
        return
    if args.config == 'verify':
        r = run_verify_bench(args, dist)
        line = summarize_verify(args, dist, r, lib.bmpow_version().decode())
        if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
            line['cpu_baseline'] = cpu_verify_baseline(min(args.cpu_seconds, 10.0))
        if dist.rank == 0:
            print(json.dumps(line), flush=True)
        dist.close()
        return
    runner = {'c1': run_c1_bench, 'c2': run_batch_bench, 'c3': run_c3_bench, 'c4': run_batch_bench,
              'c5': run_batch_bench}[args.config]
    if args.service or args.run_batch:
        if args.config not in ('c2', 'c5'):
            raise SystemExit('--service / --run-batch apply to c2 and c5')
        runner = run_service_bench if args.service else run_runbatch_bench
    if args.serial:
        if args.config not in ('c2', 'c4', 'c5'):
            raise SystemExit('--serial applies to c2, c4 and c5')
        runner = run_serial_bench
    if args.devices:
        n = lib.bmpow_get_devices((ctypes.c_int * 64)(), 64)
        if n != args.devices * args.shards_per_device:
            raise SystemExit('asked for %d shards, the library selected %d' % (args.devices * args.shards_per_device, n))
    r = runner(args, dist)
    r['devices'] = args.devices
    r['pci_bus_id'] = device_pci_bus_id(lib)
    line = summarize(args, dist, r, lib.bmpow_version().decode())
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline(args.cpu_seconds, args.cpu_threads or None)
    if dist.world > 1 and not args.devices and not args.no_nonce_sharded and args.config in ('c2', 'c4', 'c5'):
        # the nonce split over the node's GPUs (C3, C4), outside the timed region: rank 0 alone, in a
        # child process under a time limit, so a failure there costs this line nothing but the field
        dist.barrier()
        if dist.rank == 0:
            line['nonce_sharded'] = run_nonce_sharded_child(dist.world, args.share_device)
        dist.barrier()
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


def per_device(lib, ids):
    """Work per physical device of the shard set `ids` since bmpow_reset_stats: PCI bus id, trials and
    summed kernel time of its shards (bmpow_get_shard_stats: the engine's launches and run()'s pieces)."""
    tr, ms = (ctypes.c_uint64 * 64)(), (ctypes.c_double * 64)()
    n = lib.bmpow_get_shard_stats(tr, ms, 64)
    out = []
    for dev in sorted(set(ids)):
        shards = [i for i, d in enumerate(ids) if d == dev and i < n]
        buf = ctypes.create_string_buffer(64)
        bus = buf.value.decode() if lib.bmpow_device_pci_bus_id(dev, buf, 64) >= 0 else None
        out.append({'device': dev, 'pci_bus_id': bus, 'shards': len(shards),
                    'trials': int(sum(tr[i] for i in shards)), 'kernel_ms': round(sum(ms[i] for i in shards), 2)})
    return out


def nonce_sharded(lib, n, share=False, c3_log2=38, c4_objs=None):
    """The north star's nonce split on a multi-GPU node (BASELINE.json C3 and C4 over 1/2/4/8 GPUs),
    measured in ONE process over n devices -- the SCALE run's ranks each drive one GPU with object
    sharding, which never splits an object.  Run by rank 0 after the timed region while the other ranks
    wait at a barrier (their GPUs idle):
      * C3: a run() sweep of 2^c3_log2 nonces with no hit (target 0), one interleaved piece per device
        sharing the cross-device bound: every nonce hashed exactly once (2^38: BASELINE.json's C3 size,
        ~5 s over 8 GPUs, ~41 s when a one-GPU rehearsal puts every piece on one device);
      * C4: the 64 objects of 20x difficulty as one batch on the engine, one stepper per device (object
        mode, then windows split over the devices at the tail), answers re-hashed with hashlib.
    Falls back to n shards of device 0 when fewer than n devices are visible (then a rehearsal: the
    per_device list shows one bus id).  The rank's own device selection is restored after."""
    from pybitmessage_amd import _lib, proofofwork
    import numpy as np
    visible = lib.bmpow_device_count()
    ids = [0] * n if share or visible < n else list(range(n))
    own = (ctypes.c_int * 64)()
    k = lib.bmpow_get_devices(own, 64)
    own_ids = list(own[:k])
    _lib.check(lib, lib.bmpow_set_devices((ctypes.c_int * n)(*ids), n), 'bmpow_set_devices')
    out = {'devices': ids, 'device_groups': len(set(ids)),
           'what': 'rank 0 alone after the timed region, one process over %d device(s) (bmpow_set_devices); the '
                   'other ranks at a barrier%s' % (len(set(ids)), '' if len(set(ids)) == n else
                                                   ' -- fewer devices visible than ranks: a rehearsal, not scaling')}
    try:
        # C3: no hit anywhere in [1, 2^k]: exactly 2^k trials over the pieces
        ih = hashlib.sha512(b'bmpow-sweep').digest()
        nn, tt = ctypes.c_uint64(), ctypes.c_uint64()
        lib.bmpow_reset_stats()
        t0 = time.perf_counter()
        rc = _lib.check(lib, lib.bmpow_search(ih, 0, 1, 1 << c3_log2, ctypes.byref(nn), ctypes.byref(tt)), 'search')
        el = time.perf_counter() - t0
        st = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(st))
        out['c3'] = {'nonces': 1 << c3_log2, 'seconds': round(el, 3), 'ghs': round((1 << c3_log2) / el / 1e9, 4),
                     'not_found': rc == _lib.NOT_FOUND, 'trials_exact': int(st.trials) == 1 << c3_log2,
                     'per_device': per_device(lib, ids)}
        # C4: the batch, exact answers
        objs = c4_objs if c4_objs is not None else make_objects('c4', 0)[0]
        m = len(objs)
        tg = np.array([t for t, _ in objs], dtype=np.uint64)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        h = lib.bmpow_batch_create(m, b''.join(ih for _, ih in objs), tg.ctypes.data_as(p64), None)
        if not h:
            raise RuntimeError('bmpow_batch_create: %s' % lib.bmpow_last_error().decode())
        try:
            lib.bmpow_reset_stats()
            t0 = time.perf_counter()
            solve_batch(lib, h)
            el = time.perf_counter() - t0
            st = _lib.BmpowStats()
            lib.bmpow_get_stats(ctypes.byref(st))
            nonce, trial = np.zeros(m, dtype=np.uint64), np.zeros(m, dtype=np.uint64)
            done = np.zeros(m, dtype=np.uint8)
            lib.bmpow_batch_results(h, nonce.ctypes.data_as(p64), trial.ctypes.data_as(p64),
                                    done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), None)
        finally:
            lib.bmpow_batch_destroy(h)
        for i in range(m):
            assert done[i] == _lib.DONE_FOUND
            proofofwork._verify(int(tg[i]), objs[i][1], int(trial[i]), int(nonce[i]))
        useful = float(sum(int(x) for x in nonce))
        out['c4'] = {'objects': m, 'seconds': round(el, 3), 'ghs': round(useful / el / 1e9, 4),
                     'performed_ghs': round(int(st.trials) / el / 1e9, 4),
                     'wasted_frac': round(1.0 - useful / int(st.trials), 5) if st.trials else None,
                     'past_answers': past_answers(st), 'per_device': per_device(lib, ids)}
    finally:
        lib.bmpow_set_devices((ctypes.c_int * len(own_ids))(*own_ids), len(own_ids))
    out['c3_ghs'], out['c4_ghs'] = out['c3']['ghs'], out['c4']['ghs']
    out['c4_wasted_frac'] = out['c4']['wasted_frac']
    return out


def run_nonce_sharded_child(n, share=False, timeout=600, argv=None):
    """nonce_sharded over n devices in a child process (`bench.py --nonce-sharded-child N`), bounded by
    `timeout` seconds: its JSON, or {'error': ...} when it fails, times out or prints none."""
    argv = argv or ([sys.executable, os.path.abspath(__file__), '--nonce-sharded-child', str(n)] +
                    (['--share-device'] if share else []))
    env = dict(os.environ)
    for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)  # the child is a single process
    try:
        r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {'error': 'timed out after %d s' % timeout}
    lines = [x for x in r.stdout.splitlines() if x.startswith('{')]
    if r.returncode != 0 or not lines:
        return {'error': 'exit status %d' % r.returncode, 'stderr': r.stderr[-800:]}
    return json.loads(lines[-1])


def device_pci_bus_id(lib, shard=0):
    """PCI bus id of the device a shard runs on (bmpow_device_pci_bus_id), or None."""
    if not hasattr(lib, 'bmpow_device_pci_bus_id'):
        return None
    ids = (ctypes.c_int * 64)()
    if lib.bmpow_get_devices(ids, 64) <= shard:
        return None
    buf = ctypes.create_string_buffer(64)
    if lib.bmpow_device_pci_bus_id(ids[shard], buf, 64) < 0:
        return None
    return buf.value.decode()


def rank_device(dist, share=False, visible=None):
    """The device ordinal this rank drives: its LOCAL_RANK among the visible gfx950 devices.  A launcher
    that gives every rank one GPU of its own through HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES leaves one
    visible device per rank: then device 0 (that rank's own GPU).  --share-device: device 0 for every
    rank (a rehearsal on one GPU)."""
    if share:
        return 0
    if visible is None:
        from pybitmessage_amd import _lib
        visible = _lib.load().bmpow_device_count()  # counts without selecting (bmpow_init reads the choice)
    if visible == 1 and dist.local_rank > 0:
        return 0
    if dist.local_rank >= max(visible, 1):
        raise SystemExit('rank %d (local rank %d) has no GPU: %d visible' % (dist.rank, dist.local_rank, visible))
    return dist.local_rank


def summarize(args, dist, r, lib_version):
    """Whole-job line: max-over-ranks wall time, sum-over-ranks work (every rank calls it)."""
    st = r['stats']
    el_max = dist.reduce(r['elapsed'], 'max')
    useful = dist.reduce(r['useful'], 'sum')
    objects = dist.reduce(r['objects'], 'sum')
    performed = dist.reduce(st.trials, 'sum')
    kernel_ms = st.kernel_ms
    launches = st.launches
    line = {
        'metric': METRIC,
        'value': round(useful / el_max / 1e9, 4),
        'unit': 'GH/s',
        'n_gpus': dist.world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(el_max * 1e3 / args.steps, 2),
        'higher_is_better': True,
        'scaling': r.get('scaling', 'weak'),
        'vs_baseline': None,
        'dtype': 'u64',
        'data': 'synthetic',
        'config': {'workload': r['desc'], 'objects_per_rank_per_step': r['objects'] // max(args.steps, 1),
                   'parallelism': 'object-sharded dp%d (one process per GPU, no collective)' % dist.world,
                   'block': 256, 'lib': lib_version},
        'objects_per_s': round(objects / el_max, 3),
        'performed_ghs': round(performed / el_max / 1e9, 4),
        'wasted_frac': round(1.0 - useful / performed, 5) if performed else None,
    }
    cut = dist.reduce(getattr(st, 'cut_trials', 0), 'sum')
    if cut:
        # run()'s kernel: nonces that hashed only their first compression before the call's answer
        # was published below them (not in performed); as half-trials, the work they cost
        line['cut_trials'] = int(cut)
        line['wasted_frac_incl_cut'] = round(1.0 - useful / (performed + 0.5 * cut), 5)
    # per-GPU kernel rate, averaged over the ranks (each rank's device-counted trials over its own
    # summed kernel time, HIP events on the launching stream); one rank: that GPU's
    rank_ghs = st.trials / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    mean_ghs = dist.reduce(rank_ghs, 'sum') / dist.world
    min_ghs = -dist.reduce(-rank_ghs, 'max')
    if mean_ghs > 0:
        kernel_ghs = mean_ghs
        achieved = OPS_PER_TRIAL * kernel_ghs * 1e9 / 1e12
        line['roofline'] = {
            'bound': 'valu', 'kernel': r.get('kernel', 'bm_search_kernel'),
            'achieved': round(achieved, 3), 'peak': round(PEAK_TOPS, 3),
            'unit': 'T int32 lane-ops/s (8,288 algorithmic ops per trial)',
            'frac': round(achieved / PEAK_TOPS, 4), 'traffic': None,
            'scope': ('per GPU: one MI355X' if dist.world == 1 else
                      'per GPU: mean over the %d ranks (min %.4f GH/s); peak is one GPU\'s' % (dist.world, min_ghs)),
            'kernel_ghs': round(kernel_ghs, 4),
            'avg_launch_ms': round(kernel_ms / max(launches, 1), 3), 'launches': int(launches),
            'kernel_busy_frac': round(kernel_ms * 1e-3 / r['elapsed'], 4),
        }
        pmc = pmc_counters(r.get('kernel', 'bm_search_kernel'))
        if pmc:
            # PMC bytes per 2^28-trial launch, scaled to this run's launches (the traffic -- the block
            # queue's atomics and the item loads -- grows with the trials a launch hashes)
            pmc_traffic, pmc_trials = pmc.pop('traffic'), pmc.pop('trials_per_launch', None)
            per_launch = st.trials / max(launches, 1)
            if pmc_traffic is not None and pmc_trials:
                line['roofline']['traffic'] = round(pmc_traffic * per_launch / pmc_trials)
                line['roofline']['traffic_basis'] = ('%.0f B per %d-trial PMC launch x %.0f trials per launch here'
                                                     % (pmc_traffic, pmc_trials, per_launch))
            else:
                line['roofline']['traffic'] = pmc_traffic
            line['roofline']['counters'] = pmc
            if pmc.get('valu_instr_per_trial') and pmc.get('eff_clock_ghz'):
                # one wave64 VALU instruction per SIMD per quad-cycle, at the PMC run's clock
                ceil = SIMDS * pmc['eff_clock_ghz'] * 1e9 / 4 * 64 / pmc['valu_instr_per_trial'] / 1e9
                line['roofline']['single_issue_ceiling'] = {
                    'ghs': round(ceil, 4), 'frac': round(kernel_ghs / ceil, 4),
                    'basis': '1,024 SIMDs x one VALU instruction per quad-cycle x 64 lanes / VALU instructions '
                             'per trial (SQ_INSTS_VALU), at the PMC run clock (GRBM_GUI_ACTIVE / 8 / kernel time)'}
                # every v_bitop3_b32 paired with another wave's: the hard issue bound of this
                # instruction mix (the other 73 % issue one per quad-cycle)
                slots = pmc['valu_instr_per_trial'] - BITOP3_PER_TRIAL / 2
                pceil = SIMDS * pmc['eff_clock_ghz'] * 1e9 / 4 * 64 / slots / 1e9
                line['roofline']['all_pairs_bound'] = {
                    'ghs': round(pceil, 4), 'frac': round(kernel_ghs / pceil, 4),
                    'basis': 'one issue slot per quad-cycle for each VALU instruction but a pair of v_bitop3_b32 '
                             '(%d per trial, tools/isa_census.py) sharing one: (VALU per trial - %d / 2) slots'
                             % (BITOP3_PER_TRIAL, BITOP3_PER_TRIAL)}
                mix = free_running_mix()
                if mix:
                    # what the kernel's instruction mix issues free-running (no dependences, no
                    # barriers): a measured reference point, not a ceiling -- the kernel itself issues
                    # more, its per-block barrier phasing the waves better
                    line['roofline']['free_running_mix'] = dict(mix, ghs=round(ceil * mix['valu_per_simd_quadcycle'], 4))
    if r.get('host_cpu'):
        line['host_cpu_per_s'] = r['host_cpu']['process_cpu_per_s']
        line['host_cpu'] = r['host_cpu']
        w1 = one_wait(st, r['elapsed'])
        if w1:
            line['host_cpu']['wait']['run_calls'] = w1
    if r.get('exact_sample'):
        line['exact_sample'] = r['exact_sample']
    pa = past_answers(st)
    if pa:
        line['past_answers'] = pa
    if dist.world > 1:
        # which physical GPU each rank drove, and its work: a reader can see that N distinct devices
        # (PCI bus ids) did the job -- the one-GPU rehearsals (--share-device) show one id
        line['per_rank'] = dist.gather({'rank': dist.rank, 'local_rank': dist.local_rank,
                                        'device_pci_bus_id': r.get('pci_bus_id'), 'trials': int(st.trials),
                                        'kernel_ms': round(float(kernel_ms), 3),
                                        'elapsed_s': round(float(r['elapsed']), 4)})
    for k in ('call_ms', 'path', 'per_call'):
        if r.get(k) is not None:
            line[k] = r[k]
    if r.get('devices'):
        spd = getattr(args, 'shards_per_device', 1)
        line['config']['parallelism'] = ('in-process over %d device(s) x %d shard(s): one stepper thread and stream '
                                         'per shard claiming windows from the objects\' frontiers (bmsched::Engine), '
                                         'host min-reduction, no collective%s'
                                         % (r['devices'], spd, '; shards share a GPU: a rehearsal of the multi-device '
                                            'path, not a scaling number' if spd > 1 else ''))
        line['n_gpus'] = r['devices']
        if args.throttle:
            line['config']['throttle'] = args.throttle
        import ctypes

        from pybitmessage_amd import _lib
        lib = _lib.get()
        rates = (ctypes.c_double * 64)()
        n = lib.bmpow_get_shard_rates(rates, 64)
        line['shard_rates_ghs'] = [round(rates[i] * 1e3 / 1e9, 4) for i in range(min(n, 64))]
        tr, ms = (ctypes.c_uint64 * 64)(), (ctypes.c_double * 64)()
        n = lib.bmpow_get_shard_stats(tr, ms, 64)
        line['shard_stats'] = [{'trials': int(tr[i]), 'kernel_ms': round(ms[i], 2),
                                'busy_frac': round(ms[i] * 1e-3 / r['elapsed'], 4)} for i in range(min(n, 64))]
    return line


def free_running_mix():
    """bm_search_kernel's nonce-loop VALU stream issued free-running (profiles/mix_ceiling.json, from
    tools/ubench_mix.py on the GPU box): opcode for opcode, data dependences removed, every
    v_bitop3_b32 bank-split, best of the compiler's order, an even spread and grouped bitop3.  The
    kernel issues more per quad-cycle than this stream (round 3), so it is reported as a measured
    reference point, not as a ceiling."""
    path = os.path.join(ROOT, 'profiles', 'mix_ceiling.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return {'valu_per_simd_quadcycle': d['ceiling_valu_per_simd_quadcycle'], 'waves_per_simd': d['waves_per_simd'],
            'source': 'profiles/mix_ceiling.json (%s)' % d['source']}


def lib_md5(path):
    import hashlib as hl
    try:
        with open(path, 'rb') as f:
            return hl.md5(f.read()).hexdigest()
    except OSError:
        return None


def pmc_counters(kernel='bm_search_kernel'):
    """bm_search_kernel's hardware counters from the committed rocprofv3 PMC passes
    (tools/profile_pmc.sh -> tools/pmc_summary.py -> profiles/pmc_latest.json; C3 launches of 2^28
    trials, one counter group per pass): HBM bytes per launch = FETCH_SIZE doubled (gfx950
    under-count, MI355X_MICROARCH.md section HBM) + WRITE_SIZE -- the algorithmic traffic is ~0 (9
    words per workgroup) --, and the VALU issue figures (SQ_ACTIVE_INST_VALU / _VALU2 per SIMD
    quad-cycle)."""
    # run()'s bm_search1_kernel has its own passes (tools/profile_pmc.sh with PMC_ONE=1), when committed
    name = 'pmc_one_latest.json' if kernel == 'bm_search1_kernel' else 'pmc_latest.json'
    path = os.path.join(ROOT, 'profiles', name)
    if not os.path.exists(path):
        if name == 'pmc_latest.json':
            return None
        name, kernel = 'pmc_latest.json', 'bm_search_kernel'
        path = os.path.join(ROOT, 'profiles', name)
        if not os.path.exists(path):
            return None
    with open(path) as f:
        full = json.load(f)
    d = full['derived']
    out = {'traffic': d.get('hbm_bytes_per_launch_upper'),
           'source': 'profiles/%s (%s, C3, 2^28-trial launches)' % (name, kernel),
           'build': full.get('build'), 'trials_per_launch': full.get('raw', {}).get('trials_per_launch')}
    # provenance: were the counters collected on the device code this run loaded?  The device code's
    # md5 (the .hip_fatbin section, tools/lib_code_md5.py) is reproduced by a rebuild of the same
    # sources; the whole file's md5 is not (the host code carries the build time)
    from pybitmessage_amd import _lib
    try:
        from tools.lib_code_md5 import code_md5
    except ImportError:  # (a tree without tools/: the whole file's md5 decides)
        def code_md5(_path):
            return None
    build = full.get('build') or {}
    out['benched_lib_md5'] = lib_md5(_lib.lib_path())
    out['benched_code_md5'] = code_md5(_lib.lib_path())
    if build.get('code_md5') and out['benched_code_md5']:
        out['stale'] = build['code_md5'] != out['benched_code_md5']
    else:
        out['stale'] = out['benched_lib_md5'] is None or build.get('lib_md5') != out['benched_lib_md5']
    for k in ('valu_instr_per_trial', 'valu_issue_util', 'valu_instr_per_simd_quad_cycle', 'dual_issue_share',
              'simd_busy_frac', 'wave_issue_stall_share', 'wave_wait_share', 'eff_clock_ghz'):
        if d.get(k) is not None:
            out[k] = round(d[k], 4)
    return out


if __name__ == '__main__':
    main()
