"""Soak: every entry point of the product at once, for BMPOW_SOAK_S seconds (default 30), with the shard
layout changing between phases -- the way a long-running node uses the library.

* A PowService (the worker thread's batches, class_singleWorker.py:219-250 through run_batch's service)
  takes random batches of 1-64 objects;
* two threads make serial run() calls (api.py:1304,1350 and the worker's ack-then-msg,
  class_singleWorker.py:236,1276) -- run()'s single-object path, split into pieces where the phase
  forces it;
* one thread calls run_batch on small batches (a fresh service per call beside the long-lived one);
* one thread verifies batches of received objects (isProofOfWorkSufficient_batch, the receive side,
  protocol.py:258-286): objects given a valid nonce by run_batch at the network difficulty, the same
  with one payload byte changed, and objects with random nonces, each verdict against targets.py's
  per-object restatement.

Phases, run three times over: one shard; two shards sharing the device (objects nonce-sharded between them,
cross-shard bound slots in use); three forced run() pieces on CU slices; four shards.  Every answer is
re-hashed (trial <= target) and, while the checkers keep up, proven minimal with the C oracle
(oracle/); the rest is counted as checked for validity only.  The process's resident memory at the end
of each phase of the third pass is compared with the same phase of the second (after gc and
malloc_trim): a leak per call or per layout change shows there, while what a layout holds (its streams,
rings and staging buffers) and the HIP runtime's high-water marks, set in the first pass, do not
(tools/diag/rss_layout.py).
"""
import ctypes
import gc
import hashlib
import os
import queue
import random
import threading
import time

import pytest

from tests.test_gpu_engine import run_split  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu
U64 = (1 << 64) - 1
SOAK_S = float(os.environ.get('BMPOW_SOAK_S', '30'))
PHASES = (([0], False), ([0, 0], False), ([0, 0, 0], True), ([0, 0, 0, 0], False))
# BMPOW_SOAK_LAYOUTS=wide: eight shards, with and without forced pieces, and two forced pieces
if os.environ.get('BMPOW_SOAK_LAYOUTS') == 'wide':
    PHASES = (([0] * 8, False), ([0] * 8, True), ([0, 0], True), ([0], False))
EXPECT = (20, 200, 2000, 20000, 200000)      # expected trials per object (target = 2^64 / E)
WEIGHT = (2, 3, 3, 2, 1)
BACKLOG = 400                                  # past this many unchecked answers: validity only


def _rss():
    gc.collect()
    ctypes.CDLL(None).malloc_trim(0)
    with open('/proc/self/statm') as f:
        return int(f.read().split()[1]) * os.sysconf('SC_PAGE_SIZE')


def _object(rng):
    e = rng.choices(EXPECT, WEIGHT)[0]
    return U64 // e, rng.randbytes(64)


def test_soak_every_entry_point_at_once(gpulib, shards, run_split, coracle):  # noqa: F811
    from pybitmessage_amd import proofofwork, targets, verify, worker
    phases = PHASES * 3
    per = SOAK_S / len(phases)
    rss = []
    for p, (layout, split) in enumerate(phases):
        shards(layout)
        run_split(split)
        stop = threading.Event()
        todo = queue.Queue()
        counts = {'service': 0, 'serial': 0, 'batch': 0, 'verify': 0, 'valid': 0}
        stats = {'minimal': 0, 'valid_only': 0}
        bad, crashed = [], []
        lock = threading.Lock()

        def put(kind, t, ih, got):
            todo.put((kind, t, ih, [int(x) for x in got], todo.qsize() < BACKLOG))
            with lock:
                counts[kind] += 1

        def guard(fn):
            def body(*a):
                try:
                    fn(*a)
                except Exception as e:  # surfaced by the assertion below
                    crashed.append(repr(e))
                    stop.set()
            return body

        @guard
        def service_loop(svc, rng):
            while not stop.is_set():
                objs = [_object(rng) for _ in range(rng.randint(1, 64))]
                for (t, ih), f in zip(objs, svc.submit_many(objs)):
                    put('service', t, ih, f.result(timeout=120))

        @guard
        def serial_loop(rng):
            while not stop.is_set():
                t, ih = _object(rng)
                put('serial', t, ih, proofofwork.run(t, ih))

        @guard
        def batch_loop(rng):
            while not stop.is_set():
                objs = [_object(rng) for _ in range(rng.randint(1, 8))]
                for (t, ih), r in zip(objs, proofofwork.run_batch(objs)):
                    put('batch', t, ih, r)

        @guard
        def verify_loop(rng):
            while not stop.is_set():
                now = int(time.time())
                # a few objects given a valid nonce by run_batch (TTL 300 s, network difficulty), the
                # same with a payload byte changed, and objects with random nonces
                made = [(now + 300).to_bytes(8, 'big') + rng.randbytes(rng.randint(8, 200))
                        for _ in range(rng.randint(1, 4))]
                sol = proofofwork.run_batch([(int(targets.object_target(len(m), 300)), hashlib.sha512(m).digest())
                                             for m in made])
                good = [nonce.to_bytes(8, 'big') + m for (_, nonce), m in zip(sol, made)]
                bent = [o[:-1] + bytes([o[-1] ^ 1]) for o in good]
                junk = [rng.randbytes(8) + (now + rng.randint(-3600, 30000)).to_bytes(8, 'big')
                        + rng.randbytes(rng.randint(6, 1000)) for _ in range(rng.randint(1, 512))]
                objs = good + bent + junk
                rng.shuffle(objs)
                got = verify.isProofOfWorkSufficient_batch(objs, 0, 0, now)
                want = [targets.isProofOfWorkSufficient(o, 0, 0, now) for o in objs]
                if got != want or not all(targets.isProofOfWorkSufficient(o, 0, 0, now) for o in good):
                    bad.append(('verify', [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:4]))
                with lock:
                    counts['verify'] += len(objs)
                    counts['valid'] += sum(got)

        def checker():
            while True:
                item = todo.get()
                if item is None:
                    return
                kind, t, ih, got, full = item
                if full:
                    ok = list(coracle.search(ih, t)) == got
                else:
                    ok = got[0] <= t and coracle.trial(got[1], ih) == got[0]
                with lock:
                    stats['minimal' if full else 'valid_only'] += 1
                if not ok:
                    bad.append((kind, t, ih.hex(), got))

        checkers = [threading.Thread(target=checker) for _ in range(4)]
        for c in checkers:
            c.start()
        svc = worker.PowService().start()
        rngs = [random.Random(9000 + 10 * p + k) for k in range(5)]
        th = [threading.Thread(target=service_loop, args=(svc, rngs[0])),
              threading.Thread(target=serial_loop, args=(rngs[1],)),
              threading.Thread(target=serial_loop, args=(rngs[2],)),
              threading.Thread(target=batch_loop, args=(rngs[3],)),
              threading.Thread(target=verify_loop, args=(rngs[4],))]
        t0 = time.time()
        for x in th:
            x.start()
        stop.wait(per)
        stop.set()
        for x in th:
            x.join(120)
        svc.stop(30)
        for _ in checkers:
            todo.put(None)
        for c in checkers:
            c.join(300)
        rss.append(_rss())
        print('soak phase %d layout=%s split=%s %.1fs answers=%s checked=%s rss=%.1f MiB'
              % (p, layout, split, time.time() - t0, counts, stats, rss[-1] / 2**20), flush=True)
        assert not crashed, crashed
        assert not any(x.is_alive() for x in th)
        assert not bad, bad[:4]
        assert all(counts[k] > 0 for k in counts), counts
        assert stats['minimal'] >= min(100, counts['service'] + counts['serial'] + counts['batch']), stats
    n = len(PHASES)
    growth = max(b - a for a, b in zip(rss[n:2 * n], rss[2 * n:]))
    assert growth < 64 * 2**20, 'resident memory grew by %.1f MiB between passes (%s MiB)' % (
        growth / 2**20, [round(x / 2**20) for x in rss])
