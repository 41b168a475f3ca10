"""GPU parity: the HIP path through the C ABI vs the oracle and the reference's golden
vectors.  Bit-exact everywhere (integer work).  Run on an MI355X: pytest -m gpu."""
import ctypes
import hashlib
import random
import threading
import time

import numpy as np
import pytest


from pybitmessage_amd import _lib, proofofwork, state

pytestmark = pytest.mark.gpu
U64 = (1 << 64) - 1
P64 = ctypes.POINTER(ctypes.c_uint64)


def gpu_trials(lib, ih, nonces):
    nonces = np.ascontiguousarray(nonces, dtype=np.uint64)
    out = np.zeros_like(nonces)
    _lib.check(lib, lib.bmpow_trials(ih, nonces.ctypes.data_as(P64), nonces.size, out.ctypes.data_as(P64)),
               'bmpow_trials')
    return out


def gpu_search(lib, ih, target, start=1, max_trials=1 << 40):
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    rc = _lib.check(lib, lib.bmpow_search(ih, target, start, max_trials, ctypes.byref(n), ctypes.byref(t)),
                    'bmpow_search')
    return (t.value, n.value) if rc == _lib.FOUND else None


# ---------------- trial function ----------------
def test_trial_kats_bit_exact(gpulib, golden):
    kats = golden('trial_kats.json')['kats']
    by_ih = {}
    for k in kats:
        by_ih.setdefault(k['ih'], []).append(k)
    for ihx, ks in by_ih.items():
        got = gpu_trials(gpulib, bytes.fromhex(ihx), [k['nonce'] for k in ks])
        assert [int(x) for x in got] == [k['trial'] for k in ks]


def test_trials_random_vs_c_oracle(gpulib, coracle):
    rng = np.random.default_rng(5)
    for r in range(4):
        ih = rng.bytes(64)
        nonces = rng.integers(0, 2 ** 63, size=20000, dtype=np.uint64) * np.uint64(2) + np.uint64(r & 1)
        nonces[:256] = np.arange(256, dtype=np.uint64)           # small nonces
        nonces[256:512] = np.uint64(U64) - np.arange(256, dtype=np.uint64)  # top of the space
        assert np.array_equal(gpu_trials(gpulib, ih, nonces), coracle.trials(ih, nonces))


# ---------------- first-nonce search ----------------
def test_first_nonce_kats(gpulib, golden):
    for k in golden('first_nonce_kats.json')['kats']:
        got = gpu_search(gpulib, bytes.fromhex(k['ih']), k['target'])
        assert got == (k['trial'], k['nonce']), k['note']


def test_batch_kats_run_batch(gpulib, golden):
    d = golden('batch_kats.json')
    objs = [(k['target'], bytes.fromhex(k['ih'])) for k in d['kats']]
    res = proofofwork.run_batch(objs)
    assert res == [[k['trial'], k['nonce']] for k in d['kats']]


def test_run_matches_golden(gpulib, golden):
    for k in golden('first_nonce_kats.json')['kats'][:12]:
        assert proofofwork.run(k['target'], bytes.fromhex(k['ih'])) == [k['trial'], k['nonce']]


def test_random_batch_vs_c_oracle(gpulib, coracle):
    rng = random.Random(99)
    objs = []
    for _ in range(300):
        ih = rng.randbytes(64)
        objs.append((U64 // rng.choice([1, 2, 7, 100, 1000, 30000, 200000]), ih))
    want = [list(r) for r in coracle.search_many(objs)]
    assert proofofwork.run_batch(objs) == want


@pytest.mark.parametrize('layout,split', [([0], False), ([0, 0, 0], False), ([0, 0, 0], True)])
def test_duplicate_objects_and_one_hash_many_targets(gpulib, shards, engine_split, coracle, layout, split):
    """A batch may hold the same object more than once (the same payload queued twice) and one
    initialHash under several targets (a payload re-sent at another difficulty): each entry is solved on
    its own to the same `_doSafePoW` answer (src/proofofwork.py:100-111), whatever the slots, shards and
    cross-shard bound slots the engine gives them.  Layouts: one shard; three shards of this device (one
    device group: no object on two shards); three shards as separate device groups (every tail window
    split into pieces sharing the cross-shard bound, the multi-device path rehearsed)."""
    shards(layout)
    engine_split(split)
    gpulib.bmpow_set_step_trials(1 << 22)
    rng = random.Random(31 + len(layout) + split)
    ih = rng.randbytes(64)
    dup = (U64 // 60000, rng.randbytes(64))
    objs = [dup] * 6 + [(U64 // d, ih) for d in (1, 2, 50, 3000, 70000, 3000, 1)] + [dup]
    objs += [(U64 // rng.choice([20, 4000, 90000]), rng.randbytes(64)) for _ in range(10)] + [dup] * 3
    rng.shuffle(objs)
    want = [list(r) for r in coracle.search_many(objs)]
    assert proofofwork.run_batch(objs) == want
    # the same entries through the library's service, submitted by two producers at once
    from pybitmessage_amd import worker
    svc = worker.PowService().start()
    try:
        half = len(objs) // 2
        futs = []
        th = [threading.Thread(target=lambda part: futs.extend(svc.submit_many(part)), args=(p,))
              for p in (objs[:half], objs[half:])]
        for x in th:
            x.start()
        for x in th:
            x.join(60)
        got = sorted([list(f.result(timeout=120)) for f in futs])
    finally:
        svc.stop(30)
    assert got == sorted(want)


@pytest.mark.parametrize('layout,step', [([0], 1 << 28), ([0], 8192 * 3), ([0, 0], 1 << 20),
                                         ([0, 0, 0], 8192 * 5), ([0, 0], 3001), ([0], (1 << 26) + 777)])
def test_shard_layouts_and_step_sizes(gpulib, shards, coracle, golden, layout, step):
    """Several shards on one GPU exercise the multi-device nonce-sharding path (each shard
    is its own stream + object table); tiny steps force windows to split across shards and
    objects to span many launches."""
    shards(layout)
    gpulib.bmpow_set_step_trials(step)
    rng = random.Random(len(layout) * 7 + step)
    objs = [(U64 // rng.choice([3, 900, 40000]), rng.randbytes(64)) for _ in range(40)]
    want = [list(r) for r in coracle.search_many(objs)]
    assert proofofwork.run_batch(objs) == want
    for k in golden('first_nonce_kats.json')['kats'][:10]:
        assert gpu_search(gpulib, bytes.fromhex(k['ih']), k['target']) == (k['trial'], k['nonce'])


@pytest.mark.parametrize('layout,step', [([0], 1 << 28), ([0, 0], 1 << 24)])
def test_many_objects_per_step(gpulib, shards, coracle, layout, step):
    """Thousands of objects in one step (more work items per shard than the scheduler's initial
    staging holds, so it grows mid-step; round 1 lost the items already written there)."""
    shards(layout)
    gpulib.bmpow_set_step_trials(step)
    rng = random.Random(4242 + len(layout))
    objs = [(U64 // rng.choice([2, 40, 300, 9000]), rng.randbytes(64)) for _ in range(6000)]
    want = [list(r) for r in coracle.search_many(objs)]
    assert proofofwork.run_batch(objs) == want


def test_edge_targets(gpulib, coracle):
    ih = hashlib.sha512(b'hello').digest()
    t1 = coracle.trial(1, ih)
    assert gpu_search(gpulib, ih, U64) == (coracle.trial(1, ih), 1)
    assert gpu_search(gpulib, ih, t1) == (t1, 1)
    assert gpu_search(gpulib, ih, t1 - 1) == coracle.search(ih, t1 - 1)
    assert proofofwork.run(2 ** 64, ih) == [t1, 1]          # target above 2^64-1 accepts all
    assert proofofwork.run(float(2 ** 63), ih)[1] >= 1      # float targets are int()-ed
    # an initialHash is hashed as given (src/proofofwork.py:104-107): b'' is the nonce alone, not
    # the 64 zero bytes of _doCPoW's buffer (test_gpu_len.py covers every length edge)
    assert proofofwork.run(t1, b'') == list(coracle.search_len(b'', t1))
    assert proofofwork.run(t1, b'') != list(coracle.search(bytes(64), t1))


def test_budget_and_resume(gpulib):
    ih = hashlib.sha512(b'hello').digest()
    assert gpu_search(gpulib, ih, U64 // 1000, 1, 1314) is None
    assert gpu_search(gpulib, ih, U64 // 1000, 1, 1315) == (2417842470843601, 1315)
    assert gpu_search(gpulib, ih, U64 // 1000, 1315, 1) == (2417842470843601, 1315)
    assert gpu_search(gpulib, ih, U64 // 1000, 1, 0) is None


def test_top_of_nonce_space(gpulib, coracle):
    """Windows clipped at 2^64-1: a hit among the last nonces, and exhaustion."""
    ih = hashlib.sha512(b'edge').digest()
    start = U64 - 20000
    tv = coracle.trials(ih, np.uint64(start) + np.arange(20000, dtype=np.uint64))
    tv = np.append(tv, coracle.trial(U64, ih))
    m = int(tv.min())
    want = (m, start + int(np.argmin(tv)))
    assert gpu_search(gpulib, ih, m, start, 1 << 30) == want
    assert gpu_search(gpulib, ih, 0, start, 1 << 30) is None
    assert gpu_search(gpulib, ih, 0, U64, 5) is None
    # batch API reports exhaustion
    h = gpulib.bmpow_batch_create(1, ih, _lib.u64_array([0]), _lib.u64_array([U64 - 100]))
    assert h
    try:
        assert gpulib.bmpow_batch_step(h, 0) == 0
        done = (ctypes.c_uint8 * 1)()
        gpulib.bmpow_batch_results(h, None, None, done, None)
        assert done[0] == _lib.DONE_EXHAUSTED
    finally:
        gpulib.bmpow_batch_destroy(h)


def test_hit_at_nonce_2_64_minus_1(gpulib, coracle):
    """Nonce 2^64-1 is a legal answer (the device's 'no hit yet' is a separate flag, not a
    sentinel nonce): found by bmpow_search, the batch session and bmpow_search_batch."""
    ih = hashlib.sha512(b'top').digest()
    t_top = coracle.trial(U64, ih)
    assert gpu_search(gpulib, ih, U64, U64, 1) == (t_top, U64)
    assert gpu_search(gpulib, ih, t_top, U64, 1) == (t_top, U64)
    assert gpu_search(gpulib, ih, t_top - 1, U64, 1) is None if t_top else True
    # a window ending at 2^64-1 whose only hit is the last nonce: target = trial(2^64-1) when
    # every earlier nonce of the window is above it
    start = U64 - 4000
    m, _ = coracle.min_trial(ih, start, 4000)  # [start, 2^64-1)
    if m > t_top:
        assert gpu_search(gpulib, ih, t_top, start, 1 << 20) == (t_top, U64)
    # batch session starting at the top, and the stateless batch call
    h = gpulib.bmpow_batch_create(2, ih + ih, _lib.u64_array([U64, 0]), _lib.u64_array([U64, U64]))
    assert h
    try:
        assert gpulib.bmpow_batch_step(h, 0) == 0
        nonce, trial = (ctypes.c_uint64 * 2)(), (ctypes.c_uint64 * 2)()
        done, nxt = (ctypes.c_uint8 * 2)(), (ctypes.c_uint64 * 2)()
        gpulib.bmpow_batch_results(h, nonce, trial, done, nxt)
        assert (done[0], nonce[0], trial[0], nxt[0]) == (_lib.DONE_FOUND, U64, t_top, U64)
        assert done[1] == (_lib.DONE_FOUND if t_top == 0 else _lib.DONE_EXHAUSTED)
    finally:
        gpulib.bmpow_batch_destroy(h)
    nxt = _lib.u64_array([U64])
    nonce, trial, done = (ctypes.c_uint64 * 1)(), (ctypes.c_uint64 * 1)(), (ctypes.c_uint8 * 1)()
    assert gpulib.bmpow_search_batch(1, ih, _lib.u64_array([U64]), nxt, 0, nonce, trial, done) == 0
    assert (done[0], nonce[0], trial[0]) == (_lib.DONE_FOUND, U64, t_top)
    assert proofofwork.run_batch([(U64, ih)]) == [[coracle.trial(1, ih), 1]]


def gpu_min_trial(lib, ihs, starts, counts):
    n = len(starts)
    mn, arg = np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint64)
    st, ct = np.array(starts, dtype=np.uint64), np.array(counts, dtype=np.uint64)
    _lib.check(lib, lib.bmpow_min_trial_batch(n, b''.join(ihs), st.ctypes.data_as(P64), ct.ctypes.data_as(P64),
                                              mn.ctypes.data_as(P64), arg.ctypes.data_as(P64)),
               'bmpow_min_trial_batch')
    return [(int(a), int(b)) for a, b in zip(mn, arg)]


@pytest.mark.parametrize('layout,step', [([0], 1 << 28), ([0, 0, 0], 8192 * 3), ([0, 0], 5000)])
def test_min_trial_probe_vs_c_oracle(gpulib, shards, coracle, layout, step):
    """The min-trial probe is bit-exact against the C oracle on ranges the oracle finishes in
    seconds: ragged sizes, empty ranges, ranges ending at 2^64-1, several shards and tiny steps."""
    shards(layout)
    gpulib.bmpow_set_step_trials(step)
    rng = random.Random(len(layout) * 31 + step)
    ihs, starts, counts = [], [], []
    for k in range(40):
        ihs.append(rng.randbytes(64))
        if k % 10 == 0:
            starts.append(U64 - rng.randrange(0, 3000))
            counts.append(rng.randrange(0, 5000))   # clipped at 2^64-1
        else:
            starts.append(rng.choice([0, 1, rng.randrange(1 << 40)]))
            counts.append(rng.choice([0, 1, 255, 256, 257, 8191, 8192, 8193, rng.randrange(1, 60000)]))
    want = [coracle.min_trial(ih, s, c) for ih, s, c in zip(ihs, starts, counts)]
    assert gpu_min_trial(gpulib, ihs, starts, counts) == want
    m, a = ctypes.c_uint64(), ctypes.c_uint64()
    assert gpulib.bmpow_min_trial(ihs[1], starts[1], counts[1], ctypes.byref(m), ctypes.byref(a)) == 0
    assert (m.value, a.value) == want[1]


def test_min_trial_large_range(gpulib, coracle):
    """Two million nonces (hundreds of workgroups, several steps at 2^20 trials) against the
    oracle's sequential minimum."""
    gpulib.bmpow_set_step_trials(1 << 20)
    try:
        ih = hashlib.sha512(b'min-trial').digest()
        assert gpu_min_trial(gpulib, [ih], [12345], [2000000]) == [coracle.min_trial(ih, 12345, 2000000)]
    finally:
        gpulib.bmpow_set_step_trials(0)  # the library's default


def test_search_batch_stateless_resume(gpulib, coracle):
    rng = random.Random(3)
    n = 50
    ihs = [rng.randbytes(64) for _ in range(n)]
    tg = [U64 // rng.choice([10, 5000, 100000]) for _ in range(n)]
    nxt = _lib.u64_array([1] * n)
    nonce, trial = (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)()
    done = (ctypes.c_uint8 * n)()
    calls = 0
    while True:
        calls += 1
        p = _lib.check(gpulib, gpulib.bmpow_search_batch(n, b''.join(ihs), _lib.u64_array(tg), nxt, 1 << 16,
                                                         nonce, trial, done), 'search_batch')
        if p == 0:
            break
    assert calls > 2
    for i in range(n):
        assert done[i] == _lib.DONE_FOUND
        assert (trial[i], nonce[i]) == coracle.search(ihs[i], tg[i])


def test_minimality_property_large_objects(gpulib):
    """Default-difficulty objects (C2-sized, ~1e7-1e8 trials each) are too slow for the CPU
    oracle; check size-independent properties instead: trial(nonce) <= target (hashlib), and
    every nonce in [1, nonce) misses -- re-hashed with bmpow_trials, whose bit-exactness
    against the oracle is pinned by the tests above."""
    rng = random.Random(20250216)
    objs = []
    for _ in range(6):
        L = rng.randrange(512, 16385)
        payload = rng.randbytes(L)
        t = int(2 ** 64 / (1000 * (L + 8 + 1000 + ((345600 * (L + 8 + 1000)) / (2 ** 16)))))
        objs.append((t, hashlib.sha512(payload).digest()))
    res = proofofwork.run_batch(objs)
    for (t, ih), (tv, nonce) in zip(objs, res):
        assert tv <= t
        lo = 1
        while lo < nonce:
            hi = min(nonce, lo + (1 << 26))
            tr = gpu_trials(gpulib, ih, np.arange(lo, hi, dtype=np.uint64))
            assert int(tr.min()) > t
            lo = hi


def test_abort_from_another_thread(gpulib):
    timer = threading.Timer(0.3, gpulib.bmpow_abort)
    timer.start()
    t0 = time.time()
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    rc = gpulib.bmpow_search(bytes(64), 0, 1, 1 << 42, ctypes.byref(n), ctypes.byref(t))
    gpulib.bmpow_clear_abort()
    assert rc == _lib.E_ABORTED
    # bound: the abort is seen at the next window boundary (one 2^29-trial window, ~80 ms, with one more
    # queued behind it) after the 0.3 s timer: under 0.5 s; 5 s leaves 10x
    assert time.time() - t0 < 5


def test_state_shutdown_interrupts_run(gpulib, monkeypatch):
    monkeypatch.setattr(proofofwork, 'CALL_TRIALS', 1 << 28)
    timer = threading.Timer(0.3, lambda: setattr(state, 'shutdown', 1))
    timer.start()
    try:
        with pytest.raises(StopIteration, match='Interrupted'):
            proofofwork.run(0, bytes(64))
    finally:
        state.shutdown = 0


def test_bitmessagepow_compat_shim(gpulib):
    ih = hashlib.sha512(b'hello').digest()
    assert gpulib.BitmessagePOW(ih, U64 // 1000) == 1315


def test_stats_count_trials(gpulib):
    gpulib.bmpow_reset_stats()
    ih = hashlib.sha512(b'hello').digest()
    assert gpu_search(gpulib, ih, 184467440737095) == (141019321561983, 129430)
    st = _lib.BmpowStats()
    gpulib.bmpow_get_stats(ctypes.byref(st))
    assert st.launches >= 1 and st.trials >= 129430 and st.kernel_ms > 0


def test_concurrent_callers_are_serialised_and_exact(gpulib, coracle):
    """The reference calls run() from the worker thread and the API thread at once
    (class_singleWorker.py:236, api.py:1304); every entry point is thread safe and exact."""
    from concurrent.futures import ThreadPoolExecutor
    rng = random.Random(77)
    jobs = [(U64 // rng.choice([50, 3000, 70000]), rng.randbytes(64)) for _ in range(24)]
    with ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda j: proofofwork.run(*j), jobs))
        batches = list(ex.map(proofofwork.run_batch, [jobs[i::3] for i in range(3)]))
    assert got == [list(r) for r in coracle.search_many(jobs)]
    for i in range(3):
        assert batches[i] == got[i::3]


def test_batch_park_and_schedule(gpulib, coracle):
    """bmpow_batch_set_pending: parked objects are skipped, scheduled ones solve exactly, in
    any order of scheduling (bench.py's cross-rank claiming)."""
    rng = random.Random(5)
    n = 12
    objs = [(U64 // rng.choice([100, 5000]), rng.randbytes(64)) for _ in range(n)]
    tg = np.array([t for t, _ in objs], dtype=np.uint64)
    h = gpulib.bmpow_batch_create(n, b''.join(ih for _, ih in objs), tg.ctypes.data_as(P64), None)
    assert h
    try:
        assert gpulib.bmpow_batch_set_pending(h, 0, n, 0) == 0
        assert gpulib.bmpow_batch_step(h, 0) == 0  # nothing scheduled: nothing to do
        done = np.zeros(n, dtype=np.uint8)
        nonce = np.zeros(n, dtype=np.uint64)
        trial = np.zeros(n, dtype=np.uint64)
        for lo, hi in [(8, 12), (0, 3), (3, 8)]:  # out of order
            gpulib.bmpow_batch_set_pending(h, lo, hi - lo, 1)
            while gpulib.bmpow_batch_step(h, 0) > 0:
                pass
            gpulib.bmpow_batch_results(h, nonce.ctypes.data_as(P64), trial.ctypes.data_as(P64),
                                       done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), None)
            assert (done[lo:hi] == _lib.DONE_FOUND).all()
        for i, (t, ih) in enumerate(objs):
            assert (int(trial[i]), int(nonce[i])) == coracle.search(ih, t)
        assert gpulib.bmpow_batch_set_pending(h, n, 1, 1) < 0  # range outside the batch
    finally:
        gpulib.bmpow_batch_destroy(h)


def test_session_add_and_take_done(gpulib, coracle):
    """The resident session PowService runs on: objects appended between steps
    (bmpow_batch_add) join the next step, finished ones are popped in finishing order
    (bmpow_batch_take_done) and their slots are reused by later adds; every answer exact."""
    rng = random.Random(8)
    h = gpulib.bmpow_batch_create(0, None, None, None)
    assert h
    pu32 = ctypes.POINTER(ctypes.c_uint32)
    cap = 256
    slot_b, nonce_b = np.zeros(cap, dtype=np.uint32), np.zeros(cap, dtype=np.uint64)
    trial_b, done_b = np.zeros(cap, dtype=np.uint64), np.zeros(cap, dtype=np.uint8)
    live, got, max_slot = {}, {}, -1
    try:
        serial = 0
        for rnd in range(12):
            objs = [(U64 // rng.choice([3, 500, 20000, 300000]), rng.randbytes(64)) for _ in range(rng.randrange(1, 400))]
            tg = np.array([t for t, _ in objs], dtype=np.uint64)
            slots = np.zeros(len(objs), dtype=np.uint32)
            assert gpulib.bmpow_batch_add(h, len(objs), b''.join(ih for _, ih in objs), tg.ctypes.data_as(P64), None,
                                          slots.ctypes.data_as(pu32)) >= len(objs)
            assert len(set(slots.tolist()) | set(live)) == len(live) + len(objs)  # no live slot handed out twice
            if rnd >= 4:
                assert slots.min() <= max_slot  # released slots are reused
            for o, sl in zip(objs, slots.tolist()):
                live[sl] = (serial, o)
                serial += 1
                max_slot = max(max_slot, sl)
            gpulib.bmpow_set_step_trials(1 << 22)
            assert gpulib.bmpow_batch_step(h, 0) >= 0
            while True:
                k = gpulib.bmpow_batch_take_done(h, cap, slot_b.ctypes.data_as(pu32), nonce_b.ctypes.data_as(P64),
                                                 trial_b.ctypes.data_as(P64),
                                                 done_b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
                for j in range(k):
                    sid, o = live.pop(int(slot_b[j]))
                    assert done_b[j] == _lib.DONE_FOUND
                    got[sid] = (o, (int(trial_b[j]), int(nonce_b[j])))
                if k < cap:
                    break
        while live:
            gpulib.bmpow_batch_step(h, 0)
            k = gpulib.bmpow_batch_take_done(h, cap, slot_b.ctypes.data_as(pu32), nonce_b.ctypes.data_as(P64),
                                             trial_b.ctypes.data_as(P64),
                                             done_b.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
            for j in range(k):
                sid, o = live.pop(int(slot_b[j]))
                got[sid] = (o, (int(trial_b[j]), int(nonce_b[j])))
    finally:
        gpulib.bmpow_batch_destroy(h)
        gpulib.bmpow_set_step_trials(0)  # the library's default
    assert len(got) == serial
    objs = [o for o, _ in got.values()]
    assert [res for _, res in got.values()] == coracle.search_many(objs)


def test_native_service_producers_cancel_abort(gpulib, coracle):
    """bmpow_service_*: the library's stepping thread.  Four producers submit concurrently while
    one consumer polls; tickets are unique and every answer exact.  A cancel drops everything in
    flight and the service keeps going; an abort surfaces as the poll's error, and a cancel
    recovers from it."""
    gpulib.bmpow_set_step_trials(1 << 22)
    s = gpulib.bmpow_service_create(0, _lib.SERVICE_VERIFY)
    assert s
    cap = 512
    tk, nn = np.zeros(cap, dtype=np.uint64), np.zeros(cap, dtype=np.uint64)
    tv, dn = np.zeros(cap, dtype=np.uint64), np.zeros(cap, dtype=np.uint8)
    pu8 = ctypes.POINTER(ctypes.c_uint8)

    def poll(timeout_ms=2000):
        k = gpulib.bmpow_service_poll(s, cap, timeout_ms, tk.ctypes.data_as(P64), nn.ctypes.data_as(P64),
                                      tv.ctypes.data_as(P64), dn.ctypes.data_as(pu8))
        if k < 0:
            return k
        return [(int(tk[j]), int(tv[j]), int(nn[j]), int(dn[j])) for j in range(k)]

    def submit(objs):
        tg = np.array([t for t, _ in objs], dtype=np.uint64)
        out = np.zeros(len(objs), dtype=np.uint64)
        assert gpulib.bmpow_service_submit(s, len(objs), b''.join(ih for _, ih in objs), tg.ctypes.data_as(P64),
                                           out.ctypes.data_as(P64)) == 0
        return out.tolist()
    try:
        jobs, lock = {}, threading.Lock()

        def producer(seed):
            rng = random.Random(seed)
            for _ in range(10):
                objs = [(U64 // rng.choice([3, 500, 20000, 300000]), rng.randbytes(64))
                        for _ in range(rng.randrange(1, 60))]
                with lock:  # the ticket map must hold a ticket before a poll can return it
                    for t, o in zip(submit(objs), objs):
                        assert t not in jobs
                        jobs[t] = o
                time.sleep(rng.random() * 0.02)
        ths = [threading.Thread(target=producer, args=(k,)) for k in range(4)]
        for t in ths:
            t.start()
        got = {}
        deadline = time.time() + 120
        while (any(t.is_alive() for t in ths) or len(got) < len(jobs)) and time.time() < deadline:
            r = poll(200)
            assert not isinstance(r, int), r
            for t, trial, nonce, d in r:
                assert d == _lib.DONE_FOUND and t not in got
                got[t] = (trial, nonce)
        for t in ths:
            t.join()
        assert len(got) == len(jobs) and gpulib.bmpow_service_outstanding(s) == 0
        want = coracle.search_many(list(jobs.values()))
        for t, w in zip(jobs, want):
            assert got[t] == w
        # cancel drops in-flight work (a target-0 object never finishes) and the service goes on
        submit([(0, bytes(64))] * 3)
        time.sleep(0.2)
        assert gpulib.bmpow_service_cancel(s) == 0 and gpulib.bmpow_service_outstanding(s) == 0
        ih = hashlib.sha512(b'after-cancel').digest()
        (t1,) = submit([(U64 // 1000, ih)])
        r = poll(10000)
        assert [(t, tr, n) for t, tr, n, _ in r] == [(t1,) + coracle.search(ih, U64 // 1000)]
        # abort: the step fails, the poll reports it, a cancel clears it
        submit([(0, bytes(64))])
        time.sleep(0.1)
        gpulib.bmpow_abort()
        assert poll(10000) == _lib.E_ABORTED
        gpulib.bmpow_clear_abort()
        gpulib.bmpow_service_cancel(s)
        (t2,) = submit([(U64 // 1000, ih)])
        r = poll(10000)
        assert [(t, tr, n) for t, tr, n, _ in r] == [(t2,) + coracle.search(ih, U64 // 1000)]
    finally:
        gpulib.bmpow_clear_abort()
        gpulib.bmpow_service_destroy(s)
        gpulib.bmpow_set_step_trials(0)  # the library's default
