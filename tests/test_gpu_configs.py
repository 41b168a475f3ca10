"""Every BASELINE.json config at its full size on the GPU, proven exact by size-independent
properties (the CPU oracle is far too slow at these sizes):

* each answer n satisfies trial(n) <= target, re-hashed with hashlib (``proofofwork._verify``);
* no earlier nonce does: the min-trial probe (``bmpow_min_trial_batch``, a code path apart from
  the search's hit logic, itself pinned to the C oracle in test_gpu_parity.py) over [1, n) is
  above the target -- together, n is the reference's ``_doSafePoW`` answer
  (src/proofofwork.py:100-111);
* a sample of the objects is also solved by the C oracle.

C1 (the golden nonce 10,909,138) is in test_gpu_parity.py::test_first_nonce_kats.  Workloads are
bench.py's own (``bench.make_objects``, rank 0), targets from class_singleWorker.py:222-230.
"""
import ctypes
import hashlib
import os
import random

import numpy as np
import pytest


import bench
from pybitmessage_amd import _lib, proofofwork

pytestmark = pytest.mark.gpu
U64 = (1 << 64) - 1
P64 = ctypes.POINTER(ctypes.c_uint64)
# the C oracle's exact multi-threaded search on the host's CPUs (the GPU box's quota is 16)
CPU_THREADS = max(1, min(16, os.cpu_count() or 1))


def oracle_sample(coracle, objs, res, idx):
    """objects idx solved again by the C oracle (bmo_search_mt: every nonce from 1, exact first
    hit), a restatement that shares no code with the device: the same [trialValue, nonce]."""
    for i in idx:
        t, ih = objs[i]
        got, _ = coracle.search_mt(ih, int(t), 1, res[i][1] + (1 << 20), threads=CPU_THREADS)
        assert got == tuple(res[i]), (i, got, res[i])


def assert_exact_first_nonces(lib, objs, res):
    """res[i] = [trialValue, nonce] is the first nonce >= 1 with trialValue <= target."""
    n = len(objs)
    ihs = b''.join(ih for _, ih in objs)
    starts = np.ones(n, dtype=np.uint64)
    counts = np.array([nonce - 1 for _, nonce in res], dtype=np.uint64)
    mn, arg = np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint64)
    _lib.check(lib, lib.bmpow_min_trial_batch(n, ihs, starts.ctypes.data_as(P64), counts.ctypes.data_as(P64),
                                              mn.ctypes.data_as(P64), arg.ctypes.data_as(P64)),
               'bmpow_min_trial_batch')
    tg = np.array([t for t, _ in objs], dtype=np.uint64)
    for i, ((t, ih), (tv, nonce)) in enumerate(zip(objs, res)):
        assert nonce >= 1
        proofofwork._verify(t, ih, tv, nonce)            # hashlib: trial(nonce) == tv <= target
    early = np.flatnonzero((counts > 0) & (mn <= tg))
    assert early.size == 0, 'objects with an earlier hit: %s' % early[:10].tolist()
    return int(counts.sum()) + n


def test_c2_full_batch(gpulib, coracle):
    """C2: 1,024 pending msg objects, L ~ U[512, 16384], default difficulty, TTL 4 d (~6e10
    trials to solve and as many to prove); 8 of them (seeded draw) also solved by the C oracle."""
    objs, _ = bench.make_objects('c2', 0)
    assert len(objs) == 1024
    res = proofofwork.run_batch(objs)
    hashed = assert_exact_first_nonces(gpulib, objs, res)
    assert hashed > 4e10
    oracle_sample(coracle, objs, res, random.Random(2).sample(range(len(objs)), 8))


# bm_search_kernel workgroups resident on one MI355X (4 per CU at <= 128 VGPRs x 256 CUs): a window's
# blocks in flight at once (bmpow_layout.h), one block row = ROW nonces
ROW = 1024 * 256
# Rows a sweep runs past its answer before every workgroup has read the bound (bmpow_kernels.hip sweep:
# each workgroup reads it once per block, so the blocks taken above the answer are those handed out
# while the answer's block was hashed -- as many rows as the slowest resident wave's block time over the
# fastest's, since the SIMD arbiter favours older waves).  Measured over 300 single-object C1 calls:
# median 0.14 rows, slowest 1.1 (profiles/r05/final/c1_dist_default.json; round 4's the same); the
# bound allows 48, for an answer's workgroup starved behind other shards' kernels on a shared device.
ROWS_PAST = 48


def test_c4_nonce_sharded_eight_ways(gpulib, shards, coracle):
    """C4: 64 objects at 20x nonceTrialsPerByte, TTL 28 d (~1.5e9 trials each), over 8 shards of this
    device with early exit; the object with the smallest answer (~E/64 trials for the CPU) also solved
    by the C oracle.

    The 8 shards share one device, so they form ONE device group of the engine (round 6,
    bmsched::PlanCtx::group): no window is split among them and no object is on two of them at once, so
    an object's windows run in order on one stream.  Trials past the answers, from that design:
      * windows of an object above its answer's: none hashed -- they run after the answer's launch on
        the same stream, whose hit is in best[] before their first block (bmpow_kernels.hip sweep reads
        it before the first block): past_later == 0 exactly;
      * split pieces: none (past_split == 0);
      * the window holding the answer: the rows handed out while the bound reached every workgroup,
        at most ROWS_PAST rows per object.
    (Round 5 split the tail objects into 8 pieces racing on the device's SIMDs: 2.0-5.0 % past the
    answers, GPUTEST_r05.)"""
    shards([0] * 8)
    objs, _ = bench.make_objects('c4', 0)
    assert len(objs) == 64 and all(t == 11971972251 for t, _ in objs)
    gpulib.bmpow_reset_stats()
    res = proofofwork.run_batch(objs)
    st = _lib.BmpowStats()
    gpulib.bmpow_get_stats(ctypes.byref(st))
    useful = sum(nonce for _, nonce in res)
    assert st.trials >= useful
    assert st.past_split == 0 and st.past_later == 0, (st.past_split, st.past_later)
    assert st.trials - useful <= len(objs) * ROWS_PAST * ROW, (st.trials - useful, st.past_window)
    # every shard measured its rate (the weights of the steps' slices after the first)
    rates = (ctypes.c_double * 8)()
    assert gpulib.bmpow_get_shard_rates(rates, 8) == 8
    assert all(r > 0 for r in rates), list(rates)
    assert_exact_first_nonces(gpulib, objs, res)
    oracle_sample(coracle, objs, res, [min(range(len(res)), key=lambda i: res[i][1])])


def test_c5_flood_test_mode(gpulib, coracle):
    """C5: 100,000 ack/pubkey objects at the reference's test-mode difficulty (ntpb and extra
    / 100, bitmessagemain.py:167-172): one batch of 100k objects, so a step packs one chunk per
    object for the first 32,768 pending objects; a 500-object sample also vs the C oracle."""
    objs, _ = bench.make_objects('c5', 0, test_mode=True)
    assert len(objs) == 100000
    res = proofofwork.run_batch(objs)
    assert_exact_first_nonces(gpulib, objs, res)
    for i in random.Random(5).sample(range(len(objs)), 500):
        t, ih = objs[i]
        assert tuple(res[i]) == coracle.search(ih, t), i


def test_c5_default_difficulty_slice(gpulib, shards, coracle):
    """C5 at protocol-default difficulty (the flood's own targets, class_singleWorker.py:222-230:
    acks L = 46, TTL 28 d, E ~ 4.0e7; pubkeys L = 200, TTL 4 d, E ~ 7.6e6): a 10,000-object slice of
    bench.make_objects('c5', 0) with steps of 2^26 trials, so a step's 8,192 chunks are fewer than
    the pending objects -- the 100k flood's regime, where each object spans thousands of chunks
    over many steps (round 1's lost-work-item bug lived there).  Every answer proven minimal by the
    min-trial probe; 8 of them (seeded draw) also solved by the C oracle."""
    shards([0])
    gpulib.bmpow_set_step_trials(1 << 26)
    objs, _ = bench.make_objects('c5', 0)
    objs = objs[:10000]
    kinds = {t for t, _ in objs}
    assert len(kinds) == 2 and min(kinds) > 4e11  # default difficulty, both object kinds
    res = proofofwork.run_batch(objs)
    gpulib.bmpow_set_step_trials(0)  # the library's default
    hashed = assert_exact_first_nonces(gpulib, objs, res)
    assert hashed > 1e11
    rng = random.Random(55)
    oracle_sample(coracle, objs, res, rng.sample(range(len(objs)), 8))


@pytest.mark.parametrize('nshards,split', [(1, False), (8, False), (4, True), (8, True)])
def test_c1_sweep_stops_within_rows_of_the_hit(gpulib, shards, golden, nshards, split):
    """One C1 object (1 KB msg at defaults, golden nonce 10,909,138) through run() on one shard, on 8
    shards of this device, and split into 4 and 8 forced pieces (bmpow_set_run_split).

    One piece: the workgroups take the window's blocks in order from its queue, so the trials hashed
    past the answer stay within a few block rows (the static column layout of early round 3 hashed
    29 M on one shard for the 10.9 M useful, profiles/r03/c1_columns_static.jsonl: the SIMD arbiter
    favours older waves, so the columns drifted apart).  Shards sharing a device do not split run()
    (round 5), so 8 shards of this device behave as one.

    Forced pieces on ONE device: each piece sweeps its interleaved columns of the same rows on its own
    slice of the CUs (a CU-masked stream, as a separate smaller GPU) and stops at the first hit of any
    through the cross-device bound.  Bound: one window's pieces run through at most their rows up to the
    answer's, plus the pieces of the next window stopping at their first blocks (2E + rows also holds
    with BMPOW_SPLIT_CUMASK=0, where the pieces share the whole device and a window is 2E)."""
    shards([0] * nshards)
    prev = gpulib.bmpow_set_run_split(1 if split else 0)
    k = [k for k in golden('first_nonce_kats.json')['kats'] if k['nonce'] == 10909138][0]
    ih = bytes.fromhex(k['ih'])
    e = 2 ** 64 / (k['target'] + 1)
    past = []
    try:
        for _ in range(5):
            gpulib.bmpow_reset_stats()
            assert proofofwork.run(k['target'], ih) == [k['trial'], k['nonce']]
            st = _lib.BmpowStats()
            gpulib.bmpow_get_stats(ctypes.byref(st))
            assert st.trials >= k['nonce'] - 1
            past.append(st.trials - k['nonce'])
            if split:
                # one window of 2E in nshards pieces; the pieces of the next window queued behind stop
                # at their first blocks (the relay folds the hit into every piece's minimum)
                assert st.trials <= 2 * e + 2 * nshards * ROW, (st.trials, st.launches)
    finally:
        gpulib.bmpow_set_run_split(prev)
    if not split:
        # one piece: the rows handed out while the bound reached every workgroup (ROWS_PAST)
        assert max(past) <= ROWS_PAST * ROW, past


@pytest.mark.slow
def test_c3_sweep_2_38_no_hit(gpulib):
    """C3: fixed initialHash, target 0, 2^38 nonces: no hit, and the device hashes exactly 2^38
    trials (no window lost or repeated across the 512 steps of 2^29)."""
    ih = hashlib.sha512(b'bmpow-sweep').digest()
    gpulib.bmpow_reset_stats()
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    rc = _lib.check(gpulib, gpulib.bmpow_search(ih, 0, 1, 1 << 38, ctypes.byref(n), ctypes.byref(t)), 'search')
    assert rc == _lib.NOT_FOUND
    st = _lib.BmpowStats()
    gpulib.bmpow_get_stats(ctypes.byref(st))
    assert st.trials == 1 << 38


def test_nonce_sharding_over_every_device(gpulib, shards, coracle, golden):
    """One object's nonce space split over every visible MI355X (in-process, one stream and
    object table per device): answers equal the single-device ones and the golden KATs."""
    ndev = gpulib.bmpow_device_count()
    if ndev < 2:
        pytest.skip('needs >= 2 visible gfx950 devices (this box has %d)' % ndev)
    shards(list(range(ndev)))
    for k in golden('first_nonce_kats.json')['kats'][:20]:
        assert proofofwork.run(k['target'], bytes.fromhex(k['ih'])) == [k['trial'], k['nonce']]
    objs, _ = bench.make_objects('c4', 0, 2)
    res = proofofwork.run_batch(objs)
    assert_exact_first_nonces(gpulib, objs, res)


def test_device_count_selector(gpulib, shards, golden):
    """SURVEY 8(b)'s `int bmpow_set_devices(int ndev)` form (bmpow_set_device_count): the first ndev
    visible devices, rejected below 1 or above the visible count, and the search exact after it."""
    ndev = gpulib.bmpow_device_count()
    assert ndev >= 1
    assert gpulib.bmpow_set_device_count(1) == 1
    ids = (ctypes.c_int * 64)()
    assert gpulib.bmpow_get_devices(ids, 64) == 1 and ids[0] == 0
    assert gpulib.bmpow_set_device_count(0) == _lib.E_ARG
    assert gpulib.bmpow_set_device_count(ndev + 1) == _lib.E_ARG
    assert gpulib.bmpow_set_devices(None, ndev) == ndev  # the NULL-list spelling of the same
    assert gpulib.bmpow_get_devices(ids, 64) == ndev and list(ids[:ndev]) == list(range(ndev))
    k = [k for k in golden('first_nonce_kats.json')['kats'] if k['nonce'] == 10909138][0]
    assert proofofwork.run(k['target'], bytes.fromhex(k['ih'])) == [k['trial'], k['nonce']]
