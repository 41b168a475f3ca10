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
import random

import numpy as np
import pytest

import bench
from pybitmessage_amd import _lib, proofofwork

pytestmark = pytest.mark.gpu
U64 = (1 << 64) - 1
P64 = ctypes.POINTER(ctypes.c_uint64)


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


def test_c2_full_batch(gpulib):
    """C2: 1,024 pending msg objects, L ~ U[512, 16384], default difficulty, TTL 4 d (~6e10
    trials to solve and as many to prove)."""
    objs, _ = bench.make_objects('c2', 0)
    assert len(objs) == 1024
    res = proofofwork.run_batch(objs)
    hashed = assert_exact_first_nonces(gpulib, objs, res)
    assert hashed > 4e10


def test_c4_nonce_sharded_eight_ways(gpulib, shards):
    """C4: 64 objects at 20x nonceTrialsPerByte, TTL 28 d (~1.5e9 trials each), nonce-sharded
    over 8 shards with early exit (8 streams on this device; the same slicing as 8 GPUs)."""
    shards([0] * 8)
    objs, _ = bench.make_objects('c4', 0)
    assert len(objs) == 64 and all(t == 11971972251 for t, _ in objs)
    gpulib.bmpow_reset_stats()
    res = proofofwork.run_batch(objs)
    st = _lib.BmpowStats()
    gpulib.bmpow_get_stats(ctypes.byref(st))
    useful = sum(nonce for _, nonce in res)
    assert st.trials >= useful and (st.trials - useful) / st.trials < 0.05  # trials past the answers
    assert_exact_first_nonces(gpulib, objs, res)


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


@pytest.mark.slow
def test_c3_sweep_2_38_no_hit(gpulib):
    """C3: fixed initialHash, target 0, 2^38 nonces: no hit, and the device hashes exactly 2^38
    trials (no window lost or repeated across 1,024 steps)."""
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
