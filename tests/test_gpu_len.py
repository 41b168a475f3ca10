"""initialHash values that are not 64 bytes long, on the GPU (bm_search_var_kernel and friends).

The reference's ``_doSafePoW`` hashes ``pack('>Q', nonce) + initialHash`` as given, at any length
(src/proofofwork.py:100-111).  Every caller passes a 64-byte digest -- the layout the main kernel is
specialised for -- but ``run``, ``run_batch``, ``PowService`` and ``do_opencl_pow`` accept any bytes
and must give the same answers.  Pinned by the reference's own outputs (tests/golden/len_kats.json,
tests/golden/make_len_golden.py) and the C oracle (``bmo_search_len``), at every SHA-512 block edge of
the first hash's message (8 + L bytes + 17 bytes of padding).  Bit-exact.
"""
import ctypes
import random

import numpy as np
import pytest

from pybitmessage_amd import _lib, hippow, proofofwork
from pybitmessage_amd.worker import PowService

pytestmark = pytest.mark.gpu
U64 = (1 << 64) - 1
P64 = ctypes.POINTER(ctypes.c_uint64)


def gpu_trials_len(lib, ih, nonces):
    nonces = np.ascontiguousarray(nonces, dtype=np.uint64)
    out = np.zeros_like(nonces)
    _lib.check(lib, lib.bmpow_trials_len(ih, len(ih), nonces.ctypes.data_as(P64), nonces.size,
                                         out.ctypes.data_as(P64)), 'bmpow_trials_len')
    return out


def test_len_trial_kats(gpulib, golden):
    by = {}
    for k in golden('len_kats.json')['trial']:
        by.setdefault(k['ih'], []).append(k)
    for ihx, ks in by.items():
        got = gpu_trials_len(gpulib, bytes.fromhex(ihx), [k['nonce'] for k in ks])
        assert [int(x) for x in got] == [k['trial'] for k in ks], len(ihx) // 2


def test_len_trials_random_vs_c_oracle(gpulib, coracle):
    rng = random.Random(12)
    for L in [0, 1, 9, 56, 63, 65, 96, 103, 104, 105, 120, 200, 231, 232, 233, 383, 384, 1024, 5000]:
        ih = rng.randbytes(L)
        nonces = [0, 1, 2, U64, U64 - 1] + [rng.randrange(U64) for _ in range(600)] + list(range(1000, 1300))
        got = gpu_trials_len(gpulib, ih, nonces)
        assert [int(x) for x in got] == [coracle.trial_len(n, ih) for n in nonces], L
    # the 64-byte length through the *_len entry point is the main kernel's
    ih = rng.randbytes(64)
    assert [int(x) for x in gpu_trials_len(gpulib, ih, [1, 2, 3])] == [coracle.trial(n, ih) for n in (1, 2, 3)]


def test_len_first_nonce_kats_run(gpulib, golden):
    for k in golden('len_kats.json')['first']:
        assert proofofwork.run(k['target'], bytes.fromhex(k['ih'])) == [k['trial'], k['nonce']], k['len']


def test_len_kats_run_batch_mixed_with_64(gpulib, golden):
    """One batch mixing every length KAT with 64-byte objects: the step splits each shard's items
    over the two kernels (bmsched::split_kinds)."""
    d = golden('len_kats.json')['first']
    b = golden('batch_kats.json')['kats']
    objs, want = [], []
    for i, k in enumerate(d):
        objs.append((k['target'], bytes.fromhex(k['ih'])))
        want.append([k['trial'], k['nonce']])
        kb = b[i % len(b)]
        objs.append((kb['target'], bytes.fromhex(kb['ih'])))
        want.append([kb['trial'], kb['nonce']])
    assert proofofwork.run_batch(objs) == want


def test_len_kats_powservice_and_do_opencl_pow(gpulib, golden):
    d = golden('len_kats.json')['first']
    svc = PowService().start()
    try:
        futs = [svc.submit(k['target'], bytes.fromhex(k['ih'])) for k in d[:6]]
        many = svc.submit_many([(k['target'], bytes.fromhex(k['ih'])) for k in d])
        assert [f.result(60) for f in futs] == [[k['trial'], k['nonce']] for k in d[:6]]
        assert [f.result(60) for f in many] == [[k['trial'], k['nonce']] for k in d]
    finally:
        svc.stop()
    hippow.initCL()
    for k in d[:10]:
        assert hippow.do_opencl_pow(k['ih'], k['target']) == k['nonce']


@pytest.mark.parametrize('layout,step', [([0], 1 << 28), ([0, 0, 0], 8192 * 3), ([0, 0], 1 << 20)])
def test_random_lengths_vs_c_oracle(gpulib, shards, coracle, layout, step):
    """Random lengths 0..1100 and 64, several shard layouts and step sizes (objects spanning many
    launches and split over shards), against the C oracle's sequential search."""
    shards(layout)
    gpulib.bmpow_set_step_trials(step)
    rng = random.Random(31 + len(layout))
    objs = []
    for i in range(60):
        L = 64 if i % 4 == 0 else rng.choice([rng.randrange(0, 130), rng.randrange(130, 1100)])
        objs.append((U64 // rng.choice([1, 5, 700, 20000]), rng.randbytes(L)))
    want = [list(coracle.search_len(ih, t)) for t, ih in objs]
    assert proofofwork.run_batch(objs) == want


def test_len_minimality_probe(gpulib, coracle):
    """bmpow_min_trial_var (the var-form probe) against the C oracle on ragged ranges, and as the
    minimality proof of larger var-form answers (min over [1, n) above the target)."""
    rng = random.Random(8)
    ihs = [rng.randbytes(L) for L in (0, 33, 104, 300, 64, 250)]
    starts = np.array([1, 5, 1 << 40, U64 - 300, 9, 100], dtype=np.uint64)
    counts = np.array([9000, 1, 20000, 400, 0, 8193], dtype=np.uint64)
    off = np.cumsum([0] + [len(x) for x in ihs]).astype(np.uint64)
    n = len(ihs)
    mn, arg = np.zeros(n, dtype=np.uint64), np.zeros(n, dtype=np.uint64)
    _lib.check(gpulib, gpulib.bmpow_min_trial_var(n, b''.join(ihs), off.ctypes.data_as(P64),
                                                  starts.ctypes.data_as(P64), counts.ctypes.data_as(P64),
                                                  mn.ctypes.data_as(P64), arg.ctypes.data_as(P64)),
               'bmpow_min_trial_var')
    for i, ih in enumerate(ihs):
        st, ct = int(starts[i]), int(counts[i])
        ct = min(ct, U64 - st + 1)
        if ct == 0:
            assert (int(mn[i]), int(arg[i])) == (U64, st)
            continue
        tv = [coracle.trial_len(st + j, ih) for j in range(ct)]
        m = min(tv)
        assert (int(mn[i]), int(arg[i])) == (m, st + tv.index(m)), i
    # minimality of harder answers (E ~ 5e6: thousands of chunks each)
    objs = [(U64 // 5_000_000, rng.randbytes(L)) for L in (7, 150, 600)]
    res = proofofwork.run_batch(objs)
    ihs = [ih for _, ih in objs]
    off = np.cumsum([0] + [len(x) for x in ihs]).astype(np.uint64)
    st = np.ones(3, dtype=np.uint64)
    ct = np.array([nn - 1 for _, nn in res], dtype=np.uint64)
    mn, arg = np.zeros(3, dtype=np.uint64), np.zeros(3, dtype=np.uint64)
    _lib.check(gpulib, gpulib.bmpow_min_trial_var(3, b''.join(ihs), off.ctypes.data_as(P64), st.ctypes.data_as(P64),
                                                  ct.ctypes.data_as(P64), mn.ctypes.data_as(P64),
                                                  arg.ctypes.data_as(P64)), 'bmpow_min_trial_var')
    for (t, ih), (tv, nn), m in zip(objs, res, mn):
        assert tv == coracle.trial_len(nn, ih) and tv <= t
        assert int(m) > t


def test_len_bounds(gpulib):
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    big = bytes(_lib.MAX_IH_LEN + 1)
    assert gpulib.bmpow_search_len(big, len(big), U64, 1, 10, ctypes.byref(n), ctypes.byref(t)) == _lib.E_ARG
    with pytest.raises(ValueError):
        proofofwork.run(U64, big)
    # the longest accepted initialHash still answers (one trial: target 2^64 - 1 accepts nonce 1)
    top = bytes(range(256)) * (_lib.MAX_IH_LEN // 256)
    assert proofofwork.run(U64, top)[1] == 1
