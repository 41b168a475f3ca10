"""Receive-side verification: the GPU POW values and verdicts of
``bmpow_pow_values`` / ``bmpow_verify_batch`` against fixtures judged by the reference's
``protocol.isProofOfWorkSufficient`` (tests/golden/make_verify_golden.py) and against hashlib.

CPU part: the fixtures pin the hashlib restatement and the C ABI's host-side verdict
arithmetic (``bmpow_pow_sufficient``, no device).  GPU part (``-m gpu``): the kernel."""
import ctypes
import hashlib
import os
import random
import struct
from struct import pack

import numpy as np
import pytest

from pybitmessage_amd import _lib, targets
from tests.conftest import GOLDEN
from tests.golden.make_verify_golden import regen


@pytest.fixture(scope='module')
def kats(golden):
    if not os.path.exists(os.path.join(GOLDEN, 'verify_kats.json')):
        pytest.skip('verify_kats.json not generated')
    return golden('verify_kats.json')


@pytest.fixture(scope='module')
def hostlib():
    return _lib.load()


def sufficient_host(lib, obj, ntpb, extra, recv):
    return lib.bmpow_pow_sufficient(targets.pow_value(obj), len(obj), ntpb, extra, recv,
                                    struct.unpack('>Q', obj[8:16])[0])


# ------------------------------------------------------------------ CPU (no device)
def test_pow_restatement_matches_reference(kats):
    for k in kats['pow_kats']:
        assert targets.pow_value(regen(k, False)) == k['pow'], k['L']


def test_c_oracle_sha512_multiblock(coracle, kats):
    for k in kats['pow_kats']:
        obj = regen(k, False)
        assert coracle.sha512(obj[8:]) == hashlib.sha512(obj[8:]).digest()


def test_host_verdict_arithmetic_matches_reference(hostlib, kats):
    """The exact flip points (recvTime, ntpb, extra) found with the reference function."""
    for k in kats['verdict_kats']:
        obj = regen(k, True)
        assert targets.pow_value(obj) == k['pow']
        for c in k['checks']:
            assert sufficient_host(hostlib, obj, c['ntpb'], c['extra'], c['recvTime']) == int(c['ok']), (k['L'], c)
            assert targets.isProofOfWorkSufficient(obj, c['ntpb'], c['extra'], c['recvTime']) == c['ok']


def test_fast_verdict_list():
    """_bmpow_fast.verdicts: bytes of 0/1 -> list of bools, with the singletons' reference counts
    balanced (added in two sums, released one by one when the list goes)."""
    import sys

    from pybitmessage_amd import verify
    fast = verify._fast()
    assert fast is not None, 'the CPython marshalling module is built by build()'
    rng = random.Random(3)
    ok = bytes(rng.getrandbits(1) for _ in range(10001))
    nt = sum(ok)
    assert 4000 < nt < 6000
    rt, rf = sys.getrefcount(True), sys.getrefcount(False)
    got = fast.verdicts(ok)
    dt, df = sys.getrefcount(True) - rt, sys.getrefcount(False) - rf
    assert abs(dt - nt) <= 2 and abs(df - (len(ok) - nt)) <= 2, (dt, df, nt)  # +-2: interpreter temporaries
    assert got == [bool(b) for b in ok] and all(type(v) is bool for v in got)
    del got
    assert abs(sys.getrefcount(True) - rt) <= 2 and abs(sys.getrefcount(False) - rf) <= 2
    assert fast.verdicts(b'') == []
    with pytest.raises(TypeError):
        fast.verdicts(bytearray(b'\x01'))


def test_host_verdict_random_vs_restatement(hostlib):
    rng = random.Random(11)
    for _ in range(3000):
        L = rng.choice([16, 100, 1000, 70000, 262144])
        eol = rng.randrange(0, 1 << 62)
        recv = rng.choice([1, rng.randrange(1, 1 << 40), eol - rng.randrange(-10 ** 6, 10 ** 9) if eol > 10 ** 9 else 5])
        ntpb = rng.choice([0, 1000, 1001, rng.randrange(1, 1 << 40)])
        extra = rng.choice([0, 1000, rng.randrange(1, 1 << 40)])
        # a POW near the target so both outcomes occur
        le = L + max(extra, 1000)
        ttl = max(eol - recv, 300)
        t = 2 ** 64 / (max(ntpb, 1000) * (le + ((ttl * le) / (2 ** 16))))
        pw = min(max(int(t) + rng.randrange(-2, 3), 0), (1 << 64) - 1)
        want = pw <= t
        assert hostlib.bmpow_pow_sufficient(pw, L, ntpb, extra, recv, eol) == int(want), (pw, L, ntpb, extra, recv, eol)


# ------------------------------------------------------------------ GPU
gpu = pytest.mark.gpu


@gpu
def test_gpu_pow_values_match_reference(gpulib, kats):
    from pybitmessage_amd import verify
    objs = [regen(k, False) for k in kats['pow_kats']]
    assert verify.pow_values(objs) == [k['pow'] for k in kats['pow_kats']]


@gpu
def test_gpu_verdicts_match_reference(gpulib, kats):
    from pybitmessage_amd import verify
    objs, ntpb, extra, recv, want = [], [], [], [], []
    for k in kats['verdict_kats']:
        obj = regen(k, True)
        for c in k['checks']:
            objs.append(obj)
            ntpb.append(c['ntpb'])
            extra.append(c['extra'])
            recv.append(c['recvTime'])
            want.append(c['ok'])
        objs.append(pack('>Q', k['nonce'] + 1) + obj[8:])
        ntpb.append(1000)
        extra.append(1000)
        recv.append(k['recvTime'])
        want.append(k['next_nonce_ok'])
    assert verify.isProofOfWorkSufficient_batch(objs, ntpb, extra, recv) == want


@gpu
def test_gpu_pow_random_flood_vs_hashlib(gpulib):
    from pybitmessage_amd import verify
    rng = random.Random(5)
    objs = []
    for _ in range(3000):
        L = rng.choice([8, 9, 16, 46 + 8, 119, 120, 127, 128, 200, 1000, rng.randrange(8, 5000)])
        objs.append(rng.randbytes(L))
    objs.append(bytes(8) + rng.randbytes(300000))  # one long lane among short ones
    assert verify.pow_values(objs) == [targets.pow_value(o) for o in objs]


@gpu
def test_gpu_both_verification_kernels(gpulib, shards, monkeypatch):
    """The binned kernel (one workgroup per CU, work bins per SIMD, bmsched::plan_bins) and the
    sorted one-wave-per-group kernel give the same POW values, forced either way on a ragged flood
    (BMPOW_VBINNED); the flood is too small for the default rule to bin it, so most bins are empty.
    Then a flood large enough that the default bins it (>= 2 groups per SIMD), against hashlib."""
    from pybitmessage_amd import verify
    rng = random.Random(11)
    objs = [rng.randbytes(rng.choice([8, 16, 135, 136, rng.randrange(8, 20000)])) for _ in range(4000)]
    objs.append(bytes(8) + rng.randbytes(262144))
    want = [targets.pow_value(o) for o in objs]
    for layout in ([0], [0, 0, 0]):
        shards(layout)
        for mode in ('0', '1'):
            monkeypatch.setenv('BMPOW_VBINNED', mode)
            assert verify.pow_values(objs) == want, (layout, mode)
            with verify.VerifyBatch(objs) as vb:
                assert vb.run().tolist() == want, (layout, mode)
    monkeypatch.delenv('BMPOW_VBINNED')
    shards([0])
    big = [rng.randbytes(rng.choice([54, 208, rng.randrange(520, 16392)])) for _ in range(140000)]
    got = verify.pow_values(big)
    for i in range(0, len(big), 97):
        assert got[i] == targets.pow_value(big[i]), i


@gpu
def test_gpu_verify_session_and_shards(gpulib, shards):
    from pybitmessage_amd import verify
    rng = random.Random(8)
    objs = [rng.randbytes(rng.randrange(16, 3000)) for _ in range(500)]
    want = np.array([targets.pow_value(o) for o in objs], dtype=np.uint64)
    for layout in ([0], [0, 0], [0, 0, 0]):
        shards(layout)
        with verify.VerifyBatch(objs) as vb:
            assert np.array_equal(vb.run(), want)
            assert np.array_equal(vb.run(), want)  # resident: a second pass gives the same
    st = _lib.BmpowStats()
    gpulib.bmpow_get_stats(ctypes.byref(st))
    assert st.verify_launches > 0 and st.verify_objects >= 500


@gpu
def test_gpu_verify_edge_cases(gpulib):
    from pybitmessage_amd import verify
    assert verify.pow_values([]) == []
    assert verify.isProofOfWorkSufficient_batch([]) == []
    with pytest.raises(struct.error):
        verify.isProofOfWorkSufficient_batch([bytes(16), bytes(15)])
    with pytest.raises(struct.error):
        verify.pow_values([bytes(7)])
    # recvTime 0 means now: an object expiring far in the past gets TTL 300 either way
    obj = bytes(8) + pack('>Q', 1) + bytes(30)
    assert verify.isProofOfWorkSufficient_batch([obj], recvTime=0) == \
        [targets.isProofOfWorkSufficient(obj, 0, 0, 0)]


@gpu
def test_gpu_offsets_and_pointer_entry_points_agree(gpulib, kats):
    """bmpow_verify_batch (one concatenated buffer + offsets) and bmpow_verify_batch_ptrs (the
    objects where they lie) give the same verdicts, including the malformed-object code."""
    from pybitmessage_amd import verify
    objs = [regen(k, True) for k in kats['verdict_kats']] + [bytes(12), bytes(16)]
    n = len(objs)
    data, offsets, _ = verify._pack(objs)
    ok1 = np.zeros(n, dtype=np.uint8)
    recv = np.full(n, kats['recv'], dtype=np.int64)
    _lib.check(gpulib, gpulib.bmpow_verify_batch(n, data, offsets.ctypes.data_as(verify.P64), None, None,
                                                 recv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                 ok1.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), 'offsets')
    ptrs = verify._pointers(objs)
    lens = np.fromiter(map(len, objs), dtype=np.uint64, count=n)
    ok2 = np.zeros(n, dtype=np.uint8)
    _lib.check(gpulib, gpulib.bmpow_verify_batch_ptrs(n, ptrs.ctypes.data, lens.ctypes.data_as(verify.P64), None,
                                                      None, recv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                      ok2.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), 'ptrs')
    assert ok1.tolist() == ok2.tolist()
    assert ok1.tolist() == [1] * (n - 2) + [2, 0]


def test_fast_marshalling_passes_every_object_in_place():
    """csrc/bmpow_pyext.c (the CPython walk of the object list) hands bmpow_verify_batch_ptrs each
    bytes object's own buffer and length, the scalar difficulty and recvTime, and returns its flags
    -- checked with a ctypes stand-in for the entry point (no device)."""
    import ctypes

    from pybitmessage_amd import verify
    fast = verify._load_fast()
    if fast is None:
        pytest.skip('_bmpow_fast not built')
    objs = [bytes([i % 251]) * (16 + i) for i in range(3000)]
    seen = {}
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                             ctypes.POINTER(ctypes.c_uint8))

    def fake(n, ptrs, lens, ntpb, extra, recv, ok):
        seen['n'] = n
        for i in range(n):
            assert ctypes.string_at(ptrs[i], lens[i]) == objs[i]
            assert (ntpb[i], extra[i], recv[i]) == (1234, 5678, 1700000000)
            ok[i] = lens[i] & 1
        return 0
    cb = proto(fake)
    rc, ok = fast.verify_list(ctypes.cast(cb, ctypes.c_void_p).value, objs, 1234, 5678, 1700000000)
    assert rc == 0 and seen['n'] == len(objs)
    assert list(ok) == [len(o) & 1 for o in objs]
    with pytest.raises(TypeError):
        fast.verify_list(ctypes.cast(cb, ctypes.c_void_p).value, [b'x' * 20, bytearray(20)], 0, 0, 0)

    # zero difficulty / recvTime (the network minimum, "now") go as null arrays, which the library
    # reads as 0 for every object
    def fake0(n, ptrs, lens, ntpb, extra, recv, ok):
        seen['null'] = (not ntpb, not extra, not recv)
        for i in range(n):
            ok[i] = 1
        return 0
    cb0 = proto(fake0)
    rc, ok = fast.verify_list(ctypes.cast(cb0, ctypes.c_void_p).value, objs[:50], 0, 0, 0)
    assert rc == 0 and seen['null'] == (True, True, True) and list(ok) == [1] * 50


def test_fast_marshalling_holds_the_objects_while_the_gil_is_released():
    """The walk takes a reference to every object before it releases the GIL: another thread that
    empties the list meanwhile (here the stand-in entry point itself) frees nothing the library is
    reading, and the references are dropped again afterwards."""
    import ctypes
    import sys

    from pybitmessage_amd import verify
    fast = verify._load_fast()
    if fast is None:
        pytest.skip('_bmpow_fast not built')
    objs = [bytes([7, i % 256]) * (300 + i) for i in range(200)]
    expect = [bytes(o) for o in objs]
    refs = [sys.getrefcount(o) for o in objs]
    shared = list(objs)
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64),
                             ctypes.POINTER(ctypes.c_uint8))
    state = {}

    def fake(n, ptrs, lens, ntpb, extra, recv, ok):
        state['during'] = [sys.getrefcount(o) for o in objs]
        del shared[:]
        for i in range(n):
            assert ctypes.string_at(ptrs[i], lens[i]) == expect[i]
            ok[i] = 1
        return 0
    cb = proto(fake)
    rc, ok = fast.verify_list(ctypes.cast(cb, ctypes.c_void_p).value, shared, 0, 0, 0)
    assert rc == 0 and list(ok) == [1] * len(objs)
    assert all(d == r + 2 for d, r in zip(state['during'], refs))  # the list's + the walk's own
    assert [sys.getrefcount(o) for o in objs] == refs
