"""The oracle is pinned before anything is checked against it (CPU only).

Golden vectors in tests/golden/ were produced by running the reference itself
(tests/golden/make_golden.py): ``_pool_worker`` / ``_doSafePoW`` (src/proofofwork.py:90-111),
``protocol.isProofOfWorkSufficient`` (src/protocol.py:258-286).
"""
import hashlib
import os
import random

import pytest

from oracle import oracle

U64 = 1 << 64


def test_c_sha512_matches_hashlib(coracle):
    rng = random.Random(7)
    for L in list(range(0, 300)) + [1000, 4095, 4096, 16384]:
        d = rng.randbytes(L)
        assert coracle.sha512(d) == hashlib.sha512(d).digest(), L


def test_trial_kats_python_and_c(golden, coracle):
    kats = golden('trial_kats.json')['kats']
    assert len(kats) > 300
    for k in kats:
        ih = bytes.fromhex(k['ih'])
        assert oracle.trial(k['nonce'], ih) == k['trial']
        assert coracle.trial(k['nonce'], ih) == k['trial']


def test_any_length_kats_python_and_c(golden, coracle):
    """initialHash lengths other than 64 (tests/golden/make_len_golden.py, the reference's own
    _pool_worker and _doSafePoW): every SHA-512 block edge of the first hash's message."""
    d = golden('len_kats.json')
    assert {0, 1, 63, 65, 103, 104, 231, 232, 1000} <= set(d['lengths'])
    for k in d['trial']:
        ih = bytes.fromhex(k['ih'])
        assert len(ih) == k['len']
        assert oracle.trial(k['nonce'], ih) == k['trial']
        assert coracle.trial_len(k['nonce'], ih) == k['trial']
    for k in d['first']:
        ih = bytes.fromhex(k['ih'])
        assert oracle.safe_pow(k['target'], ih) == [k['trial'], k['nonce']]
        assert coracle.search_len(ih, k['target']) == (k['trial'], k['nonce'])
    # the 64-byte path of the any-length function is the fixed-layout one
    ih = hashlib.sha512(b'hello').digest()
    assert coracle.trial_len(1315, ih) == coracle.trial(1315, ih)


def test_survey_appendix_trial_values(coracle):
    # SURVEY.md Appendix A, computed independently during the survey
    ih0 = bytes(64)
    hello = hashlib.sha512(b'hello').digest()
    assert coracle.trial(0, ih0) == 15384050719303346949
    assert coracle.trial(1, ih0) == 2274854268764994929
    assert coracle.trial(1 << 32, ih0) == 6525330889464198002
    assert coracle.trial(U64 - 1, ih0) == 2198939099669698234
    assert coracle.trial(1, hello) == 13542169780345634238
    assert coracle.trial(1 << 63, hello) == 16364079262595905430


def test_first_nonce_kats_c_oracle(golden, coracle):
    for k in golden('first_nonce_kats.json')['kats']:
        ih = bytes.fromhex(k['ih'])
        if k['nonce'] > 2_000_000:
            continue  # the slow vectors are covered by test_first_nonce_slow_kats_mt
        assert coracle.search(ih, k['target']) == (k['trial'], k['nonce']), k['note']


def test_search_many_is_search_in_order(golden, coracle):
    """search_many (the GPU tests' checker for many objects) = search per object, in input order."""
    kats = [k for k in golden('first_nonce_kats.json')['kats'] if k['nonce'] <= 200_000]
    jobs = [(k['target'], bytes.fromhex(k['ih'])) for k in kats]
    assert len(jobs) >= 8
    assert coracle.search_many(jobs, threads=4) == [(k['trial'], k['nonce']) for k in kats]
    assert coracle.search_many(jobs[:3], threads=1) == [coracle.search(ih, t) for t, ih in jobs[:3]]


def test_first_nonce_slow_kats_mt(golden, coracle):
    for k in golden('first_nonce_kats.json')['kats']:
        if k['nonce'] <= 2_000_000 or k['nonce'] > 50_000_000:
            continue
        ih = bytes.fromhex(k['ih'])
        res, done = coracle.search_mt(ih, k['target'], 1, 1 << 40, threads=os.cpu_count() or 4)
        assert res == (k['trial'], k['nonce']), k['note']
        assert done >= k['nonce'] - 1


def test_first_nonce_kats_python_restatement(golden):
    for k in golden('first_nonce_kats.json')['kats']:
        if k['nonce'] > 20000:
            continue
        ih = bytes.fromhex(k['ih'])
        assert oracle.safe_pow(k['target'], ih) == [k['trial'], k['nonce']]


def test_batch_kats(golden, coracle):
    d = golden('batch_kats.json')
    rng = random.Random(d['seed'])
    for k in d['kats']:
        payload = rng.randbytes(k['L'])
        ih = hashlib.sha512(payload).digest()
        assert ih.hex() == k['ih']
        tgt = oracle.target_from_formula(k['L'], d['ttl'], d['ntpb'], d['extra'])
        assert tgt == k['target']
        assert coracle.search(ih, tgt) == (k['trial'], k['nonce'])


def test_search_budget_and_resume(coracle):
    ih = hashlib.sha512(b'hello').digest()
    assert coracle.search(ih, U64 // 1000, 1, 1314) is None
    assert coracle.search(ih, U64 // 1000, 1315, 1) == (2417842470843601, 1315)


def test_search_mt_exact_vs_sequential(coracle):
    rng = random.Random(11)
    for _ in range(12):
        ih = rng.randbytes(64)
        tgt = U64 // rng.choice([50, 500, 5000, 50000])
        seq = coracle.search(ih, tgt)
        mt, _ = coracle.search_mt(ih, tgt, 1, 1 << 30, threads=4)
        assert seq == mt


def test_search_top_of_nonce_space(coracle):
    ih = hashlib.sha512(b'edge').digest()
    start = U64 - 300
    tv = [coracle.trial(n, ih) for n in range(start, U64)]
    m = min(tv)
    want = start + tv.index(m)
    assert coracle.search(ih, m, start, 1000) == (m, want)
    res, done = coracle.search_mt(ih, m, start, 1 << 20, threads=3)
    assert res == (m, want)
    # nothing at or below target 0 in the last 300 nonces: budget stops at 2^64-1
    assert coracle.search(ih, 0, start, 1000) is None
    assert coracle.search_mt(ih, 0, start, 1 << 20, threads=3)[1] == 300


@pytest.mark.skipif(not oracle.have_ref(), reason='oracle/_ref/bitmsghash.so not built')
def test_reference_c_library_returns_a_valid_nonce():
    """The reference's BitmessagePOW is nondeterministic and strict-<:
    only validity is checked, never equality with _doSafePoW."""
    ref = oracle.RefBitmsghash()
    ih = hashlib.sha512(b'hello').digest()
    tv, nonce = ref.pow(U64 // 1000, ih)
    assert tv < U64 // 1000 and nonce >= 1
    assert oracle.trial(nonce, ih) == tv


def test_config_targets_formula(golden):
    for t in golden('config_targets.json')['targets']:
        if t['kind'] == 'singleWorker':
            got = oracle.target_from_formula(t['L'], t['ttl'], t['ntpb'], t['extra'])
            assert got == t['target']
    c1 = [t for t in golden('config_targets.json')['targets'] if t['L'] == 1024 and t.get('ttl') == 345600
          and t['ntpb'] == 1000][0]
    assert c1['target'] == 1447073009577


def test_min_trial_oracle_vs_python(coracle):
    """bmo_min_trial (the checker of the device min-trial probe) against a hashlib loop:
    ragged ranges, empty ranges, ranges clipped at 2^64-1."""
    import random as _r
    from oracle.oracle import U64_MAX, trial
    rng = _r.Random(11)
    for start, count in [(0, 1), (1, 500), (12345, 77), (U64_MAX - 30, 31), (U64_MAX - 5, 100), (7, 0)]:
        ih = rng.randbytes(64)
        got = coracle.min_trial(ih, start, count)
        if count == 0:
            assert got == (U64_MAX, start)
            continue
        end = min(start + count, U64_MAX + 1)
        tv = [(trial(n, ih), n) for n in range(start, end)]
        assert got == min(tv)
