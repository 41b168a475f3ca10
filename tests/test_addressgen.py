"""RIPE-prefix address search against fixtures produced by the reference's
own primitives (tests/golden/make_addr_golden.py) and the reference's test vectors
(src/tests/samples.py).

CPU: the oracle (oracle/addrgen_oracle.py) and the host-side formats (encodeAddress, WIF) are
pinned to the fixtures.  GPU (``-m gpu``): pointMult, every per-try value and the exact search
result through the C ABI."""
import hashlib

import pytest

from oracle import addrgen_oracle as ao
from pybitmessage_amd import _lib, addressgen

# src/tests/samples.py (the reference's own vectors)
SAMPLE_SEED = b'TIGER, tiger, burning bright. In the forests of the night'
SAMPLE_DET_RIPE = '00cfb69416ae76f68a81c459de4e13460c7d17eb'
SAMPLE_DET_ADDR3 = 'BM-2DBPTgeSawWYZceFD69AbDT5q4iUWtj1ZN'
SAMPLE_DET_ADDR4 = 'BM-2cWzSnwjJ7yRP3nLEWUV5LisTZyREWSzUK'
SAMPLE_PRIV_S = '93d0b61371a54b53df143b954035d612f8efa8a3ed1cf842c2186bfd8f876665'
SAMPLE_PRIV_E = '4b0b73a54e19b059dc274ab69df095fe699f43b17397bca26fdf40f4d7400a3a'
SAMPLE_PUB_S = ('044a367f049ec16cb6b6118eb734a9962d10b8db59c890cd08f210c43ff08bdf09d'
                '16f502ca26cd0713f38988a1237f1fc8fa07b15653c996dc4013af6d15505ce')
SAMPLE_PUB_E = ('044597d59177fc1d89555d38915f581b5ff2286b39d022ca0283d2bdd5c36be5d3c'
                'e7b9b97792327851a562752e4b79475d1f51f5a71352482b241227f45ed36a9')
SAMPLE_RIPE = '003cd097eb7f35c87b5dc8b4538c22cb55312a9f'
SAMPLE_ADDR_V2 = 'BM-onkVu1KKL2UaUss5Upg9vXmqd3esTmV79'
SAMPLE_FACTOR = 66858749573256452658262553961707680376751171096153613379801854825275240965733
SAMPLE_POINT = (33567437183004486938355437500683826356288335339807546987348409590129959362313,
                94730058721143827257669456336351159718085716196507891067256111928318063085006)

# RIPEMD-160 test vectors of its designers (Dobbertin, Bosselaers, Preneel)
RIPEMD_VECTORS = {b'': '9c1185a5c5e9fc54612808977ee8f548b2258d31',
                  b'a': '0bdc9d2d256b3ee9daae347be6f4dc835a467ffe',
                  b'abc': '8eb208f7e05d987a9b044a8e98c6b087f15a0bfc',
                  b'message digest': '5d0689ef49d2fae572b881b123a85ffa21595f36',
                  b'abcdefghijklmnopqrstuvwxyz': 'f71c27109c692c1b56bbdceb5b9d2865b3708dbc'}


@pytest.fixture(scope='module')
def kats(golden):
    return golden('addr_kats.json')


# ------------------------------------------------------------------ CPU: oracle + formats
def test_oracle_ripemd160_vectors():
    for m, h in RIPEMD_VECTORS.items():
        assert ao.ripemd160(m).hex() == h


def test_oracle_openssl_ripemd160_matches_restatement():
    """The libcrypto RIPEMD160() binding (bench CPU baseline) against the specification vectors
    and the pure-Python restatement."""
    try:
        rmd = ao.OpenSSLRipemd160()
    except Exception as e:  # noqa: BLE001
        pytest.skip('libcrypto unavailable: %s' % e)
    import random
    for m, h in RIPEMD_VECTORS.items():
        assert rmd(m).hex() == h
    rng = random.Random(9)
    for n in (0, 55, 56, 63, 64, 65, 130, 1000):
        m = rng.randbytes(n)
        assert rmd(m) == ao.ripemd160(m)


def test_oracle_matches_reference_samples():
    assert ao.point_mult_xy(SAMPLE_FACTOR) == SAMPLE_POINT
    ps = ao.point_mult(bytes.fromhex(SAMPLE_PRIV_S))
    pe = ao.point_mult(bytes.fromhex(SAMPLE_PRIV_E))
    assert ps.hex() == SAMPLE_PUB_S and pe.hex() == SAMPLE_PUB_E
    assert ao.ripe_of(ps, pe).hex() == SAMPLE_RIPE
    k, ripe, _, _ = ao.deterministic_search(SAMPLE_SEED, 1)
    assert ripe.hex() == SAMPLE_DET_RIPE and k == 21


def test_oracle_matches_reference_fixtures(kats):
    for t in kats['pointmult_kats'][:20]:
        assert ao.point_mult(bytes.fromhex(t['priv'])).hex() == t['pub']
    for t in kats['try_kats'][::5]:
        ps, pe = ao.try_keys(bytes.fromhex(t['passphrase']), t['k'])
        assert ps.hex() == t['priv_signing'] and pe.hex() == t['priv_encryption']
        assert ao.ripe_of(ao.point_mult(ps), ao.point_mult(pe)).hex() == t['ripe']


def test_oracle_openssl_pointmult_matches_restatement():
    """The libcrypto EC_POINT_mul binding (bench CPU baseline, random-mode test) against the
    pure-Python pointMult and the reference's sample keys."""
    try:
        pm = ao.OpenSSLPointMult()
    except Exception as e:  # noqa: BLE001
        pytest.skip('libcrypto unavailable: %s' % e)
    import random
    rng = random.Random(5)
    for k in [bytes.fromhex(SAMPLE_PRIV_S), bytes.fromhex(SAMPLE_PRIV_E)] + [rng.randbytes(32) for _ in range(8)]:
        assert pm(k) == ao.point_mult(k)
    assert pm(bytes.fromhex(SAMPLE_PRIV_S)).hex() == SAMPLE_PUB_S


def test_address_formats_match_reference(kats):
    assert addressgen.encodeAddress(2, 1, bytes.fromhex(SAMPLE_RIPE)) == SAMPLE_ADDR_V2
    assert addressgen.encodeAddress(3, 1, bytes.fromhex(SAMPLE_DET_RIPE)) == SAMPLE_DET_ADDR3
    assert addressgen.encodeAddress(4, 1, bytes.fromhex(SAMPLE_DET_RIPE)) == SAMPLE_DET_ADDR4
    for s in kats['search_kats']:
        ripe = bytes.fromhex(s['ripe'])
        assert addressgen.encodeAddress(3, 1, ripe) == s['addr3']
        assert addressgen.encodeAddress(4, 1, ripe) == s['addr4']
        assert addressgen.encodeAddress(4, 2, ripe) == s['addr4_stream2']
    t = [t for t in kats['try_kats'] if t['passphrase'] == SAMPLE_SEED.hex() and t['k'] == 0][0]
    assert addressgen.wif(bytes.fromhex(t['priv_signing']))[0] == '5'
    for v in [0, 1, 252, 253, 65535, 65536, 2 ** 32 - 1, 2 ** 32, 2 ** 64 - 1]:
        assert addressgen.encodeVarint(v) == ao.encode_varint(v)


def test_wif_matches_reference(kats):
    for s in kats['search_kats']:
        pp = bytes.fromhex(s['passphrase'])
        ps, pe = ao.try_keys(pp, s['k'])
        assert addressgen.wif(ps) == s['wif_signing'] and addressgen.wif(pe) == s['wif_encryption']


# ------------------------------------------------------------------ GPU
gpu = pytest.mark.gpu


@gpu
def test_gpu_pubkeys_match_reference(gpulib, kats):
    privs = [bytes.fromhex(t['priv']) for t in kats['pointmult_kats']]
    privs += [bytes.fromhex(SAMPLE_PRIV_S), bytes.fromhex(SAMPLE_PRIV_E), SAMPLE_FACTOR.to_bytes(32, 'big')]
    got = addressgen.pubkeys(privs)
    want = [t['pub'] for t in kats['pointmult_kats']] + [SAMPLE_PUB_S, SAMPLE_PUB_E]
    assert [g.hex() for g in got[:-1]] == want
    x, y = SAMPLE_POINT
    assert got[-1] == b'\x04' + x.to_bytes(32, 'big') + y.to_bytes(32, 'big')
    assert addressgen.pubkeys([bytes(32)]) == [bytes(65)]  # k = 0: the point at infinity


@gpu
def test_gpu_pubkeys_random_vs_oracle(gpulib):
    import random
    rng = random.Random(3)
    privs = [rng.randbytes(32) for _ in range(200)]
    assert addressgen.pubkeys(privs) == [ao.point_mult(p) for p in privs]


@gpu
def test_gpu_every_try_value_matches_reference(gpulib, kats):
    """null_bytes = 0 accepts any try, so a 1-try search returns try k itself."""
    for t in kats['try_kats']:
        f = addressgen.search_deterministic(bytes.fromhex(t['passphrase']), 0, t['k'], 1)
        assert f.k == t['k']
        assert (f.priv_signing.hex(), f.priv_encryption.hex()) == (t['priv_signing'], t['priv_encryption'])
        assert (f.pub_signing.hex(), f.pub_encryption.hex()) == (t['pub_signing'], t['pub_encryption'])
        assert f.ripe.hex() == t['ripe'], (t['passphrase'][:16], t['k'])


@gpu
def test_gpu_search_matches_reference(gpulib, kats):
    runs = {}
    for s in kats['search_kats']:
        runs.setdefault((s['passphrase'], s['null_bytes']), []).append(s)
    for (pp, nb), ss in runs.items():
        got = addressgen.deterministic_addresses(bytes.fromhex(pp), len(ss), 4, 1, nb)
        for g, s in zip(got, ss):
            assert (g['k'], g['ripe'].hex(), g['address']) == (s['k'], s['ripe'], s['addr4']), s['label']
            assert g['privSigningKey'] == s['wif_signing'] and g['privEncryptionKey'] == s['wif_encryption']
    # the reference's own sample (src/tests/samples.py:32-36)
    g = addressgen.deterministic_addresses(SAMPLE_SEED, 1, 3)[0]
    assert g['address'] == SAMPLE_DET_ADDR3 and g['ripe'].hex() == SAMPLE_DET_RIPE


@gpu
def test_gpu_search_budget_and_shards(gpulib, shards):
    assert addressgen.search_deterministic(SAMPLE_SEED, 1, 0, 21) is None  # answer is k = 21
    assert addressgen.search_deterministic(SAMPLE_SEED, 1, 0, 22).k == 21
    assert addressgen.search_deterministic(SAMPLE_SEED, 1, 21, 1).k == 21
    shards([0, 0, 0])
    assert addressgen.search_deterministic(SAMPLE_SEED, 1).k == 21
    assert addressgen.search_deterministic(b'two null bytes', 2).k == 5640


@pytest.fixture
def comb24(gpulib):
    """Force the 24-bit comb (10.7 GB table) for the test, restore automatic choice after."""
    lib = _lib.get()
    lib.bmpow_addr_set_comb(24)
    yield lib
    lib.bmpow_addr_set_comb(0)


@gpu
def test_gpu_large_comb_every_try_and_search(comb24, kats):
    """The 24-bit comb (ragged last window of 16 bits) gives the reference's values for every
    per-try fixture and the reference's first k for every search fixture."""
    for t in kats['try_kats']:
        f = addressgen.search_deterministic(bytes.fromhex(t['passphrase']), 0, t['k'], 1)
        assert comb24.bmpow_addr_last_comb() == 24
        assert (f.pub_signing.hex(), f.pub_encryption.hex()) == (t['pub_signing'], t['pub_encryption'])
        assert f.ripe.hex() == t['ripe'], (t['passphrase'][:16], t['k'])
    runs = {}
    for s in kats['search_kats']:
        runs.setdefault((s['passphrase'], s['null_bytes']), []).append(s)
    for (pp, nb), ss in runs.items():
        got = addressgen.deterministic_addresses(bytes.fromhex(pp), len(ss), 4, 1, nb)
        for g, s in zip(got, ss):
            assert (g['k'], g['ripe'].hex(), g['address']) == (s['k'], s['ripe'], s['addr4']), s['label']
    g = addressgen.deterministic_addresses(SAMPLE_SEED, 1, 3)[0]
    assert g['address'] == SAMPLE_DET_ADDR3 and g['ripe'].hex() == SAMPLE_DET_RIPE


@gpu
def test_gpu_comb_policy(gpulib, shards):
    """Automatic choice: the 16-bit comb for short searches, the 24-bit one once built (and on
    every shard); an explicit width is validated."""
    lib = _lib.get()
    assert lib.bmpow_addr_set_comb(0) in (0, 16, 24)
    shards([0, 0])  # fresh shards: no table built yet
    assert addressgen.search_deterministic(SAMPLE_SEED, 1).k == 21
    assert lib.bmpow_addr_last_comb() == 16
    lib.bmpow_addr_set_comb(24)
    assert addressgen.search_deterministic(SAMPLE_SEED, 1).k == 21
    assert lib.bmpow_addr_last_comb() == 24
    lib.bmpow_addr_set_comb(0)
    assert addressgen.search_deterministic(b'two null bytes', 2).k == 5640
    assert lib.bmpow_addr_last_comb() == 24  # already built: used
    assert lib.bmpow_addr_set_comb(20) < 0
    assert lib.bmpow_addr_set_comb(16) == 0
    assert addressgen.search_deterministic(b'two null bytes', 2).k == 5640
    assert lib.bmpow_addr_last_comb() == 16
    lib.bmpow_addr_set_comb(0)


@gpu
def test_gpu_random_address_property(gpulib):
    import os
    seed, priv_s = os.urandom(64), os.urandom(32)
    a = addressgen.random_address(4, 1, 1, priv_s, seed)
    lib = _lib.get()
    assert a['ripe'][:1] == b'\x00'
    # re-derive everything on the host: the keys must reproduce the ripe
    pe = hashlib.sha512(seed + ao.encode_varint(a['k'])).digest()[:32]
    assert a['pubEncryptionKey'] == ao.point_mult(pe) and a['pubSigningKey'] == ao.point_mult(priv_s)
    assert ao.ripe_of(a['pubSigningKey'], a['pubEncryptionKey']) == a['ripe']
    assert addressgen.wif(priv_s) == a['privSigningKey'] and addressgen.wif(pe) == a['privEncryptionKey']
    assert lib is not None


# ------------------------------------------------------------------ GPU: field arithmetic edges
P = 2 ** 256 - 2 ** 32 - 977
C = 2 ** 32 + 977  # 2^256 mod p


def _fe_edges():
    """Operands a random key essentially never produces: unreduced values (>= p), values next to
    0, p and 2^256, and the ones that make a sum carry twice or a difference borrow twice."""
    import random
    rng = random.Random(11)
    base = [0, 1, 2, 977, C - 1, C, C + 1, 2 ** 32, 2 ** 64 - 1, P - 2, P - 1, P, P + 1, P + C - 1,
            2 ** 256 - C, 2 ** 256 - C - 1, 2 ** 256 - 2, 2 ** 256 - 1, 2 ** 255, 2 ** 255 - 1]
    base += [P + rng.randrange(C) for _ in range(8)] + [rng.randrange(2 ** 256) for _ in range(8)]
    base += [rng.randrange(2 ** 66) for _ in range(4)] + [2 ** 256 - 1 - rng.randrange(2 ** 40) for _ in range(4)]
    pairs = [(a, b) for a in base for b in base]
    pairs += [(rng.randrange(2 ** 256), rng.randrange(2 ** 256)) for _ in range(2000)]
    return pairs


def _fe_probe(op, pairs):
    import ctypes
    lib = _lib.get()
    n = len(pairs)
    limbs = lambda v: [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]  # noqa: E731
    a = (ctypes.c_uint32 * (8 * n))(*[w for x, _ in pairs for w in limbs(x)])
    b = (ctypes.c_uint32 * (8 * n))(*[w for _, y in pairs for w in limbs(y)])
    out = (ctypes.c_uint32 * (8 * n))()
    _lib.check(lib, lib.bmpow_fe_probe(op, n, a, b, out), 'bmpow_fe_probe')
    return [sum(out[8 * k + i] << (32 * i) for i in range(8)) for k in range(n)]


@gpu
@pytest.mark.parametrize('op', [0, 1, 2, 3])
def test_gpu_field_ops_weakly_reduced_at_the_edges(gpulib, op):
    """add/sub/mul/sqr on any inputs < 2^256: result < 2^256 and congruent mod p (weak reduction,
    secp256k1_dev.h), including the second carry/borrow folds."""
    pairs = _fe_edges()
    want = [(a + b, a - b, a * b, a * a)[op] % P for a, b in pairs]
    got = _fe_probe(op, pairs)
    bad = [(hex(a), hex(b)) for (a, b), g, w in zip(pairs, got, want) if g >= 2 ** 256 or g % P != w]
    assert not bad, bad[:4]


@gpu
def test_gpu_field_normalize_inverse_is_zero(gpulib):
    pairs = _fe_edges()
    assert _fe_probe(4, pairs) == [a % P for a, _ in pairs]
    assert _fe_probe(5, pairs) == [pow(a % P, -1, P) if a % P else 0 for a, _ in pairs]
    assert _fe_probe(6, pairs) == [int(a % P == 0) for a, _ in pairs]


@gpu
def test_gpu_pubkeys_at_the_group_order(gpulib):
    """Scalars around the group order n: k = n sums to the point at infinity inside the comb's
    last window (P + (-P)), n + 1 is G, n - 1 is -G, and 2^256 - 1 = (2^256 - 1 - n) G."""
    n = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    ks = [n, n + 1, n - 1, 2 ** 256 - 1, n - 2 ** 240, 2 ** 240]
    got = addressgen.pubkeys([k.to_bytes(32, 'big') for k in ks])
    assert got[0] == bytes(65)
    for k, g in zip(ks[1:], got[1:]):
        assert g == ao.point_mult((k % n).to_bytes(32, 'big'))


@gpu
def test_gpu_random_mode_first_try_and_lane_boundaries(gpulib):
    """Random mode runs four tries per lane (one inversion for four encryption keys): the search
    must still return the FIRST k >= start with the prefix, whatever the alignment of start and
    of the budget to the lanes.  The answer comes from the host restatement of the loop."""
    import ctypes
    seed = hashlib.sha512(b'bmpow random-mode test').digest()
    priv_s = hashlib.sha256(b'bmpow random-mode signing key').digest()
    try:  # libcrypto's EC_POINT_mul (pinned by test_oracle_openssl_pointmult_matches_restatement)
        pm = ao.OpenSSLPointMult()
    except Exception:  # noqa: BLE001
        pm = ao.point_mult
    pub_s = pm(priv_s)

    def prefix_at(k):
        pe = hashlib.sha512(seed + ao.encode_varint(k)).digest()[:32]
        return ao.ripe_of(pub_s, pm(pe))[:1] == b'\x00'

    hits, k = [], 0
    while len(hits) < 3 and k < 4000:
        if prefix_at(k):
            hits.append(k)
        k += 1
    assert len(hits) == 3, hits
    lib = _lib.get()

    def search(start, n):
        out = _lib.BmpowAddress()
        rc = _lib.check(lib, lib.bmpow_address_search_random(priv_s, seed, len(seed), start, n, 1, ctypes.byref(out)),
                        'bmpow_address_search_random')
        return out.k if rc == _lib.FOUND else None

    for h in hits[:3]:
        for start in {max(h - d, 0) for d in (0, 1, 2, 3, 4, 5, 7, 64, 257)}:
            want = next(x for x in hits if x >= start)
            assert search(start, 2000) == want, (start, want)
            assert search(start, h - start + 1) == want  # the budget ends on the hit
            if want == h and h > start:
                assert search(start, h - start) is None  # ... or just before it
