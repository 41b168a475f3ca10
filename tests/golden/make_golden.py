#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only):

    BITMESSAGE_HOME=$(mktemp -d) PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--slow]

What each fixture pins, and which reference code produced it:

* ``trial_kats.json``   trial(n, ih) at boundary and random nonces, produced by the reference's
  ``proofofwork._pool_worker(n - 1, ih, 2**64, 1)`` (src/proofofwork.py:90-97), whose first
  iteration hashes nonce ``n`` and always accepts.
* ``first_nonce_kats.json``  (ih, target) -> [trialValue, nonce] from the reference's
  ``proofofwork._doSafePoW`` (src/proofofwork.py:100-111).  ``--slow`` adds the C1 object
  (~11M trials, ~20 s) and the test_openclpow vector (src/tests/test_openclpow.py:22-26),
  whose 224M-trial answer comes from the C oracle's exhaustive scan; the reference's
  ``_pool_worker`` then rescans the last 2^16 nonces below it and must land on it.
* ``batch_kats.json``   SURVEY Appendix A batch at test-mode difficulty (ntpb = extra = 10),
  payloads ``random.Random(20250216).randbytes(L)`` drawn in sequence, solved by ``_doSafePoW``.
* ``config_targets.json`` target formula (class_singleWorker.py:219-231) for the BASELINE
  configs, evaluated with the same float expression, plus the API variant (api.py:1288-1293).
* ``verifier_kats.json`` finished objects (nonce || payload) at default difficulty, solved by
  the C oracle and judged by the reference's ``protocol.isProofOfWorkSufficient``
  (src/protocol.py:258-286) at a fixed recvTime.
"""
import argparse
import hashlib
import json
import os
import random
import sys
import time
from struct import pack

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = '/root/reference/src'
SEED = 20250216
U64 = 1 << 64


def hx(b):
    return b.hex()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--slow', action='store_true')
    args = ap.parse_args()
    sys.path.insert(0, REF_SRC)
    import proofofwork  # reference module (do NOT call proofofwork.init(): it runs make in the ref tree)
    import protocol

    def ref_trial(n, ih):
        tv, nn = proofofwork._pool_worker(n - 1, ih, U64, 1)
        assert nn == n
        return tv

    ih0 = bytes(64)
    ih_hello = hashlib.sha512(b'hello').digest()
    rng = random.Random(SEED + 1)

    # ---------------- trial KATs ----------------
    kats = []
    special = [1, 2, 255, 256, 65535, 65536, (1 << 32) - 1, 1 << 32, (1 << 32) + 1,
               (1 << 40) + 12345, (1 << 63) - 1, 1 << 63, U64 - 2, U64 - 1]
    ihs = [ih0, ih_hello, bytes(range(64)), b'\xff' * 64]
    for ih in ihs:
        for n in special:
            kats.append({'ih': hx(ih), 'nonce': n, 'trial': ref_trial(n, ih)})
    for _ in range(64):
        ih = rng.randbytes(64)
        n = rng.randrange(1, U64)
        kats.append({'ih': hx(ih), 'nonce': n, 'trial': ref_trial(n, ih)})
    # a contiguous run (exercises consecutive-lane nonces inside one wave)
    ihr = hashlib.sha512(b'bmpow-run').digest()
    for n in range(1, 257):
        kats.append({'ih': hx(ihr), 'nonce': n, 'trial': ref_trial(n, ihr)})
    # nonce 0 is not reachable through _pool_worker(-1, ..) without packing -1; use the
    # reference expression (proofofwork.py:106-107) verbatim for it
    from struct import unpack
    for ih in ihs:
        tv, = unpack('>Q', hashlib.sha512(hashlib.sha512(pack('>Q', 0) + ih).digest()).digest()[0:8])
        kats.append({'ih': hx(ih), 'nonce': 0, 'trial': tv})
    dump('trial_kats.json', {'source': 'reference proofofwork._pool_worker (src/proofofwork.py:90-97)',
                             'kats': kats})

    # ---------------- first-nonce KATs ----------------
    fn = []

    def add(ih, target, note):
        t0 = time.time()
        tv, nonce = proofofwork._doSafePoW(target, ih)
        fn.append({'ih': hx(ih), 'target': target, 'nonce': nonce, 'trial': tv, 'note': note,
                   'source': 'reference _doSafePoW'})
        print('  %-40s nonce=%d (%.1fs)' % (note, nonce, time.time() - t0))

    add(ih_hello, U64 // 1000, 'hello 2^64//1000 (SURVEY App.A: 1315)')
    add(ih_hello, 184467440737095, 'hello 2^64/1e5 (SURVEY App.A: 129430)')
    add(ih0, U64 - 1, 'target 2^64-1: nonce 1')
    t1 = ref_trial(1, ih_hello)
    add(ih_hello, t1, 'target == trial(1): nonce 1 (<= accepted)')
    add(ih_hello, t1 - 1, 'target == trial(1)-1: skips nonce 1')
    for i in range(40):
        ih = rng.randbytes(64)
        e = rng.choice([16, 100, 1000, 5000, 20000, 60000])
        add(ih, U64 // e, 'random #%d E=%d' % (i, e))
    # pairs of objects sharing a prefix-close target: catches min-vs-any confusion
    for i in range(8):
        ih = rng.randbytes(64)
        add(ih, U64 // 300000, 'random hard #%d E=3e5' % i)
    if args.slow:
        c1_payload = random.Random(SEED).randbytes(1024)
        c1_ih = hashlib.sha512(c1_payload).digest()
        c1_target = int(2 ** 64 / (1000 * (1024 + 8 + 1000 + ((345600 * (1024 + 8 + 1000)) / (2 ** 16)))))
        add(c1_ih, c1_target, 'C1 1KB msg at defaults (SURVEY: 10909138)')
        ocl_ih = bytes.fromhex(
            '3758f55b5a8d902fd3597e4ce6a2d3f23daff735f65d9698c270987f4e67ad59'
            '0b93f3ffeba0ef2fd08a8dc2f87b68ae5a0dc819ab57f22ad2c4c9c8618a43b3')
        fn.append(openclpow_vector(proofofwork, ocl_ih, 54227212183))
    dump('first_nonce_kats.json', {'kats': fn})

    # ---------------- batch KATs (test-mode difficulty) ----------------
    brng = random.Random(SEED)
    batch = []
    for L in [46, 200, 512, 1024, 4096, 16384]:
        payload = brng.randbytes(L)
        ih = hashlib.sha512(payload).digest()
        target = int(2 ** 64 / (10 * (L + 8 + 10 + ((345600 * (L + 8 + 10)) / (2 ** 16)))))
        tv, nonce = proofofwork._doSafePoW(target, ih)
        batch.append({'L': L, 'ih': hx(ih), 'target': target, 'nonce': nonce, 'trial': tv})
        print('  batch L=%d nonce=%d' % (L, nonce))
    dump('batch_kats.json', {'ntpb': 10, 'extra': 10, 'ttl': 345600, 'seed': SEED,
                             'source': 'reference _doSafePoW', 'kats': batch})

    # ---------------- target formula ----------------
    def sw_target(L, ttl, ntpb=1000, extra=1000):
        return 2 ** 64 / (ntpb * (L + 8 + extra + ((ttl * (L + 8 + extra)) / (2 ** 16))))

    def api_target(L, ntpb=1000, extra=1000):
        return 2 ** 64 / ((L + extra + 8) * ntpb)

    tg = []
    for (L, ttl, ntpb, extra) in [(1024, 345600, 1000, 1000), (46, 2419200, 1000, 1000),
                                  (200, 345600, 1000, 1000), (1024, 2419200, 20000, 1000),
                                  (512, 345600, 1000, 1000), (16384, 345600, 1000, 1000),
                                  (0, 300, 1000, 1000), (262144, 2419200, 1000, 1000),
                                  (1024, 3600, 10, 10), (1024, 345600, 20000000, 1000)]:
        tf = sw_target(L, ttl, ntpb, extra)
        tg.append({'kind': 'singleWorker', 'L': L, 'ttl': ttl, 'ntpb': ntpb, 'extra': extra,
                   'target_float': tf.hex(), 'target': int(tf)})
    for (L, ntpb, extra) in [(1024, 1000, 1000), (200, 1000, 1000), (5000, 2000, 3000)]:
        tf = api_target(L, ntpb, extra)
        tg.append({'kind': 'api', 'L': L, 'ntpb': ntpb, 'extra': extra,
                   'target_float': tf.hex(), 'target': int(tf)})
    dump('config_targets.json', {'targets': tg})

    # ---------------- verifier KATs ----------------
    # isProofOfWorkSufficient clamps ntpb/extra up to the network defaults (protocol.py:272-275),
    # so objects are solved at the defaults; the solve uses the C oracle (fast), the verdict is
    # the reference's.
    sys.path.insert(0, os.path.join(HERE, '..', '..'))
    from oracle.oracle import COracle
    co = COracle()
    recv = 1700000000
    ver = []
    vrng = random.Random(SEED + 2)
    for k in range(6):
        ttl = [3600, 345600, 2419200, 300, 100, 86400][k]
        body = pack('>Q', recv + ttl) + b'\x00\x00\x00\x02' + b'\x01\x01' + vrng.randbytes(40 + 30 * k)
        ntpb, extra = 1000, 1000
        L = len(body)
        ttl_eff = max(ttl, 300)
        target = int(2 ** 64 / (ntpb * (L + 8 + extra + ((ttl_eff * (L + 8 + extra)) / (2 ** 16)))))
        ih = hashlib.sha512(body).digest()
        (tv, nonce), _ = co.search_mt(ih, target, 1, 1 << 40, threads=os.cpu_count() or 8)
        obj = pack('>Q', nonce) + body
        ok = protocol.isProofOfWorkSufficient(obj, ntpb, extra, recvTime=recv)
        assert ok
        nxt = protocol.isProofOfWorkSufficient(pack('>Q', nonce + 1) + body, ntpb, extra, recvTime=recv)
        late = protocol.isProofOfWorkSufficient(obj, ntpb, extra, recvTime=recv - 10 ** 6)
        ver.append({'object': hx(obj), 'ntpb': ntpb, 'extra': extra, 'recvTime': recv,
                    'sufficient': ok, 'object_next_nonce_sufficient': nxt,
                    'recvTime_minus_1e6_sufficient': late})
        print('  verifier ttl=%d nonce=%d next=%s late=%s' % (ttl, nonce, nxt, late))
    dump('verifier_kats.json', {'source': 'reference protocol.isProofOfWorkSufficient', 'kats': ver})


def openclpow_vector(proofofwork, ih, target):
    """test_openclpow vector: 224M trials is too slow for _doSafePoW in Python, so the exact
    first nonce comes from the C oracle's exhaustive scan; the reference then confirms it:
    _doSafePoW restarted just below the answer (window of 2^16) must land on it, and the
    reference trial at the answer must satisfy the target."""
    sys.path.insert(0, os.path.join(HERE, '..', '..'))
    from oracle.oracle import COracle
    res, _ = COracle().search_mt(ih, target, 1, 1 << 32, threads=os.cpu_count() or 8)
    tv, nonce = res
    lo = max(1, nonce - (1 << 16))
    # reference restart: replicate _doSafePoW's loop from `lo` using its own trial code
    n = lo - 1
    while True:
        t2, n2 = proofofwork._pool_worker(n, ih, target, 1)
        if n2 == nonce:
            break
        assert n2 < nonce
        n = n2
    assert t2 == tv <= target
    return {'ih': ih.hex(), 'target': target, 'nonce': nonce, 'trial': tv,
            'note': 'src/tests/test_openclpow.py:22-26 vector (SURVEY App.A: 224121278)',
            'source': 'C-oracle exhaustive scan; reference _pool_worker confirms the last 2^16 window'}


def dump(name, obj):
    with open(os.path.join(HERE, name), 'w') as f:
        json.dump(obj, f, indent=1)
    print('wrote', name)


if __name__ == '__main__':
    main()
