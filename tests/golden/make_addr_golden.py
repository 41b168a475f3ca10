#!/usr/bin/env python3
"""Generate tests/golden/addr_kats.json -- address-search fixtures from the REFERENCE's own
primitives (build container only; needs /root/reference, read-only):

    BITMESSAGE_HOME=$(mktemp -d) PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_addr_golden.py

RIPEMD-160 lives in OpenSSL 3's legacy provider, which this image's hashlib does not load by
default (the reference's ``fallback.RIPEMD160Hash`` is then None); the script re-runs itself with
an ``OPENSSL_CONF`` that activates it, so the reference code runs unmodified.

* ``pointmult_kats``: ``highlevelcrypto.pointMult`` (src/highlevelcrypto.py:111-140, OpenSSL
  EC_POINT_mul) for random and edge private keys.
* ``try_kats``: the per-try values of the deterministic loop (class_addressGenerator.py:249-266):
  keys, public keys and ripe at try indices around every varint boundary of 2k / 2k+1.
* ``search_kats``: first k meeting the prefix, and the reference's ``addresses.encodeAddress``
  (v3 and v4) and WIF encoding (class_addressGenerator.py:169-178 via
  ``arithmetic.changebase``), for passphrases exercising the 1- and 2-block SHA-512 tails and the
  midstate path, plus a 3-address run (nonces continue) and a 2-null-byte search.
"""
import hashlib
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = '/root/reference/src'
CNF = '''openssl_conf = openssl_init
[openssl_init]
providers = provider_sect
[provider_sect]
default = default_sect
legacy = legacy_sect
[default_sect]
activate = 1
[legacy_sect]
activate = 1
'''


def main():
    try:
        hashlib.new('ripemd160')
    except ValueError:
        with tempfile.NamedTemporaryFile('w', suffix='.cnf', delete=False) as f:
            f.write(CNF)
        env = dict(os.environ, OPENSSL_CONF=f.name)
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))
    sys.path.insert(0, REF_SRC)
    import highlevelcrypto
    from addresses import encodeAddress, encodeVarint
    from fallback import RIPEMD160Hash
    from pyelliptic import arithmetic

    n_order = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    rng = random.Random(20250216 + 4)
    keys = [1, 2, 3, 255, 256, 2 ** 64 - 1, 2 ** 128 + 7, n_order - 1, n_order + 1, 2 ** 256 - 1]
    keys += [rng.randrange(1, 2 ** 256) for _ in range(40)]
    pm = [{'priv': k.to_bytes(32, 'big').hex(), 'pub': highlevelcrypto.pointMult(k.to_bytes(32, 'big')).hex()}
          for k in keys]
    print('pointMult kats:', len(pm))

    def try_values(pp, k):
        ps = hashlib.sha512(pp + encodeVarint(2 * k)).digest()[:32]
        pe = hashlib.sha512(pp + encodeVarint(2 * k + 1)).digest()[:32]
        pubs, pube = highlevelcrypto.pointMult(ps), highlevelcrypto.pointMult(pe)
        ripe = RIPEMD160Hash(hashlib.sha512(pubs + pube).digest()).digest()
        return ps, pe, pubs, pube, ripe

    def wif(key):
        raw = b'\x80' + key
        return arithmetic.changebase(raw + hashlib.sha256(hashlib.sha256(raw).digest()).digest()[0:4],
                                     256, 58).decode()

    seed = b'TIGER, tiger, burning bright. In the forests of the night'  # src/tests/samples.py:32
    tries = []
    for pp in [seed, b'', b'x' * 118, b'y' * 127, b'z' * 300]:
        for k in [0, 1, 125, 126, 127, 128, 32767, 32768, 2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1, 2 ** 40 + 3]:
            ps, pe, pubs, pube, ripe = try_values(pp, k)
            tries.append({'passphrase': pp.hex(), 'k': k, 'priv_signing': ps.hex(), 'priv_encryption': pe.hex(),
                          'pub_signing': pubs.hex(), 'pub_encryption': pube.hex(), 'ripe': ripe.hex()})
    print('try kats:', len(tries))

    searches = []

    def search(pp, null_bytes, count=1, label=''):
        k = 0
        for idx in range(count):
            while True:
                ps, pe, pubs, pube, ripe = try_values(pp, k)
                if ripe[:null_bytes] == b'\x00' * null_bytes:
                    break
                k += 1
            searches.append({'passphrase': pp.hex(), 'null_bytes': null_bytes, 'index': idx, 'k': k,
                             'ripe': ripe.hex(), 'addr3': encodeAddress(3, 1, ripe),
                             'addr4': encodeAddress(4, 1, ripe), 'addr4_stream2': encodeAddress(4, 2, ripe),
                             'wif_signing': wif(ps), 'wif_encryption': wif(pe), 'label': label})
            print('  search %-24s nb=%d #%d k=%d %s' % (label, null_bytes, idx, k, encodeAddress(4, 1, ripe)))
            k += 1

    search(seed, 1, 1, 'samples.sample_seed')
    search(b'', 1, 1, 'empty')
    search(b'correct horse battery staple', 1, 3, '3 addresses')
    search(b'p' * 111, 1, 1, 'tail fills block 1')
    search(b'q' * 200, 1, 1, 'midstate + tail')
    search('chan ünïcode'.encode('utf-8'), 1, 1, 'utf-8')
    search(b'two null bytes', 2, 1, '2 null bytes')
    with open(os.path.join(HERE, 'addr_kats.json'), 'w') as f:
        json.dump({'source': 'reference highlevelcrypto.pointMult (OpenSSL), fallback.RIPEMD160Hash, '
                             'addresses.encodeAddress/encodeVarint, pyelliptic.arithmetic.changebase',
                   'pointmult_kats': pm, 'try_kats': tries, 'search_kats': searches}, f, indent=1)
    print('wrote addr_kats.json')


if __name__ == '__main__':
    main()
