#!/usr/bin/env python3
"""Generate tests/golden/len_kats.json by running the REFERENCE itself: the proof of work for
initialHash values that are NOT 64 bytes long.

Run in the build container only (needs /root/reference, read-only):

    BITMESSAGE_HOME=$(mktemp -d) PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_len_golden.py

The reference's ``_doSafePoW`` (src/proofofwork.py:100-111) hashes ``pack('>Q', nonce) +
initialHash`` as given, whatever its length; every caller passes a 64-byte sha512 digest, but
``run`` accepts any bytes.  The lengths cover every SHA-512 block edge of the first hash's
message (8 + L bytes + 17 bytes of padding): one block up to L = 103, two from 104 to 231, three
from 232; plus L = 0 (the nonce alone) and the 64-byte layout's neighbours 63 and 65.

* ``trial``: trial(n, ih) from the reference's ``_pool_worker(n - 1, ih, 2**64, 1)``
  (src/proofofwork.py:90-97), whose first iteration hashes nonce ``n`` and always accepts;
* ``first``: [trialValue, nonce] from the reference's ``_doSafePoW`` at two difficulties.
"""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = '/root/reference/src'
U64 = 1 << 64
LENGTHS = [0, 1, 8, 32, 63, 65, 100, 103, 104, 111, 112, 127, 128, 200, 231, 232, 255, 256, 500, 1000]


def main():
    sys.path.insert(0, REF_SRC)
    import proofofwork  # reference module (do NOT call proofofwork.init(): it runs make in the ref tree)

    rng = random.Random(20250216 + 7)
    trials, first = [], []
    for L in LENGTHS:
        ih = rng.randbytes(L)
        for n in [1, 2, 255, 1 << 32, (1 << 63) + 5, U64 - 1]:
            tv, nn = proofofwork._pool_worker(n - 1, ih, U64, 1)
            assert nn == n
            trials.append({'len': L, 'ih': ih.hex(), 'nonce': n, 'trial': tv})
        for e in (3000, 40000):
            t0 = time.time()
            tv, nonce = proofofwork._doSafePoW(U64 // e, ih)
            first.append({'len': L, 'ih': ih.hex(), 'target': U64 // e, 'nonce': nonce, 'trial': tv})
            print('  L=%-5d E=%-6d nonce=%-7d (%.1fs)' % (L, e, nonce, time.time() - t0))
    out = {'source': 'reference proofofwork._pool_worker / _doSafePoW (src/proofofwork.py:90-111)',
           'lengths': LENGTHS, 'trial': trials, 'first': first}
    with open(os.path.join(HERE, 'len_kats.json'), 'w') as f:
        json.dump(out, f, indent=1)
        f.write('\n')
    print('wrote len_kats.json: %d trial, %d first-nonce KATs' % (len(trials), len(first)))


if __name__ == '__main__':
    main()
