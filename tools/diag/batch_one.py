#!/usr/bin/env python3
"""run_batch of ONE object: run()'s single-object path (proofofwork.BATCH_ONE, the default) against the
continuous-batching service the batch entry points use for more objects.  C1's object (golden nonce
10,909,138), N calls each way, interleaved in blocks of 10; prints the per-call wall times.

    python3 tools/diag/batch_one.py [N]
"""
import hashlib
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    os.environ.setdefault('BMPOW_DEVICES', '0')
    from pybitmessage_amd import proofofwork, targets
    ih = hashlib.sha512(random.Random(20250216).randbytes(1024)).digest()
    t = int(targets.object_target(1024, 345600))
    ms = {True: [], False: []}
    for one in (True, False):  # warm both paths
        proofofwork.BATCH_ONE = one
        assert proofofwork.run_batch([(t, ih)])[0][1] == 10909138
    for block in range(2 * n // 10):
        one = block % 2 == 0
        proofofwork.BATCH_ONE = one
        for _ in range(10):
            t0 = time.perf_counter()
            r = proofofwork.run_batch([(t, ih)])
            ms[one].append((time.perf_counter() - t0) * 1e3)
            assert r[0][1] == 10909138
    out = {}
    for one, name in ((True, 'single_object_path'), (False, 'service')):
        xs = sorted(ms[one])
        out[name] = {'calls': len(xs), 'mean_ms': round(statistics.mean(xs), 4), 'median_ms': round(xs[len(xs) // 2], 4),
                     'ghs': round(10909138 / (statistics.mean(xs) * 1e-3) / 1e9, 4)}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
