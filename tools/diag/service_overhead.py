#!/usr/bin/env python3
"""Fixed cost of a batch through the library's service (what iter_batch pays per call besides the
hashing): bmpow_service_create, submit, the poll that returns the objects, destroy -- timed for a batch
of trivially easy objects (target 2^64 - 1: nonce 1 answers), N times.

    python3 tools/diag/service_overhead.py [N] [objects]
"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    os.environ.setdefault('BMPOW_DEVICES', '0')
    import numpy as np
    from pybitmessage_amd import _lib
    lib = _lib.get()
    p64 = ctypes.POINTER(ctypes.c_uint64)
    ihs = os.urandom(64 * m)
    tg = np.full(m, (1 << 64) - 1, dtype=np.uint64)
    parts = {'create': [], 'submit': [], 'poll': [], 'destroy': [], 'total': []}
    for it in range(n + 3):
        t0 = time.perf_counter()
        s = lib.bmpow_service_create(0, _lib.SERVICE_VERIFY)
        t1 = time.perf_counter()
        tick = np.zeros(m, dtype=np.uint64)
        _lib.check(lib, lib.bmpow_service_submit(s, m, ihs, tg.ctypes.data_as(p64), tick.ctypes.data_as(p64)), 'submit')
        t2 = time.perf_counter()
        got = 0
        nonce, trial = np.zeros(m, dtype=np.uint64), np.zeros(m, dtype=np.uint64)
        done = np.zeros(m, dtype=np.uint8)
        while got < m:
            got += _lib.check(lib, lib.bmpow_service_poll(s, m, 1000, tick.ctypes.data_as(p64), nonce.ctypes.data_as(p64),
                                                          trial.ctypes.data_as(p64),
                                                          done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), 'poll')
        t3 = time.perf_counter()
        lib.bmpow_service_destroy(s)
        t4 = time.perf_counter()
        if it >= 3:
            for k, v in (('create', t1 - t0), ('submit', t2 - t1), ('poll', t3 - t2), ('destroy', t4 - t3), ('total', t4 - t0)):
                parts[k].append(v * 1e3)
    print(json.dumps({'objects': m, 'calls': n, 'median_ms': {k: round(statistics.median(v), 4) for k, v in parts.items()}}))


if __name__ == '__main__':
    main()
