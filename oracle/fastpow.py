"""TEST INFRASTRUCTURE ONLY -- the reference's ``_doFastPoW`` mechanism restated for bench.py's
``cpu_baseline`` leg (the hashlib + multiprocessing CPU backend).

Restated from ``src/proofofwork.py:88-154``:

* ``Pool(processes=P)``, P = ``cpu_count()`` capped by the ``maxcores`` setting (``:116-126``);
* worker ``i`` (``_pool_worker``, ``:88-97``) runs at idle priority (``os.nice(20)``, ``:70-72``)
  and tests ``i+P, i+2P, ...`` (so nonces ``1..P-1`` of workers ``i >= 1`` come first only by
  accident, and nonce ``0`` is never tested), accepting ``trialValue <= target``;
* the caller polls every 0.2 s and returns the result of the LOWEST-INDEX ready worker, which is
  a valid nonce but not necessarily the minimal one (``:133-154``).

The product never imports this: its answers are the exact ``_doSafePoW`` ones, on the GPU.
"""
import hashlib
import multiprocessing
import os
import time
from struct import pack, unpack


def _pool_worker(nonce, initial_hash, target, pool_size):
    try:
        os.nice(20)
    except OSError:
        pass
    trial = float('inf')
    while trial > target:
        nonce += pool_size
        trial, = unpack('>Q', hashlib.sha512(hashlib.sha512(pack('>Q', nonce) + initial_hash).digest())
                        .digest()[0:8])
    return [trial, nonce]


def fast_pow(target, initial_hash, pool_size):
    """One object the ``_doFastPoW`` way; returns ``(trialValue, nonce)``."""
    pool = multiprocessing.get_context('fork').Pool(processes=pool_size)
    try:
        result = [pool.apply_async(_pool_worker, args=(i, initial_hash, target, pool_size))
                  for i in range(pool_size)]
        while True:
            for r in result:
                if r.ready():
                    tv, nonce = r.get()
                    return tv, nonce
            time.sleep(0.2)
    finally:
        pool.terminate()
        pool.join()
