"""TEST INFRASTRUCTURE ONLY -- the parity oracle for the Bitmessage PoW hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product (``pybitmessage_amd``) never does: its search runs on the
GPU or raises.

Three checkers, all pinned against ``tests/golden/`` (generated from the reference):

* :func:`trial` / :func:`safe_pow` -- pure-Python hashlib restatement of the reference
  (``src/proofofwork.py:95-96,100-111``).  Small cases only (~1 us per trial).
* :class:`COracle` -- ctypes binding of ``oracle/liboracle.so`` (plain-C FIPS 180-4
  restatement, ``bmpow_oracle.c``): trial values, bounded sequential search, exact
  multi-threaded search (the CPU-baseline "port").
* :class:`RefBitmsghash` -- ctypes binding of ``oracle/_ref/bitmsghash.so``: the
  reference's own ``BitmessagePOW`` (``src/bitmsghash/bitmsghash.cpp:127-165``) compiled
  from its source by ``oracle/Makefile``.  Nondeterministic by design,
  so it is used as a rate baseline and for "returns *a* valid nonce" checks only.
"""
import ctypes
import hashlib
import os
from struct import pack, unpack

HERE = os.path.dirname(os.path.abspath(__file__))
U64_MAX = (1 << 64) - 1


def trial(nonce, initial_hash):
    """trialValue for one nonce: ``src/proofofwork.py:106-107``."""
    return unpack('>Q', hashlib.sha512(hashlib.sha512(
        pack('>Q', nonce) + initial_hash).digest()).digest()[0:8])[0]


def safe_pow(target, initial_hash, start=1, max_trials=None):
    """``_doSafePoW`` restated (``src/proofofwork.py:100-111``): first ``n >= start`` with
    ``trial(n) <= target``.  Returns ``[trialValue, nonce]`` or ``None`` when the optional
    budget runs out."""
    nonce = start
    end = None if max_trials is None else start + max_trials
    while end is None or nonce < end:
        tv = trial(nonce, initial_hash)
        if tv <= target:
            return [tv, nonce]
        nonce += 1
    return None


def target_from_formula(payload_len, ttl, ntpb=1000, extra=1000):
    """Sender-side target, float arithmetic as ``class_singleWorker.py:7,222-230``
    (``from __future__ import division``) truncated by ``int()`` in ``proofofwork.py:293``."""
    return int(2 ** 64 / (ntpb * (payload_len + 8 + extra + ((ttl * (payload_len + 8 + extra)) / (2 ** 16)))))


class COracle(object):
    """ctypes view of ``oracle/liboracle.so`` (build with ``make -C oracle``)."""

    def __init__(self, path=None):
        path = path or os.path.join(HERE, 'liboracle.so')
        self.lib = lib = ctypes.CDLL(path)
        u64, p64 = ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)
        lib.bmo_trial.restype = u64
        lib.bmo_trial.argtypes = [ctypes.c_char_p, u64]
        lib.bmo_trials.restype = None
        lib.bmo_trials.argtypes = [ctypes.c_char_p, p64, ctypes.c_size_t, p64]
        lib.bmo_search.restype = ctypes.c_int
        lib.bmo_search.argtypes = [ctypes.c_char_p, u64, u64, u64, p64, p64]
        lib.bmo_search_mt.restype = ctypes.c_int
        lib.bmo_search_mt.argtypes = [ctypes.c_char_p, u64, u64, u64, ctypes.c_int, p64, p64, p64]
        lib.bmo_sha512.restype = None
        lib.bmo_sha512.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        lib.bmo_min_trial.restype = ctypes.c_int
        lib.bmo_min_trial.argtypes = [ctypes.c_char_p, u64, u64, p64, p64]
        lib.bmo_trial_len.restype = u64
        lib.bmo_trial_len.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64]
        lib.bmo_search_len.restype = ctypes.c_int
        lib.bmo_search_len.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u64, u64, u64, p64, p64]

    def sha512(self, data):
        out = ctypes.create_string_buffer(64)
        self.lib.bmo_sha512(data, len(data), out)
        return out.raw

    def trial(self, nonce, ih):
        return self.lib.bmo_trial(ih, nonce)

    def trial_len(self, nonce, ih):
        """trial for an initialHash of any length (the reference hashes it as given)."""
        return self.lib.bmo_trial_len(ih, len(ih), nonce)

    def search_len(self, ih, target, start=1, max_trials=U64_MAX):
        """Sequential exact search for an initialHash of any length; (trialValue, nonce) or None."""
        n, t = ctypes.c_uint64(), ctypes.c_uint64()
        if self.lib.bmo_search_len(ih, len(ih), min(target, U64_MAX), start, max_trials, ctypes.byref(n),
                                   ctypes.byref(t)):
            return t.value, n.value
        return None

    def trials(self, ih, nonces):
        import numpy as np
        nonces = np.ascontiguousarray(nonces, dtype=np.uint64)
        out = np.empty_like(nonces)
        p64 = ctypes.POINTER(ctypes.c_uint64)
        self.lib.bmo_trials(ih, nonces.ctypes.data_as(p64), nonces.size, out.ctypes.data_as(p64))
        return out

    def search(self, ih, target, start=1, max_trials=U64_MAX):
        """Sequential exact search; returns (trialValue, nonce) or None."""
        n, t = ctypes.c_uint64(), ctypes.c_uint64()
        if self.lib.bmo_search(ih, min(target, U64_MAX), start, max_trials, ctypes.byref(n), ctypes.byref(t)):
            return t.value, n.value
        return None

    def search_many(self, jobs, threads=None):
        """``search`` of every (target, ih) in jobs, in order: the same sequential search, the objects
        spread over a pool of threads (ctypes releases the GIL for each call).  Threads default to the
        CPUs this process may use, at most 16 (the GPU box's quota)."""
        from concurrent.futures import ThreadPoolExecutor
        jobs = list(jobs)
        if threads is None:
            threads = max(1, min(16, len(os.sched_getaffinity(0))))
        if threads <= 1 or len(jobs) <= 1:
            return [self.search(ih, t) for t, ih in jobs]
        with ThreadPoolExecutor(threads) as ex:
            return list(ex.map(lambda j: self.search(j[1], j[0]), jobs))

    def min_trial(self, ih, start, count):
        """(min trial over [start, start+count), first nonce reaching it); (U64_MAX, start)
        for an empty range."""
        m, a = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.bmo_min_trial(ih, start, count, ctypes.byref(m), ctypes.byref(a))
        return m.value, a.value

    def search_mt(self, ih, target, start=1, max_trials=U64_MAX, threads=1):
        """Exact multi-threaded search; returns ((trialValue, nonce) | None, trials_performed)."""
        n, t, done = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        hit = self.lib.bmo_search_mt(ih, min(target, U64_MAX), start, max_trials, threads,
                                     ctypes.byref(n), ctypes.byref(t), ctypes.byref(done))
        return ((t.value, n.value) if hit else None), done.value


class RefBitmsghash(object):
    """The reference's ``BitmessagePOW`` built from ``src/bitmsghash/bitmsghash.cpp``."""

    def __init__(self, path=None):
        path = path or os.path.join(HERE, '_ref', 'bitmsghash.so')
        self.lib = ctypes.CDLL(path)
        self.fn = self.lib.BitmessagePOW
        self.fn.restype = ctypes.c_ulonglong  # as src/proofofwork.py:387-388

    def pow(self, target, ih):
        """Mirror of ``_doCPoW`` (``src/proofofwork.py:157-170``) minus LogOutput; blocks until
        some thread finds ``trial < target`` (strict, bitmsghash.cpp:65)."""
        buf = ctypes.pointer(ctypes.create_string_buffer(ih, 64))
        nonce = self.fn(buf, ctypes.c_ulonglong(target))
        return [trial(nonce, ih), nonce]


def have_c_oracle():
    return os.path.exists(os.path.join(HERE, 'liboracle.so'))


def have_ref():
    return os.path.exists(os.path.join(HERE, '_ref', 'bitmsghash.so'))
