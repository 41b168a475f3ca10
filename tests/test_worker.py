"""Batched worker, the openclpow-compatible module and LogOutput.

CPU tests drive the host logic against test doubles of the device layer that answer from the
C oracle (the doubles live here in tests/; the product has no fallback).  GPU tests run the
same flows on the device and compare with the oracle."""
import ctypes
import hashlib
import logging
import random
import struct
import subprocess
import threading
import time
from struct import pack, unpack

import numpy as np
import pytest

from pybitmessage_amd import _lib, hippow, proofofwork, state, targets, worker

U64 = (1 << 64) - 1


# ------------------------------------------------------------------ test doubles
@pytest.fixture
def oracle_batch(monkeypatch, coracle):
    """proofofwork.iter_batch answered by the C oracle (index order, like one big step)."""
    calls = []

    def fake_iter(objects, step_trials=0):
        objs = list(objects)
        calls.append(len(objs))
        for i, (t, ih) in enumerate(objs):
            if state.shutdown:
                raise proofofwork.PowInterrupted('Interrupted')
            tv, nonce = coracle.search(proofofwork._ih_bytes(ih), proofofwork._clamp_target(t)[0])
            yield i, tv, nonce
    monkeypatch.setattr(proofofwork, 'iter_batch', fake_iter)
    yield calls
    state.shutdown = 0


class BatchLib(object):
    """Test double of the resident-session ABI (bmpow_batch_create/add/step/take_done/destroy,
    include/bmpow.h): each step advances every pending object by WINDOW nonces, searched with the
    C oracle; finished slots are queued for take_done and freed for reuse, as the library does.
    The bmpow_service_* calls run the library's stepping thread over those sessions."""
    WINDOW = 3000

    def __init__(self, coracle):
        self.co = coracle
        self.calls = 0
        self.sizes = []
        self.sessions = {}
        self.next_handle = 1
        self.services = []
        self.fail_step = False
        self.bad_tickets = set()
        self.single_calls = 0

    def bmpow_batch_create(self, n, ihs, tg, start):
        h = self.next_handle
        self.next_handle += 1
        self.sessions[h] = {'objs': [], 'queue': [], 'free': []}
        if n:
            assert start is None
            self.bmpow_batch_add(h, n, ihs, tg, None, (ctypes.c_uint32 * n)())
        return h

    def bmpow_batch_add(self, h, n, ihs, tg, start, slot_out):
        assert start is None
        ses = self.sessions[h]
        tg = np.ctypeslib.as_array(ctypes.cast(tg, ctypes.POINTER(ctypes.c_uint64)), shape=(n,))
        slots = np.ctypeslib.as_array(ctypes.cast(slot_out, ctypes.POINTER(ctypes.c_uint32)), shape=(n,))
        for i in range(n):
            o = {'ih': ihs[64 * i:64 * i + 64], 't': int(tg[i]), 'next': 1, 'state': _lib.PENDING}
            if ses['free']:
                k = ses['free'].pop()
                ses['objs'][k] = o
            else:
                k = len(ses['objs'])
                ses['objs'].append(o)
            slots[i] = k
        return sum(o['state'] == _lib.PENDING for o in ses['objs'])

    def bmpow_batch_step(self, h, budget):
        self.calls += 1
        ses = self.sessions[h]
        pend = [k for k, o in enumerate(ses['objs']) if o['state'] == _lib.PENDING]
        self.sizes.append(len(pend))
        for k in pend:
            o = ses['objs'][k]
            r = self.co.search(o['ih'], o['t'], o['next'], self.WINDOW)
            if r is None:
                o['next'] += self.WINDOW
            else:
                o['trial'], o['nonce'] = r
                o['state'] = _lib.DONE_FOUND
                ses['queue'].append(k)
        time.sleep(0.002)
        return sum(o['state'] == _lib.PENDING for o in ses['objs'])

    def bmpow_batch_take_done(self, h, cap, slot_out, nonce_out, trial_out, done_out):
        ses = self.sessions[h]
        view = lambda p, t: np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(t)), shape=(cap,))  # noqa: E731
        slots, nonce = view(slot_out, ctypes.c_uint32), view(nonce_out, ctypes.c_uint64)
        trial, done = view(trial_out, ctypes.c_uint64), view(done_out, ctypes.c_uint8)
        k = 0
        while k < cap and ses['queue']:
            j = ses['queue'].pop(0)
            o = ses['objs'][j]
            slots[k], nonce[k], trial[k], done[k] = j, o['nonce'], o['trial'], o['state']
            o['state'] = _lib.FREE
            ses['free'].append(j)
            k += 1
        return k

    def bmpow_batch_destroy(self, h):
        del self.sessions[h]

    # bmpow_service_*: the library's stepping thread, emulated over the session double above
    def bmpow_service_create(self, budget, flags):
        assert flags == _lib.SERVICE_VERIFY
        svc = {'h': self.bmpow_batch_create(0, None, None, None), 'cv': threading.Condition(), 'in': [],
               'out': [], 'ticket': 0, 'stop': False, 'cancel': False, 'error': 0, 'live': {}}
        svc['th'] = threading.Thread(target=self._service_loop, args=(svc,), daemon=True)
        svc['th'].start()
        self.services.append(svc)
        return len(self.services)

    def _service_loop(self, svc):
        slots = (ctypes.c_uint32 * 64)()
        nonce, trial, done = (ctypes.c_uint64 * 64)(), (ctypes.c_uint64 * 64)(), (ctypes.c_uint8 * 64)()
        while True:
            with svc['cv']:
                svc['cv'].wait_for(lambda: svc['stop'] or svc['cancel'] or svc['in'] or
                                   (svc['live'] and not svc['error']))
                if svc['stop']:
                    return
                if svc['cancel']:
                    self.bmpow_batch_destroy(svc['h'])
                    svc['h'] = self.bmpow_batch_create(0, None, None, None)
                    svc['live'], svc['cancel'] = {}, False
                new, svc['in'] = svc['in'], []
            h = svc['h']
            if new:
                tg = (ctypes.c_uint64 * len(new))(*[t for _, _, t in new])
                sl = (ctypes.c_uint32 * len(new))()
                self.bmpow_batch_add(h, len(new), b''.join(ih for _, ih, _ in new), tg, None, sl)
                for (tk, _, _), k in zip(new, sl):
                    svc['live'][k] = tk
            fin, rc = [], 0
            if not svc['live']:  # the library steps only a non-empty session
                pass
            elif self.fail_step:
                rc = -3
            else:
                self.bmpow_batch_step(h, 0)
                while True:
                    k = self.bmpow_batch_take_done(h, 64, slots, nonce, trial, done)
                    fin += [(svc['live'].pop(slots[j]), nonce[j], trial[j], done[j]) for j in range(k)]
                    if k < 64:
                        break
            with svc['cv']:
                if not svc['cancel']:
                    svc['out'] += fin
                    svc['error'] = rc
                svc['cv'].notify_all()

    def bmpow_service_submit(self, sh, n, ihs, tg, tickets_out):
        svc = self.services[sh - 1]
        tg = np.ctypeslib.as_array(ctypes.cast(tg, ctypes.POINTER(ctypes.c_uint64)), shape=(n,))
        tk = np.ctypeslib.as_array(ctypes.cast(tickets_out, ctypes.POINTER(ctypes.c_uint64)), shape=(n,))
        with svc['cv']:
            for i in range(n):
                tk[i] = svc['ticket']
                svc['in'].append((svc['ticket'], ihs[64 * i:64 * i + 64], int(tg[i])))
                svc['ticket'] += 1
            svc['cv'].notify_all()
        return 0

    def bmpow_service_poll(self, sh, cap, timeout_ms, tickets, nonce_out, trial_out, done_out):
        svc = self.services[sh - 1]
        view = lambda p, t: np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(t)), shape=(cap,))  # noqa: E731
        tk, nonce = view(tickets, ctypes.c_uint64), view(nonce_out, ctypes.c_uint64)
        trial, done = view(trial_out, ctypes.c_uint64), view(done_out, ctypes.c_uint8)
        with svc['cv']:
            if not svc['cv'].wait_for(lambda: svc['out'] or svc['error'] or svc['stop'], timeout_ms / 1000.0):
                return 0
            if not svc['out'] and svc['error']:
                return svc['error']
            k = min(cap, len(svc['out']))
            for j in range(k):
                tk[j], nonce[j], trial[j], done[j] = svc['out'][j]
                if int(tk[j]) in self.bad_tickets:  # the library's host re-check caught a wrong answer
                    done[j] = _lib.DONE_BADHASH
            del svc['out'][:k]
            return k

    def bmpow_service_cancel(self, sh):
        svc = self.services[sh - 1]
        with svc['cv']:
            svc['cancel'], svc['error'], svc['in'], svc['out'] = True, 0, [], []
            svc['cv'].notify_all()
        return 0

    def bmpow_service_stop(self, sh):
        svc = self.services[sh - 1]
        with svc['cv']:
            svc['stop'] = True
            svc['cv'].notify_all()
        svc['th'].join()

    def bmpow_service_destroy(self, sh):
        self.bmpow_service_stop(sh)
        self.bmpow_batch_destroy(self.services[sh - 1]['h'])

    def bmpow_last_error(self):
        return b'injected step failure' if self.fail_step else b''

    def bmpow_search_len(self, ih, ih_len, target, start, max_trials, nonce_out, trial_out):
        """run()'s bounded single-object search (the one-object batch takes it), by the C oracle."""
        self.single_calls += 1
        r = self.co.search(bytes(ih[:ih_len]), target, start, max_trials)
        if r is None:
            return _lib.NOT_FOUND
        trial_out._obj.value, nonce_out._obj.value = r
        return _lib.FOUND


@pytest.fixture
def batchlib(monkeypatch, coracle):
    lib = BatchLib(coracle)
    monkeypatch.setattr(_lib, 'get', lambda: lib)
    yield lib
    state.shutdown = 0


# ------------------------------------------------------------------ CPU: host logic
def test_powobject_matches_singleworker_formula(golden):
    for t in golden('config_targets.json')['targets']:
        if t['kind'] != 'singleWorker':
            continue
        o = worker.PowObject(bytes(t['L']), t['ttl'], t['ntpb'], t['extra'])
        assert o.target.hex() == t['target_float']
        assert o.initial_hash == hashlib.sha512(bytes(t['L'])).digest()


def test_ack_ttl_buckets():
    r = random.Random(1)
    for ttl, bucket in [(3600, 86400), (86399, 86400), (86400, 604800), (604799, 604800),
                        (604800, 2419200), (2419200, 2419200)]:
        v = worker.ack_ttl(ttl, r)
        assert bucket - 300 <= v < bucket + 300


def test_create_packet_layout():
    p = worker.create_packet('object', b'abc')
    magic, cmd, ln, ck = unpack('!L12sL4s', p[:24])
    assert magic == 0xE9BEB4D9 and cmd == b'object' + bytes(6) and ln == 3
    assert ck == hashlib.sha512(b'abc').digest()[:4] and p[24:] == b'abc'


def test_pow_objects_order_and_bytes(oracle_batch, coracle, golden, caplog):
    kats = golden('batch_kats.json')
    rng = random.Random(kats['seed'])
    objs = [worker.PowObject(rng.randbytes(k['L']), kats['ttl'], kats['ntpb'], kats['extra']) for k in kats['kats']]
    seen = []
    with caplog.at_level('INFO', logger='default'):
        out = worker.pow_objects(objs, on_done=lambda i, tv, n: seen.append(i))
    # the batch's line in the log (per-batch rate; here without device statistics)
    assert any(r.getMessage().startswith('PoW batch of %d objects took' % len(objs)) for r in caplog.records)
    assert oracle_batch == [len(objs)]  # one batch for all objects
    for o, k, fin in zip(objs, kats['kats'], out):
        assert o.initial_hash.hex() == k['ih'] and int(o.target) == k['target']
        assert fin == pack('>Q', k['nonce']) + o.payload
    assert sorted(seen) == list(range(len(objs)))


def test_send_msgs_two_phases(oracle_batch):
    """All acks in one batch first, every msg (embedding its ack) in a second batch."""
    rng = random.Random(4)
    jobs = [(rng.randbytes(38), 3600, {'k': k}) if k % 3 else (None, 3600, {'k': k}) for k in range(7)]
    built = []

    def build_msg(ctx, ack):
        built.append((ctx['k'], ack))
        return b'msg%d' % ctx['k'] + ack, 3600, 10, 10
    now = 1700000000
    out = worker.send_msgs(jobs, build_msg, rng=random.Random(9), now=now)
    assert oracle_batch == [4, 7]
    for (k, ack), (ackdata, _, _) in zip(built, jobs):
        if ackdata is None:
            assert ack == b''
        else:
            assert ack[24 + 8 + 8:] == ackdata  # header, nonce, embeddedTime
            body = ack[24:]
            assert targets.pow_value(body) <= int(targets.object_target(len(body) - 8,
                                                                         unpack('>Q', body[8:16])[0] - now))
    for k, o in enumerate(out):
        assert o[8:] == b'msg%d' % k + built[k][1]


def test_pow_objects_interrupted(oracle_batch):
    state.shutdown = 0
    objs = [worker.PowObject(b'x' * 10, 3600, 10, 10)] * 3

    def stop(i, tv, n):
        state.shutdown = 1
    with pytest.raises(StopIteration):
        worker.pow_objects(objs, on_done=stop)


def test_powservice_concurrent_producers(batchlib, coracle):
    svc = worker.PowService().start()
    try:
        rng = random.Random(2)
        jobs = [(U64 // rng.choice([50, 2000, 9000]), rng.randbytes(64)) for _ in range(24)]
        results = {}

        def producer(lo, hi):
            for j in range(lo, hi):
                results[j] = svc.run(*jobs[j])
        ths = [threading.Thread(target=producer, args=(a, a + 6)) for a in range(0, 24, 6)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(60)
        for j, (t, ih) in enumerate(jobs):
            assert results[j] == list(coracle.search(ih, t))
        assert max(batchlib.sizes) > 1  # producers shared device calls
        assert not batchlib.sessions or all(not ses['queue'] for ses in batchlib.sessions.values())
    finally:
        svc.stop(5)


def test_iter_batch_stepping_thread(batchlib, coracle):
    """proofofwork.run_batch / iter_batch over the session ABI (stepping thread + take_done):
    exact answers in input order, objects yielded as they finish, interrupt and early close."""
    rng = random.Random(21)
    objs = [(U64 // rng.choice([3, 400, 7000]), rng.randbytes(64)) for _ in range(60)]
    assert proofofwork.run_batch(objs) == [list(coracle.search(ih, t)) for t, ih in objs]
    seen = [i for i, _, _ in proofofwork.iter_batch(objs)]
    assert sorted(seen) == list(range(len(objs))) and seen != list(range(len(objs)))  # finishing order
    gen = proofofwork.iter_batch(objs)
    next(gen)
    gen.close()  # the stepping thread stops and the session is destroyed
    assert not batchlib.sessions
    hard = [(0, rng.randbytes(64)), (0, rng.randbytes(64))]  # never found (two: the service path)
    timer = threading.Timer(0.2, lambda: setattr(state, 'shutdown', 1))
    timer.start()
    try:
        with pytest.raises(StopIteration):
            proofofwork.run_batch(hard)
    finally:
        timer.join()
        state.shutdown = 0
    assert not batchlib.sessions
    batchlib.bad_tickets = {1}  # a wrong device answer caught by the library's host re-check
    with pytest.raises(_lib.BmpowError, match='object 1: .*re-check'):
        proofofwork.run_batch(objs[:3])
    assert not batchlib.sessions


def test_one_object_batch_takes_the_single_object_path(batchlib, coracle):
    """run_batch / iter_batch / pow_objects of ONE object use run()'s bounded single-object search
    (bmpow_search_len), not a service and a session set up for one object; the answer is the same."""
    rng = random.Random(5)
    t, ih = U64 // 900, rng.randbytes(64)
    assert proofofwork.run_batch([(t, ih)]) == [list(coracle.search(ih, t))]
    assert batchlib.single_calls == 1 and not batchlib.services and not batchlib.sessions
    assert list(proofofwork.iter_batch([(t, ih)])) == [(0,) + tuple(coracle.search(ih, t))]
    with pytest.raises(ValueError):
        list(proofofwork.iter_batch([(-1, ih)]))
    state.shutdown = 1
    try:
        with pytest.raises(RuntimeError):
            proofofwork.run_batch([(t, ih)])
    finally:
        state.shutdown = 0


def test_powservice_submit_many(batchlib, coracle):
    svc = worker.PowService().start()
    try:
        rng = random.Random(12)
        jobs = [(U64 // rng.choice([50, 2000, 9000]), rng.randbytes(64)) for _ in range(40)] + [(-1, bytes(64))]
        futs = svc.submit_many(jobs)
        for (t, ih), f in zip(jobs[:-1], futs[:-1]):
            assert f.result(60) == list(coracle.search(ih, t))
        with pytest.raises(ValueError):
            futs[-1].result(1)
        assert svc.solved == 40
    finally:
        svc.stop(5)


def test_powservice_shutdown_and_errors(batchlib, coracle):
    svc = worker.PowService().start()
    try:
        fut = svc.submit(0, bytes(64))  # target 0: never found
        time.sleep(0.05)
        state.shutdown = 1
        with pytest.raises(StopIteration):
            fut.result(10)
        state.shutdown = 0
        with pytest.raises(ValueError):
            svc.submit(-1, bytes(64)).result(1)
        # a failing step fails what is live with the library's error; the service then recovers
        batchlib.fail_step = True
        with pytest.raises(_lib.BmpowError, match='injected'):
            svc.submit(U64 // 10, bytes(64)).result(10)
        batchlib.fail_step = False
        batchlib.bad_tickets = {2}  # the service's third ticket: a wrong device answer
        with pytest.raises(_lib.BmpowError, match='re-check'):
            svc.submit(U64 // 10, bytes(64)).result(10)
        # a wrong answer disables the backend (_doGPUPoW, src/proofofwork.py:176-190) until resetPoW
        assert proofofwork.getPowType() == 'none'
        with pytest.raises(_lib.BmpowUnavailable, match='disabled'):
            svc.submit(U64 // 10, bytes(64)).result(10)
        proofofwork._disabled = None  # what resetPoW() does besides re-selecting the devices
        ih = bytes(range(64))
        assert svc.submit(U64 // 10, ih).result(10) == list(coracle.search(ih, U64 // 10))
        pending = svc.submit(0, bytes(64))
    finally:
        state.shutdown = 0
        svc.stop(5)
    with pytest.raises(RuntimeError, match='stopped'):
        pending.result(1)
    with pytest.raises(RuntimeError):
        svc.submit(1, bytes(64))
    assert not batchlib.sessions  # the service's session was destroyed


def test_logoutput_captures_native_stdout(caplog):
    """Mirror of the reference's src/tests/test_log.py:13-21."""
    with caplog.at_level(logging.INFO, logger='default'):
        with proofofwork.LogOutput():
            subprocess.call(['echo', 'HELLO'])
    assert any('PoW: HELLO' in r.getMessage() for r in caplog.records)


def test_hippow_without_device(monkeypatch):
    def unavailable():
        raise _lib.BmpowUnavailable(_lib.E_NODEV, 'no device')
    monkeypatch.setattr(_lib, 'get', unavailable)
    hippow.initCL()
    assert not hippow.openclAvailable() and not hippow.openclEnabled()
    assert hippow.do_opencl_pow('00' * 64, 2 ** 60) == 0  # reference: 0 when no GPU is enabled


def test_hippow_negative_target_never_searches(monkeypatch):
    """A negative target is unsatisfiable: do_opencl_pow must not wrap it into a u64 (which would
    accept nonce 1) -- it raises ValueError at once and never calls the search (the reference's
    numpy packing raises or wraps; it never blocks)."""
    calls = []

    class Lib(object):
        def bmpow_search_len(self, *a):
            calls.append(a)
            return _lib.FOUND
    monkeypatch.setattr(_lib, 'get', lambda: Lib())
    monkeypatch.setattr(hippow, 'enabledGpus', [0])
    with pytest.raises(ValueError, match='negative target'):
        hippow.do_opencl_pow('00' * 64, -5)
    assert calls == []


# ------------------------------------------------------------------ GPU
gpu = pytest.mark.gpu


@gpu
def test_gpu_pow_objects_vs_oracle(gpulib, coracle, golden):
    kats = golden('batch_kats.json')
    rng = random.Random(kats['seed'])
    objs = [worker.PowObject(rng.randbytes(k['L']), kats['ttl'], kats['ntpb'], kats['extra']) for k in kats['kats']]
    out = worker.pow_objects(objs)
    assert out == [pack('>Q', k['nonce']) + o.payload for o, k in zip(objs, kats['kats'])]


@gpu
def test_gpu_send_msgs_and_verify(gpulib):
    """Two-phase send on the GPU; every finished ack and msg passes the receive-side check."""
    from pybitmessage_amd import verify
    rng = random.Random(12)
    now = int(time.time())
    jobs = [(rng.randbytes(38), 3600, k) for k in range(6)]

    def build_msg(k, ack):
        payload = pack('>Q', now + 3600) + b'\x00\x00\x00\x02\x01\x01' + rng.randbytes(50) + ack
        return payload, 3600, 1000, 1000
    msgs = worker.send_msgs(jobs, build_msg, rng=random.Random(3), now=now)
    acks = [m[8 + 8 + 6 + 50:] for m in msgs]
    assert all(a[:4] == pack('!L', worker.MAGIC) for a in acks)
    assert verify.isProofOfWorkSufficient_batch(msgs, recvTime=now) == [True] * 6
    assert verify.isProofOfWorkSufficient_batch([a[24:] for a in acks], recvTime=now) == [True] * 6


@gpu
def test_gpu_powservice(gpulib, coracle):
    svc = worker.PowService().start()
    try:
        rng = random.Random(21)
        jobs = [(U64 // rng.choice([100, 30000, 300000]), rng.randbytes(64)) for _ in range(40)]
        futs = []
        for t, ih in jobs:
            futs.append(svc.submit(t, ih))
            time.sleep(rng.random() * 0.01)  # arrivals while earlier objects are in flight
        for f, (t, ih) in zip(futs, jobs):
            assert f.result(120) == list(coracle.search(ih, t))
    finally:
        svc.stop(10)


@gpu
def test_gpu_hippow_openclpow_vector(gpulib, golden):
    """src/tests/test_openclpow.py:22-31 through the openclpow-compatible module, with the
    exact-answer assertion the reference test lacks."""
    hippow.initCL()
    assert hippow.openclAvailable() and hippow.openclEnabled()
    k = [k for k in golden('first_nonce_kats.json')['kats'] if '224121278' in k['note']][0]
    nonce = hippow.do_opencl_pow(k['ih'], k['target'])
    assert nonce == k['nonce'] == 224121278
    ih = bytes.fromhex(k['ih'])
    tv, = unpack('>Q', hashlib.sha512(hashlib.sha512(pack('>Q', nonce) + ih).digest()).digest()[0:8])
    assert (nonce - tv) < k['target'] and tv <= k['target']
    hippow.initCL('NVIDIA Corporation')  # another vendor selected: present but not enabled
    assert hippow.openclAvailable() and not hippow.openclEnabled()
    assert hippow.do_opencl_pow(k['ih'], k['target']) == 0
    hippow.initCL()


@gpu
def test_gpu_hippow_shutdown(gpulib):
    hippow.initCL()
    t = threading.Timer(0.3, lambda: setattr(state, 'shutdown', 1))
    t.start()
    try:
        with pytest.raises(Exception, match='Interrupted'):
            hippow.do_opencl_pow('00' * 64, 0)
    finally:
        state.shutdown = 0


@gpu
def test_gpu_batch_and_service_shutdown(gpulib, coracle):
    """state.shutdown interrupts run_batch and PowService on the device within a poll interval plus a
    step (the dev/powinterrupttest.py pattern), and both work again once it is cleared."""
    hard = [(0, bytes(64)), (U64 // 1000, hashlib.sha512(b'a').digest())]  # target 0: never found
    t = threading.Timer(0.3, lambda: setattr(state, 'shutdown', 1))
    t.start()
    t0 = time.time()
    try:
        with pytest.raises(StopIteration, match='Interrupted'):
            proofofwork.run_batch(hard)
        # bound: the caller's poll interval plus the step in flight (two engine launches, ~160 ms) after
        # the 0.3 s timer: under 1 s; 5 s leaves 5x
        assert time.time() - t0 < 5
    finally:
        t.join()
        state.shutdown = 0
    svc = worker.PowService().start()
    try:
        f = svc.submit(0, bytes(64))
        time.sleep(0.2)
        state.shutdown = 1
        t0 = time.time()
        with pytest.raises(StopIteration, match='Interrupted'):
            f.result(10)
        assert time.time() - t0 < 5  # the same bound: a poll interval plus a step
        state.shutdown = 0
        ih = hashlib.sha512(b'after').digest()
        assert svc.submit(U64 // 5000, ih).result(30) == list(coracle.search(ih, U64 // 5000))
    finally:
        state.shutdown = 0
        svc.stop(10)
    assert proofofwork.run_batch(hard[1:]) == [list(coracle.search(hard[1][1], hard[1][0]))]


# ------------------------------------------------------------------ every singleWorker object kind
def _mixed_objects(rng, ntpb=None, extra=None, now=1700000000):
    from pybitmessage_amd import worker as w
    pub_s, pub_e = b'\x04' + rng.randbytes(64), b'\x04' + rng.randbytes(64)
    sig = rng.randbytes(71)
    objs = [
        ('pubkey v2', w.pubkey_object(2, 1, w.pubkey_v2_body(pub_s, pub_e), rng, now, ntpb, extra)),
        ('pubkey v3', w.pubkey_object(3, 1, w.pubkey_v3_body(pub_s, pub_e, 1000, 1000, sig), rng, now, ntpb, extra)),
        ('pubkey v4', w.pubkey_object(4, 1, rng.randbytes(32) + rng.randbytes(300), rng, now, ntpb, extra)),
        ('onionpeer v3', w.onionpeer_object('a' * 56 + '.onion', 8444, rng, now, ntpb, extra)),
        ('onionpeer v2', w.onionpeer_object('b' * 16 + '.onion', 8444, rng, now, ntpb, extra)),
        ('broadcast v4', w.broadcast_object(3, 1, rng.randbytes(400), 4 * 24 * 3600, b'', rng, now, ntpb, extra)),
        ('broadcast v5', w.broadcast_object(4, 1, rng.randbytes(900), 60, rng.randbytes(32), rng, now, ntpb, extra)),
        ('getpubkey v3', w.getpubkey_object(3, 1, rng.randbytes(20), 0, rng, now, ntpb, extra)),
        ('getpubkey v4 retry 5', w.getpubkey_object(4, 1, rng.randbytes(32), 5, rng, now, ntpb, extra)),
        ('msg to v4', w.msg_object(rng.randbytes(700), 4, 1, w.msg_ttl(4 * 24 * 3600, 0, rng),
                                   *((2000, 1500) if ntpb is None else (20, 15)), rng=rng, now=now,
                                   default_ntpb=ntpb, default_extra=extra)),
        ('ack', w.ack_object(rng.randbytes(32), 4 * 24 * 3600, rng, now)),
    ]
    if ntpb is not None:  # the ack builder always uses the network default: give it the same one
        objs[-1] = ('ack', w.PowObject(objs[-1][1].payload, objs[-1][1].ttl, ntpb, extra))
    return objs


def test_object_builders_follow_the_reference_layout():
    """TTL rules and unencrypted headers of class_singleWorker.py:252-715, 1375-1493."""
    from pybitmessage_amd import worker as w
    rng = random.Random(1)
    now = 1700000000
    for _ in range(50):
        assert 28 * 86400 - 300 <= w.pubkey_ttl(rng) < 28 * 86400 + 300
        assert 7 * 86400 - 300 <= w.onionpeer_ttl(rng) < 7 * 86400 + 300
        assert 3600 - 300 <= w.broadcast_ttl(10, rng) < 3600 + 300
        assert 28 * 86400 - 300 <= w.broadcast_ttl(10 ** 9, rng) < 28 * 86400 + 300
        t = w.getpubkey_ttl(2, rng)
        assert isinstance(t, float) and 10 * 86400 - 300 <= t < 10 * 86400 + 300
        assert 28 * 86400 - 300 <= w.getpubkey_ttl(7, rng) < 28 * 86400 + 300
        assert 28 * 86400 - 300 <= w.msg_ttl(4 * 86400, 3, rng) < 28 * 86400 + 300
    assert w.msg_difficulty(2, 5000, 5000) == (1000, 1000)      # v2: network defaults
    assert w.msg_difficulty(4, 10, 20) == (1000, 1000)          # v3+: at least the defaults
    assert w.msg_difficulty(4, 3000, 1500) == (3000, 1500)
    objs = dict(_mixed_objects(random.Random(2), now=now))
    for name, o in objs.items():
        expires = struct.unpack('>Q', o.payload[:8])[0]
        assert expires == int(now + o.ttl), name
        assert o.target == targets.object_target(len(o.payload), o.ttl, o.ntpb, o.extra)
    assert objs['pubkey v2'].payload[8:12] == b'\x00\x00\x00\x01' and objs['pubkey v2'].payload[12:14] == b'\x02\x01'
    assert len(objs['pubkey v2'].payload) == 8 + 4 + 2 + 4 + 128
    assert objs['onionpeer v3'].payload[8:12] == struct.pack('>I', 0x746f72)
    assert objs['onionpeer v3'].payload[12:14] == b'\x03\x01' and objs['onionpeer v2'].payload[12:14] == b'\x02\x01'
    assert objs['onionpeer v3'].payload[14:17] == b'\xfd\x20\xfc'  # varint(8444)
    assert objs['broadcast v4'].payload[8:14] == b'\x00\x00\x00\x03\x04\x01'
    assert objs['broadcast v5'].payload[8:14] == b'\x00\x00\x00\x03\x05\x01'
    assert objs['getpubkey v3'].payload[8:14] == b'\x00\x00\x00\x00\x03\x01'
    assert objs['msg to v4'].payload[8:14] == b'\x00\x00\x00\x02\x01\x01'
    assert (objs['msg to v4'].ntpb, objs['msg to v4'].extra) == (2000, 1500)
    assert w.encode_host('127.0.0.1') == b'\x00' * 10 + b'\xff\xff\x7f\x00\x00\x01'


def test_mixed_kinds_in_one_batch_cpu(oracle_batch, coracle):
    """Every object kind in one pow_objects batch (test-mode difficulty), each answer the
    sequential _doSafePoW nonce."""
    objs = [o for _, o in _mixed_objects(random.Random(3), ntpb=10, extra=10)]
    done = worker.pow_objects(objs)
    for o, d in zip(objs, done):
        nonce = struct.unpack('>Q', d[:8])[0]
        assert d[8:] == o.payload
        assert coracle.search(o.initial_hash, int(o.target))[1] == nonce


@pytest.mark.gpu
def test_gpu_mixed_kinds_in_one_batch(gpulib, coracle):
    """Every singleWorker object kind (pubkey v2/v3/v4, onionpeer, broadcast v4/v5, getpubkey,
    msg, ack) in one device batch at test-mode difficulty, vs the C oracle."""
    rng = random.Random(4)
    objs = []
    for _ in range(20):
        objs += [o for _, o in _mixed_objects(rng, ntpb=10, extra=10)]
    done = worker.pow_objects(objs)
    for o, d in zip(objs, done):
        assert d[8:] == o.payload
        assert (coracle.trial(struct.unpack('>Q', d[:8])[0], o.initial_hash), struct.unpack('>Q', d[:8])[0]) == \
            coracle.search(o.initial_hash, int(o.target))
