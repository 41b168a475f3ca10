"""Batched proof-of-work worker -- the PoW half of the reference's ``class_singleWorker``
(SURVEY.md 8(f) row 1).

The reference worker is strictly serial: every outgoing object (msg, broadcast, pubkey v2/3/4,
getpubkey, onionpeer, ack) goes through ``_doPOWDefaults`` (``class_singleWorker.py:219-250``)
or the msg-specific block (``:1256-1290``), one ``proofofwork.run`` at a time, and each msg
nests its ack's PoW inside its own assembly (``:1220`` -> ``generateFullAckMessage``
``:1495-1519``).  Here the same per-object unit -- target formula, ``initialHash =
sha512(payload)``, ``pack('>Q', nonce) + payload`` -- runs as batches on the GPU:

* :func:`pow_objects` -- many objects, one device batch (``proofofwork.iter_batch``);
* :func:`full_ack_messages` / :func:`send_msgs` -- the ack-then-msg dependency as two batched
  phases: every ack first, then every msg that embeds one;
* :class:`PowService` -- one long-lived device batch fed by several producer threads (the
  singleWorker thread and the API thread both call ``run``, ``api.py:1304,1350``).

Every nonce is the ``_doSafePoW`` answer, so the finished objects are byte-identical to the
serial worker's.  There is no CPU fallback (see ``proofofwork``).
"""
import ctypes
import hashlib
import logging
import random
import struct
import threading
import time
from concurrent.futures import Future
from struct import pack

from . import _lib
from . import proofofwork
from . import state
from . import targets

logger = logging.getLogger('default')
_P64 = ctypes.POINTER(ctypes.c_uint64)

#: ``protocol.Header`` (``protocol.py:63``) and the network magic (``:298``)
_HEADER = struct.Struct('!L12sL4s')
MAGIC = 0xE9BEB4D9
#: object type numbers (``protocol.py`` OBJECT_*; ``class_singleWorker.py:1305``)
OBJECT_GETPUBKEY, OBJECT_PUBKEY, OBJECT_MSG, OBJECT_BROADCAST = 0, 1, 2, 3
#: the largest object the worker may send (``class_singleWorker.py:1296``)
MAX_OBJECT_SIZE = 2 ** 18


class PowObject(object):
    """One object awaiting PoW: the unit of ``_doPOWDefaults`` (``:219-250``) or of the msg
    block (``:1256-1276``, recipient-specific ``ntpb``/``extra``)."""

    __slots__ = ('payload', 'ttl', 'ntpb', 'extra', 'tag')

    def __init__(self, payload, ttl, ntpb=targets.networkDefaultProofOfWorkNonceTrialsPerByte,
                 extra=targets.networkDefaultPayloadLengthExtraBytes, tag=None):
        self.payload = bytes(payload)
        self.ttl = ttl
        self.ntpb = ntpb
        self.extra = extra
        self.tag = tag

    @property
    def target(self):
        """The float the reference passes to ``run`` (``:222-230``, ``:1256-1264``)."""
        return targets.object_target(len(self.payload), self.ttl, self.ntpb, self.extra)

    @property
    def initial_hash(self):
        """``hashlib.sha512(payload).digest()`` (``:231``, ``:1275``)."""
        return hashlib.sha512(self.payload).digest()


def pow_objects(objects, step_trials=0, on_done=None):
    """PoW every object in one device batch.  Returns ``pack('>Q', nonce) + payload`` per
    object, in input order (``:249``, ``:1290``).  ``on_done(index, trialValue, nonce)`` is
    called as each object finishes (the reference logs "Found proof of work" there,
    ``:237-240``).  Raises ``StopIteration("Interrupted")`` on ``state.shutdown``."""
    objs = list(objects)
    if not objs:
        return []
    if state.shutdown != 0:
        raise RuntimeError('No active exception to reraise')  # run()'s bare raise, proofofwork.py:291-292
    out = [None] * len(objs)
    t0 = time.time()
    trials0 = _trials_hashed()
    try:
        for i, tv, nonce in proofofwork.iter_batch([(o.target, o.initial_hash) for o in objs], step_trials):
            out[i] = pack('>Q', nonce) + objs[i].payload
            logger.info('Found proof of work %s Nonce: %s (object %d of %d, %.1f s into the batch)',
                        tv, nonce, i + 1, len(objs), time.time() - t0)
            if on_done is not None:
                on_done(i, tv, nonce)
    except proofofwork.PowInterrupted:
        raise StopIteration('Interrupted')
    trials1 = _trials_hashed()
    _log_batch(len(objs), time.time() - t0, None if trials0 is None or trials1 is None else trials1 - trials0)
    return out


def _trials_hashed():
    """Trials the library's kernels have hashed so far (every device; bmpow_get_stats), or None
    when no statistics are available (a test double of the library)."""
    try:
        lib = _lib.get()
        st = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(st))
        return st.trials
    except (_lib.BmpowError, AttributeError):
        return None


def _log_batch(n, seconds, trials):
    """The batch's line in the reference's log (``_doPOWDefaults`` logs "PoW took %.1f seconds, speed
    %s", ``class_singleWorker.py:234-246``, with nonce / time as the rate): here the trials the
    devices actually hashed, objects/s and the device count."""
    seconds = max(seconds, 1e-9)
    if trials is None:
        logger.info('PoW batch of %d objects took %.1f seconds, %.1f objects/s', n, seconds, n / seconds)
        return
    logger.info('PoW batch of %d objects took %.1f seconds, speed %.3f GH/s (%d trials hashed), '
                '%.1f objects/s on %d device shard(s)', n, seconds, trials / seconds / 1e9, trials,
                n / seconds, proofofwork._device_count())


def pow_payload(payload, ttl, step_trials=0):
    """``_doPOWDefaults(payload, TTL)`` (``:219-250``) for one object through the batch path."""
    return pow_objects([PowObject(payload, ttl)], step_trials)[0]


# ------------------------------------------------------------------------------------------
# acks (generateFullAckMessage, :1495-1519) and packets (protocol.CreatePacket, :292-300)
# ------------------------------------------------------------------------------------------
def ack_ttl(ttl, rng=random):
    """TTL bucket of an ack (``:1503-1510``): 1 day, 1 week or 4 weeks, whichever the msg TTL
    is closest below, plus uniform jitter in [-300, 300)."""
    if ttl < 24 * 60 * 60:
        ttl = 24 * 60 * 60
    elif ttl < 7 * 24 * 60 * 60:
        ttl = 7 * 24 * 60 * 60
    else:
        ttl = 28 * 24 * 60 * 60
    return int(ttl + rng.randrange(-300, 300))


def ack_object(ackdata, ttl, rng=random, now=None):
    """The ack's PoW object: ``pack('>Q', embeddedTime) + ackdata`` with the bucketed TTL
    (``:1510-1517``)."""
    ttl = ack_ttl(ttl, rng)
    embedded = int((time.time() if now is None else now) + ttl)
    return PowObject(pack('>Q', embedded) + bytes(ackdata), ttl)


def create_packet(command, payload=b''):
    """``protocol.CreatePacket`` (``protocol.py:292-300``): 24-byte header (magic, command
    NUL-padded to 12 bytes, length, first 4 bytes of sha512(payload)) + payload."""
    if isinstance(command, str):
        command = command.encode('ascii')
    return _HEADER.pack(MAGIC, command, len(payload), hashlib.sha512(payload).digest()[0:4]) + payload


def inventory_hash(obj):
    """``addresses.calculateInventoryHash``: first 32 bytes of sha512(sha512(object))."""
    return hashlib.sha512(hashlib.sha512(obj).digest()).digest()[0:32]


def full_ack_messages(acks, rng=random, now=None, step_trials=0):
    """Phase 1 of a batched send: ``generateFullAckMessage`` for every ``(ackdata, msgTTL)``
    at once.  Returns the finished ``object`` packets in input order."""
    objs = [ack_object(ackdata, ttl, rng, now) for ackdata, ttl in acks]
    return [create_packet('object', o) for o in pow_objects(objs, step_trials)]


def send_msgs(jobs, build_msg, rng=random, now=None, step_trials=0):
    """Batched ``sendMsg`` PoW (``:717-1373``) in two phases.

    ``jobs``: ``[(ackdata_or_None, ttl, ctx), ...]``.  Phase 1 PoWs every ack
    (``ackdata`` None = no ack, ``fullAckPayload = ''``, ``:1203-1215``).  Then
    ``build_msg(ctx, fullAckPayload) -> (encryptedPayload, ttl, ntpb, extra)`` assembles,
    signs and encrypts each msg (out of scope here, ``:1222-1255``) and phase 2 PoWs every msg
    at the recipient's difficulty.  Returns the finished msg objects (nonce || payload) in
    job order; objects above 256 KiB are returned as None, as the worker drops them
    (``:1296-1302``)."""
    jobs = list(jobs)
    want_ack = [k for k, (ackdata, _, _) in enumerate(jobs) if ackdata is not None]
    packets = full_ack_messages([(jobs[k][0], jobs[k][1]) for k in want_ack], rng, now, step_trials)
    ack_of = dict(zip(want_ack, packets))
    msgs = []
    for k, (_, _, ctx) in enumerate(jobs):
        payload, ttl, ntpb, extra = build_msg(ctx, ack_of.get(k, b''))
        msgs.append(PowObject(payload, ttl, ntpb, extra, tag=k))
    done = pow_objects(msgs, step_trials)
    return [o if len(o) <= MAX_OBJECT_SIZE else None for o in done]


# ------------------------------------------------------------------------------------------
# every other object kind the worker PoWs (class_singleWorker.py:252-715, 1375-1493): the
# TTL rules and the unencrypted object header are the PoW-relevant part; signatures and the
# ECIES encryption are produced by the caller (out of scope) and passed in
# as bytes.  Each builder returns a PowObject whose target is the reference's
# (_doPOWDefaults, :219-231) at the given difficulty (network default, or the test-mode /
# extralowdifficulty ÷100 of bitmessagemain.py:167-172 when ntpb/extra are passed).
# ------------------------------------------------------------------------------------------
#: ``protocol.OBJECT_ONIONPEER`` (``protocol.py:54``) and ``BITFIELD_DOESACK`` (``:42``)
OBJECT_ONIONPEER = 0x746f72
BITFIELD_DOESACK = 1
_DAY = 24 * 60 * 60


def _varint(i):
    from .addressgen import encodeVarint
    return encodeVarint(i)


def _embedded(ttl, now):
    return int((time.time() if now is None else now) + ttl)


def _defaults(ntpb, extra):
    return (targets.networkDefaultProofOfWorkNonceTrialsPerByte if ntpb is None else ntpb,
            targets.networkDefaultPayloadLengthExtraBytes if extra is None else extra)


def pubkey_ttl(rng=random):
    """28 days +- 5 minutes (``doPOWForMyV2Pubkey`` / ``sendOutOrStoreMyV3Pubkey`` /
    ``sendOutOrStoreMyV4Pubkey``, ``:262``, ``:331``, ``:410``)."""
    return int(28 * _DAY + rng.randrange(-300, 300))


def get_bitfield(does_ack=True):
    """``protocol.getBitfield`` (``protocol.py:70-77``)."""
    return pack('>I', BITFIELD_DOESACK if does_ack else 0)


def pubkey_object(address_version, stream, body, rng=random, now=None, ntpb=None, extra=None, tag=None):
    """A pubkey object (type 1) around ``body``: for v2 the bitfield and the two 64-byte public
    keys (``:264-292``); for v3 those plus varint ntpb, varint extra, varint len(signature) and
    the signature (``:342-378``); for v4 the 32-byte tag then the encrypted blob (``:420-465``).
    ``pubkey_v2_body`` / ``pubkey_v3_body`` assemble the first two."""
    ttl = pubkey_ttl(rng)
    payload = pack('>Q', _embedded(ttl, now)) + b'\x00\x00\x00\x01'
    payload += _varint(address_version) + _varint(stream) + bytes(body)
    n, e = _defaults(ntpb, extra)
    return PowObject(payload, ttl, n, e, tag=tag)


def pubkey_v2_body(pub_signing, pub_encryption, does_ack=True):
    """Bitfield + the keys without their 0x04 prefix (``:269``, ``:287-289``)."""
    return get_bitfield(does_ack) + bytes(pub_signing)[-64:] + bytes(pub_encryption)[-64:]


def pubkey_v3_body(pub_signing, pub_encryption, ntpb, extra, signature, does_ack=True):
    """v2 body + the address's own difficulty + the length-prefixed signature (``:363-378``)."""
    return (pubkey_v2_body(pub_signing, pub_encryption, does_ack) + _varint(ntpb) + _varint(extra)
            + _varint(len(signature)) + bytes(signature))


def onionpeer_ttl(rng=random):
    """7 days +- 5 minutes (``sendOnionPeerObj``, ``:503``)."""
    return int(7 * _DAY + rng.randrange(-300, 300))


def encode_host(host):
    """``protocol.encodeHost`` (``protocol.py:102-110``)."""
    import base64
    import socket
    if host.endswith('.onion'):
        return b'\xfd\x87\xd8\x7e\xeb\x43' + base64.b32decode(host.split('.')[0], True)
    if host.find(':') == -1:
        return b'\x00' * 10 + b'\xff\xff' + socket.inet_aton(host)
    return socket.inet_pton(socket.AF_INET6, host)


def onionpeer_object(host, port, rng=random, now=None, ntpb=None, extra=None):
    """The onionpeer object (``:494-530``): object type 0x746f72, version 2 for a 22-character
    (v2) onion host else 3, stream 1, varint(port) + encodeHost(host)."""
    ttl = onionpeer_ttl(rng)
    payload = pack('>Q', _embedded(ttl, now)) + pack('>I', OBJECT_ONIONPEER)
    payload += _varint(2 if len(host) == 22 else 3) + _varint(1) + _varint(port) + encode_host(host)
    n, e = _defaults(ntpb, extra)
    return PowObject(payload, ttl, n, e)


def broadcast_ttl(ttl, rng=random):
    """The broadcast's TTL clamped to [1 hour, 28 days] +- 5 minutes (``sendBroadcast``,
    ``:599-604``)."""
    if ttl > 28 * _DAY:
        ttl = 28 * _DAY
    if ttl < 60 * 60:
        ttl = 60 * 60
    return int(ttl + rng.randrange(-300, 300))


def broadcast_object(address_version, stream, encrypted, ttl, tag=b'', rng=random, now=None, ntpb=None,
                     extra=None):
    """A broadcast object (type 3, ``:605-675``): broadcast version 4 for address version <= 3
    (no tag), 5 with the 32-byte tag otherwise, stream, tag, then the encrypted body."""
    ttl = broadcast_ttl(ttl, rng)
    payload = pack('>Q', _embedded(ttl, now)) + b'\x00\x00\x00\x03'
    payload += _varint(4 if address_version <= 3 else 5) + _varint(stream)
    if address_version >= 4:
        payload += bytes(tag)
    payload += bytes(encrypted)
    n, e = _defaults(ntpb, extra)
    return PowObject(payload, ttl, n, e)


def getpubkey_ttl(retry_number, rng=random):
    """2.5 days x 2^retryNumber, capped at 28 days, +- 5 minutes -- a float, as the reference
    leaves it (``requestPubKey``, ``:1429-1434``)."""
    ttl = 2.5 * _DAY
    ttl *= 2 ** retry_number
    if ttl > 28 * _DAY:
        ttl = 28 * _DAY
    return ttl + rng.randrange(-300, 300)


def getpubkey_object(address_version, stream, ripe_or_tag, retry_number=0, rng=random, now=None, ntpb=None,
                     extra=None):
    """A getpubkey object (type 0, ``:1436-1445``): the 20-byte ripe for address versions <= 3,
    the 32-byte tag for v4."""
    ttl = getpubkey_ttl(retry_number, rng)
    payload = pack('>Q', int((time.time() if now is None else now) + ttl)) + b'\x00\x00\x00\x00'
    payload += _varint(address_version) + _varint(stream) + bytes(ripe_or_tag)
    n, e = _defaults(ntpb, extra)
    return PowObject(payload, ttl, n, e)


def msg_ttl(ttl, retry_number=0, rng=random):
    """sendMsg's TTL: x 2^retryNumber, capped at 28 days, +- 5 minutes (``:900-905``)."""
    ttl *= 2 ** retry_number
    if ttl > 28 * _DAY:
        ttl = 28 * _DAY
    return int(ttl + rng.randrange(-300, 300))


def msg_difficulty(to_address_version, ntpb=None, extra=None, default_ntpb=None, default_extra=None):
    """The recipient's difficulty as sendMsg applies it (``:1008-1027``): v2 addresses use the
    network defaults; v3+ demand at least the defaults."""
    dn, de = _defaults(default_ntpb, default_extra)
    if to_address_version <= 2 or ntpb is None:
        return dn, de
    return max(ntpb, dn), max(extra, de)


def msg_object(encrypted, to_address_version, stream, ttl, ntpb=None, extra=None, rng=random, now=None,
               default_ntpb=None, default_extra=None):
    """A msg object (type 2, ``:1240-1256``) at the recipient's difficulty (``:1256-1264``)."""
    n, e = msg_difficulty(to_address_version, ntpb, extra, default_ntpb, default_extra)
    payload = pack('>Q', _embedded(ttl, now)) + b'\x00\x00\x00\x02' + _varint(1) + _varint(stream)
    payload += bytes(encrypted)
    return PowObject(payload, ttl, n, e)


# ------------------------------------------------------------------------------------------
# continuous batching across producer threads
# ------------------------------------------------------------------------------------------
class _Group(object):
    """One condition shared by the results of one ``submit_many`` call."""
    __slots__ = ('cv',)

    def __init__(self):
        self.cv = threading.Condition()


class BatchResult(object):
    """The result of one object of a ``PowService.submit_many`` call: ``result(timeout)``,
    ``exception(timeout)`` and ``done()`` as on a ``concurrent.futures.Future``, without its
    per-object lock and condition (a Future costs more to create than the object's whole host-side
    handling; the results of one call share one condition, notified once per completed batch).
    ``_out`` is None while pending, then ``[trialValue, nonce]`` or the exception."""
    __slots__ = ('_group', '_out')

    def __init__(self, group):
        self._group = group
        self._out = None

    def done(self):
        return self._out is not None

    def _wait(self, timeout):
        if self._out is None:
            with self._group.cv:
                if not self._group.cv.wait_for(self.done, timeout):
                    raise TimeoutError('PoW result not ready')
        return self._out

    def result(self, timeout=None):
        out = self._wait(timeout)
        if isinstance(out, BaseException):
            raise out
        return out

    def exception(self, timeout=None):
        out = self._wait(timeout)
        return out if isinstance(out, BaseException) else None

    # completion side (the service's completion thread; waiters are woken by _Sub.notify)
    def set_result(self, value):
        self._out = value

    def set_exception(self, exc):
        self._out = exc


class _Sub(object):
    """The objects of one ``bmpow_service_submit`` call: tickets ``base .. base + n - 1``."""
    __slots__ = ('base', 'ihs', 'offs', 'targets', 'futs', 'group', 'left')

    def __init__(self, ihs, targets, futs, group, offs=None):
        self.base = 0
        self.ihs = ihs  # n x 64 bytes, or the concatenated initialHashes of any lengths (offs)
        self.offs = offs  # None, or n + 1 byte offsets into ihs
        self.targets = targets  # n clamped targets
        self.futs = futs
        self.group = group  # the shared _Group of BatchResults, or None for Futures
        self.left = len(futs)

    def notify(self):
        if self.group is not None:
            with self.group.cv:
                self.group.cv.notify_all()


class PowService(object):
    """A device batch that producers join at any time.

    ``submit(target, initialHash)`` returns a ``concurrent.futures.Future`` that resolves to
    ``[trialValue, nonce]`` (the ``run`` answer) or raises ``StopIteration('Interrupted')``
    when ``state.shutdown`` is set.  The stepping runs inside the library
    (``bmpow_service_create``): a native thread owns a resident device session, appends what
    producers submitted between two steps (only 64-byte hashes and targets cross PCIe), launches
    each bounded step over every pending object and queues the finished ones -- the per-step host
    work is O(new + finished) and no Python thread (so no GIL) sits between two steps.  This
    object's completion thread pops finished objects (``bmpow_service_poll``, GIL released while
    it waits; the library re-hashes each found nonce on the host inside that call, the check
    ``_doGPUPoW`` makes with hashlib) and resolves the futures,
    overlapping the Python work with the device's next step.  An object submitted mid-flight joins
    the next step (~80 ms on one MI355X) instead of waiting for the objects ahead of it, and
    producers never contend for the device.  Replaces concurrent blocking ``run`` calls from the
    worker and API threads (``class_singleWorker.py:236,1276``, ``api.py:1304,1350``)."""

    TAKE = 4096  # finished objects popped per bmpow_service_poll call
    POLL_MS = 100  # longest wait in one poll: bounds the reaction time to state.shutdown / stop()
    SUBMIT_SLICE = 8192  # submit_many hands the library this many objects at a time, so the device
    #                      starts on the first slice while Python prepares the next

    def __init__(self, step_trials=0):
        self.step_trials = step_trials
        self._lock = threading.Lock()  # guards _subs / _bases and the service handle
        self._subs = []  # live _Sub records in ticket order
        self._bases = []  # their first tickets (bisect)
        self._lib = None
        self._lib_err = None
        self._h = None
        self._stopping = False
        self._completer = None
        self.solved = 0
        self.trace = None  # a list to record (time.perf_counter(), objects popped) per poll

    def start(self):
        with self._lock:
            if self._completer is None:
                self._stopping = False
                self._lib_err = None
                try:
                    self._lib = _lib.get()
                    h = self._lib.bmpow_service_create(self.step_trials,
                                                       _lib.SERVICE_VERIFY if proofofwork.VERIFY else 0)
                    if not h:
                        raise _lib.BmpowError(_lib.E_HIP, 'bmpow_service_create: %s'
                                              % self._lib.bmpow_last_error().decode())
                    self._h = h
                except Exception as e:  # noqa: BLE001 -- no device: every submitter sees why
                    self._lib_err = e
                self._completer = threading.Thread(target=self._complete, name='PowService-complete')
                self._completer.daemon = True
                self._completer.start()
        return self

    def stop(self, timeout=None):
        with self._lock:
            self._stopping = True
            th = self._completer
            if self._h is not None:  # wakes the completion thread's poll at once
                self._lib.bmpow_service_stop(self._h)
        if th is not None:
            th.join(timeout)
        with self._lock:
            # a completer still running (join timed out) stays registered: start() must not put a
            # second one beside it; it clears itself when it exits
            if self._completer is th and (th is None or not th.is_alive()):
                self._completer = None

    def submit(self, target, initialHash):
        fut = Future()
        t, ok = proofofwork._clamp_target(target)
        if not ok:
            fut.set_exception(ValueError('negative target: no nonce can satisfy it'))
            return fut
        ih = proofofwork._ih_bytes(initialHash)
        self._enqueue(_Sub(ih, [t], [fut], None, None if len(ih) == 64 else [0, len(ih)]))
        return fut

    def submit_many(self, objects):
        """``[submit(t, ih) for t, ih in objects]`` in a few library calls: a producer with many
        objects at once (a flood of acks, every pending pubkey) joins the next step together.
        Returns one :class:`BatchResult` per object (``result()`` gives ``[trialValue, nonce]``)."""
        group = _Group()
        out = []
        clamp, ihb = proofofwork._clamp_target, proofofwork._ih_bytes
        top = _lib.U64_MAX
        objects = list(objects)
        for lo in range(0, len(objects), self.SUBMIT_SLICE):
            chunk = objects[lo:lo + self.SUBMIT_SLICE]
            futs = [BatchResult(group) for _ in chunk]
            out.extend(futs)
            # the common case in one pass per field: 64-byte hashes and in-range int targets
            tgs = [t for t, _ in chunk]
            ihs = [ih for _, ih in chunk]
            if all(type(t) is int and 0 <= t < top for t in tgs) and \
                    all(type(ih) is bytes and len(ih) == 64 for ih in ihs):
                self._enqueue(_Sub(b''.join(ihs), tgs, futs, group))
                continue
            kf, kih, kt, offs = [], [], [], [0]
            for fut, (target, initialHash) in zip(futs, chunk):
                t, ok = clamp(target)
                if not ok:
                    fut.set_exception(ValueError('negative target: no nonce can satisfy it'))
                    continue
                kf.append(fut)
                kih.append(ihb(initialHash))
                offs.append(offs[-1] + len(kih[-1]))
                kt.append(t)
            if kf:
                var = any(len(ih) != 64 for ih in kih)
                self._enqueue(_Sub(b''.join(kih), kt, kf, group, offs if var else None))
        return out

    def _enqueue(self, sub):
        import array
        with self._lock:
            if self._stopping or self._completer is None:
                raise RuntimeError('PowService is not running')
            if self._h is None:
                self._fail([sub], self._lib_err)
                return
            if state.shutdown != 0:
                self._fail([sub], StopIteration('Interrupted'))
                return
            try:
                proofofwork.check_enabled()
            except _lib.BmpowUnavailable as e:
                self._fail([sub], e)
                return
            n = len(sub.futs)
            tg = array.array('Q', sub.targets)
            tk = (ctypes.c_uint64 * n)()
            if sub.offs is None:
                rc = self._lib.bmpow_service_submit(self._h, n, sub.ihs, ctypes.cast(tg.buffer_info()[0], _P64), tk)
            else:
                off = array.array('Q', sub.offs)
                rc = self._lib.bmpow_service_submit_var(self._h, n, sub.ihs, ctypes.cast(off.buffer_info()[0], _P64),
                                                        ctypes.cast(tg.buffer_info()[0], _P64), tk)
            if rc < 0:
                self._fail([sub], _lib.BmpowError(rc, 'bmpow_service_submit: %s'
                                                  % self._lib.bmpow_last_error().decode()))
                return
            sub.base = tk[0]  # tickets are consecutive within one call
            self._subs.append(sub)
            self._bases.append(sub.base)

    def run(self, target, initialHash):
        """Blocking ``proofofwork.run`` through the shared batch."""
        if state.shutdown != 0:
            raise RuntimeError('No active exception to reraise')
        return self.submit(target, initialHash).result()

    @staticmethod
    def _fail(subs, exc):
        for sub in subs:
            for f in sub.futs:
                if not f.done():
                    f.set_exception(exc)
            sub.notify()

    def _drop_live(self, exc):
        """Cancel everything in the library and fail its futures (caller holds the lock)."""
        dead = self._subs
        self._subs, self._bases = [], []
        self._lib.bmpow_service_cancel(self._h)
        self._fail(dead, exc)

    def _complete(self):
        """Completion thread: pop finished objects (each found nonce re-checked on the host by the
        library) and resolve their futures; cancels on state.shutdown; destroys the library service on stop()."""
        import bisect

        import numpy as np
        lib, h = self._lib, self._h
        tick = np.zeros(self.TAKE, dtype=np.uint64)
        nonce = np.zeros(self.TAKE, dtype=np.uint64)
        trial = np.zeros(self.TAKE, dtype=np.uint64)
        done = np.zeros(self.TAKE, dtype=np.uint8)
        try:
            while not self._stopping:
                if h is None:
                    time.sleep(self.POLL_MS / 1000.0)
                    continue
                if state.shutdown != 0 and self._subs:
                    with self._lock:
                        self._drop_live(StopIteration('Interrupted'))
                    continue
                k = lib.bmpow_service_poll(h, self.TAKE, self.POLL_MS, tick.ctypes.data_as(_P64),
                                           nonce.ctypes.data_as(_P64), trial.ctypes.data_as(_P64),
                                           done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
                if k < 0:
                    err = _lib.BmpowError(k, 'bmpow service step: %s' % lib.bmpow_last_error().decode())
                    with self._lock:
                        self._drop_live(err)
                    continue
                if not k:
                    continue
                if self.trace is not None:
                    self.trace.append((time.perf_counter(), k))
                work = []
                with self._lock:
                    subs, bases = self._subs, self._bases
                    for t, d, tv, nn in zip(tick[:k].tolist(), done[:k].tolist(), trial[:k].tolist(),
                                            nonce[:k].tolist()):
                        j = bisect.bisect_right(bases, t) - 1
                        if j < 0:
                            continue  # dropped by a cancel that raced this poll
                        sub = subs[j]
                        i = t - sub.base
                        if i >= len(sub.futs):
                            continue
                        sub.left -= 1
                        work.append((sub, i, d, tv, nn))
                    if any(s.left == 0 for s in subs):
                        keep = [s for s in subs if s.left > 0]
                        self._subs, self._bases = keep, [s.base for s in keep]
                touched = {}
                for sub, i, d, tv, nn in work:
                    fut = sub.futs[i]
                    if fut.done():
                        continue
                    if d == _lib.DONE_FOUND:  # re-checked on the host by the library (SERVICE_VERIFY)
                        self.solved += 1
                        if sub.group is not None:  # a BatchResult: its field, without the call
                            fut._out = [tv, nn]
                        else:
                            fut.set_result([tv, nn])
                    elif d == _lib.DONE_BADHASH:
                        try:  # disables the backend, as _doGPUPoW does (proofofwork.py:176-190)
                            proofofwork.gpu_failed('answer (nonce %d) failed the host re-check' % nn)
                        except _lib.BmpowError as e:
                            fut.set_exception(e)
                    else:
                        fut.set_exception(_lib.BmpowError(_lib.E_ARG, 'nonce space exhausted'))
                    touched[id(sub)] = sub
                for sub in touched.values():
                    sub.notify()
        finally:
            with self._lock:
                dead = self._subs
                self._subs, self._bases = [], []
                if h is not None:
                    lib.bmpow_service_destroy(h)
                if self._h is h:  # never the handle of a service started after this one
                    self._h = None
                if self._completer is threading.current_thread():
                    self._completer = None
            self._fail(dead, RuntimeError('PowService stopped'))
