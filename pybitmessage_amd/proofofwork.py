"""MI355X proof of work -- drop-in for the reference's ``src/proofofwork.py``.

Same public names and return shapes as the reference:

* ``run(target, initialHash) -> [trialValue, nonce]``      (reference ``:288-325``)
* ``init()``, ``resetPoW()``, ``getPowType()``, ``estimate()`` (``:336-394, 328-330, 229-236, 197-226``)

plus the batched entry point BASELINE.json's north star asks for:

* ``run_batch([(target, initialHash), ...]) -> [[trialValue, nonce], ...]`` in input order,
  each element equal to ``run`` on that element;
* ``iter_batch(...)`` yields ``(index, trialValue, nonce)`` as objects finish (lets a
  caller release msgs whose embedded ack just finished, ``class_singleWorker.py:1220``).

Every answer is the ``_doSafePoW`` answer (``:100-111``): the first ``nonce >= 1`` with
``trialValue <= target``, for an ``initialHash`` of any length (hashed as given, ``:104-107``;
every caller passes a 64-byte digest, the layout the main kernel is specialised for, other
lengths run on ``bm_search_var_kernel``).  The search runs on gfx950 through ``libbmpow_hip.so``
in bounded steps; between steps ``state.shutdown`` is polled and a set flag raises
``StopIteration("Interrupted")`` (the reference contract, ``:104-109``; the polling
pattern of ``dev/powinterrupttest.py:22-37``).  There is NO CPU fallback: a missing library
or device raises :class:`BmpowUnavailable` (the reference silently degraded to Python).

A GPU answer that fails the host re-check disables the backend, as ``_doGPUPoW`` disables
OpenCL (``:176-190``): the reference's error line is logged, ``hippow.enabledGpus`` is cleared,
:func:`getPowType` reports ``"none"`` and every later call raises :class:`BmpowUnavailable`
until :func:`resetPoW` -- the reference's fallback chain would continue on the CPU, which this
product does not have.
"""
import ctypes
import hashlib
import logging
import os
import subprocess
import sys
import tempfile
from struct import pack, unpack

from . import _lib
from . import state
from ._lib import BmpowError, BmpowUnavailable  # noqa: F401  (re-exported)

logger = logging.getLogger('default')

U64_MAX = _lib.U64_MAX
#: trials per bounded ``bmpow_search`` call from ``run``: a few steps of the scheduler
#: (~0.1-0.3 s on one MI355X), i.e. the shutdown-poll interval of the Python loop.
CALL_TRIALS = 1 << 30
#: a batch of one object takes run()'s single-object path (iter_batch); False sends it to the service (A/B)
BATCH_ONE = True
#: re-check every returned nonce on the host, as ``_doGPUPoW`` does with hashlib (``:176-190``):
#: hashlib here for ``run``; the library's OpenSSL SHA-512 (``BMPOW_SERVICE_VERIFY``) for batches
VERIFY = True


def _ih_bytes(initialHash):
    """initialHash as bytes, at its own length: ``_doSafePoW`` hashes ``pack('>Q', nonce) +
    initialHash`` as given (``:104-107``), so no padding (round 2 zero-padded to 64 bytes, the
    ``_doCPoW`` buffer's behaviour, ``:161``, which gives other nonces).  Up to
    ``_lib.MAX_IH_LEN`` bytes (1 MiB; the reference has no limit, its callers pass 64)."""
    if isinstance(initialHash, str):
        initialHash = initialHash.encode('latin-1')
    ih = bytes(initialHash)
    if len(ih) > _lib.MAX_IH_LEN:
        raise ValueError('initialHash longer than %d bytes (got %d)' % (_lib.MAX_IH_LEN, len(ih)))
    return ih


def _clamp_target(target):
    """``trialValue <= target`` on Python ints: any target >= 2^64-1 accepts every trial;
    a negative target accepts none (the reference then loops until shutdown)."""
    target = int(target)
    if target >= U64_MAX:
        return U64_MAX, True
    if target < 0:
        return 0, False
    return target, True


def _trial_host(nonce, ih):
    return unpack('>Q', hashlib.sha512(hashlib.sha512(pack('>Q', nonce) + ih).digest()).digest()[0:8])[0]


#: set by :func:`gpu_failed` (a wrong GPU answer), cleared by :func:`resetPoW`
_disabled = None
#: optional ``callable(message)`` the application sets to surface :func:`gpu_failed` in its UI (the
#: reference puts an ``updateStatusBar`` signal on ``queues.UISignalQueue``, ``:178-185``)
ui_notify = None


def gpu_failed(detail):
    """Disable the GPU backend after a wrong answer (``_doGPUPoW``, ``:176-190``) and raise."""
    global _disabled
    from . import hippow
    names = ', '.join(g.name for g in hippow.enabledGpus) or 'gfx950'
    logger.error('Your GPUs (%s) did not calculate correctly, disabling OpenCL. Please report to the developers.',
                 names)
    if ui_notify is not None:
        try:
            ui_notify('Your GPU(s) did not calculate correctly, disabling OpenCL. Please report to the developers.')
        except Exception:  # noqa: BLE001 -- a UI hook never masks the error below
            logger.exception('ui_notify failed')
    del hippow.enabledGpus[:]
    _disabled = detail
    raise BmpowError(_lib.E_HIP, 'GPU did not calculate correctly: %s' % detail)


def check_enabled():
    if _disabled is not None:
        raise BmpowUnavailable(_lib.E_NODEV, 'HIP PoW disabled after a wrong GPU answer (%s); resetPoW() '
                                             're-enables it' % _disabled)


def _verify(target, ih, trial, nonce):
    if VERIFY and _trial_host(nonce, ih) != trial:
        gpu_failed('wrong trial value for nonce %d' % nonce)
    if trial > target:
        gpu_failed('nonce %d above target' % nonce)


def _interrupted():
    return getattr(state, 'shutdown', 0) != 0


def _doHIPPoW(target, initialHash):
    """Single object on the GPU; replaces ``_doGPUPoW``/``_doCPoW`` (``:157-194``)."""
    check_enabled()
    lib = _lib.get()
    ih = _ih_bytes(initialHash)
    t, satisfiable = _clamp_target(target)
    start = 1
    n, tv = ctypes.c_uint64(), ctypes.c_uint64()
    logger.debug('HIP PoW start')
    while True:
        if _interrupted():
            raise StopIteration('Interrupted')
        if not satisfiable:
            # no trial can be <= a negative target: spin like the reference, interruptibly
            import time
            time.sleep(0.05)
            continue
        rc = _lib.check(lib, lib.bmpow_search_len(ih, len(ih), t, start, CALL_TRIALS, ctypes.byref(n),
                                                  ctypes.byref(tv)), 'bmpow_search_len')
        if rc == _lib.FOUND:
            break
        if start > U64_MAX - CALL_TRIALS:
            raise BmpowError(_lib.E_ARG, 'nonce space exhausted without a hit')
        start += CALL_TRIALS
    trialValue, nonce = tv.value, n.value
    _verify(t, ih, trialValue, nonce)
    if _interrupted():
        raise StopIteration('Interrupted')
    logger.debug('HIP PoW done')
    return [trialValue, nonce]


def run(target, initialHash):
    """Run the proof of work (reference ``:288-325``).  Returns ``[trialValue, nonce]``."""
    if _interrupted():
        # the reference's bare ``raise`` outside an except block (``:291-292``)
        raise RuntimeError('No active exception to reraise')
    return _doHIPPoW(int(target), initialHash)


class PowInterrupted(Exception):
    """Raised by :func:`iter_batch` when ``state.shutdown`` is set (a generator cannot raise
    StopIteration, PEP 479); :func:`run_batch` turns it into ``StopIteration("Interrupted")``."""


def iter_batch(objects, step_trials=0):
    """Solve many ``(target, initialHash)`` objects at once on the GPU, yielding
    ``(index, trialValue, nonce)`` as each finishes.

    The objects go to the library's continuous-batching service (``bmpow_service_create`` /
    ``bmpow_service_submit``): its native thread keeps the object table in HBM and steps it --
    each step one bounded launch per device over the pending objects, large objects nonce-sharded
    and small ones packed many per launch -- without ever waiting on this interpreter's GIL.  This
    generator pops the finished objects (``bmpow_service_poll``, GIL released while it waits; the
    library re-hashes each found nonce on the host there, ``BMPOW_SERVICE_VERIFY``) and yields
    them while the next step runs.  A single object takes :func:`run`'s single-object path instead
    (no service to set up; re-checked with hashlib as :func:`run` does).  ``state.shutdown`` is
    polled at least every 100 ms and raises :class:`PowInterrupted`; closing the generator stops
    the service after its current step."""
    import numpy as np
    check_enabled()
    lib = _lib.get()
    objs = list(objects)
    n = len(objs)
    if n == 0:
        return
    ihs = bytearray()
    offs = [0]
    targets = np.empty(n, dtype=np.uint64)
    for i, (target, ih) in enumerate(objs):
        ihs += _ih_bytes(ih)
        offs.append(len(ihs))
        t, ok = _clamp_target(target)
        if not ok:
            raise ValueError('object %d has a negative target: no nonce can satisfy it' % i)
        targets[i] = t
    ihs = bytes(ihs)
    if n == 1 and BATCH_ONE:
        # One object -- the common case of a send (its ack, then its msg): run()'s single-object path
        # (one launch per window and device, the result in host-mapped memory) rather than a service
        # thread and a resident session set up for one object.  Same answer, same shutdown behaviour.
        try:
            tv, nonce = _doHIPPoW(int(targets[0]), ihs)
        except StopIteration:
            raise PowInterrupted()
        yield 0, tv, nonce
        return
    var = len(ihs) != 64 * n or any(b - a != 64 for a, b in zip(offs, offs[1:]))
    p64 = ctypes.POINTER(ctypes.c_uint64)
    s = lib.bmpow_service_create(step_trials, _lib.SERVICE_VERIFY if VERIFY else 0)
    if not s:
        raise BmpowError(_lib.E_HIP, 'bmpow_service_create: %s' % lib.bmpow_last_error().decode())
    try:
        cap = min(n, 65536)
        tick = np.zeros(max(n, cap), dtype=np.uint64)
        if var:  # some initialHash is not 64 bytes: per-object offsets
            off = np.array(offs, dtype=np.uint64)
            _lib.check(lib, lib.bmpow_service_submit_var(s, n, ihs, off.ctypes.data_as(p64), targets.ctypes.data_as(p64),
                                                         tick.ctypes.data_as(p64)), 'bmpow_service_submit_var')
        else:
            _lib.check(lib, lib.bmpow_service_submit(s, n, ihs, targets.ctypes.data_as(p64), tick.ctypes.data_as(p64)),
                       'bmpow_service_submit')
        base = int(tick[0])  # tickets are consecutive from the first
        nonce = np.zeros(cap, dtype=np.uint64)
        trial = np.zeros(cap, dtype=np.uint64)
        done = np.zeros(cap, dtype=np.uint8)
        remaining = n
        while remaining:
            if _interrupted():
                raise PowInterrupted('Interrupted')
            k = _lib.check(lib, lib.bmpow_service_poll(s, cap, 100, tick.ctypes.data_as(p64), nonce.ctypes.data_as(p64),
                                                       trial.ctypes.data_as(p64),
                                                       done.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))),
                           'bmpow_service_poll')
            for t, tv, nn, d in zip(tick[:k].tolist(), trial[:k].tolist(), nonce[:k].tolist(), done[:k].tolist()):
                i = t - base
                if d == _lib.DONE_BADHASH:
                    gpu_failed('object %d: answer (nonce %d) failed the host re-check' % (i, nn))
                if d != _lib.DONE_FOUND:
                    raise BmpowError(_lib.E_ARG, 'object %d: nonce space exhausted' % i)
                yield i, tv, nn
            remaining -= k
    finally:
        lib.bmpow_service_destroy(s)


def run_batch(objects, step_trials=0):
    """``[(target, initialHash), ...] -> [[trialValue, nonce], ...]`` in input order."""
    objs = list(objects)
    out = [None] * len(objs)
    if _interrupted() and objs:
        raise RuntimeError('No active exception to reraise')
    try:
        for i, tv, nonce in iter_batch(objs, step_trials):
            out[i] = [tv, nonce]
    except PowInterrupted:
        raise StopIteration('Interrupted')
    return out


def init():
    """Load ``libbmpow_hip.so`` and select the gfx950 devices (reference ``:336-394``).
    Returns the number of device shards; when the library is not built, tries
    :func:`buildCPoW` once (the reference's build-on-demand, ``:393-394``); logs and returns 0
    when still unavailable."""
    try:
        return _device_count()
    except BmpowUnavailable as e:
        if not os.path.exists(_lib.lib_path()) and buildCPoW():
            return init()
        logger.error('HIP PoW unavailable: %s', e)
        return 0


def buildCPoW():
    """Build the native module on demand (reference ``buildCPoW``, ``:262-285``, which ran
    ``make -C bitmsghash``): ``make -C pybitmessage_amd/csrc`` with hipcc for gfx950.
    Returns True when the library exists afterwards."""
    if os.path.exists(_lib.lib_path()):
        return True
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'csrc')
    try:
        subprocess.call(['make', '-C', csrc])
    except OSError as e:
        logger.error('Failed to build the HIP PoW module: %s', e)
        return False
    ok = os.path.exists(_lib.lib_path())
    logger.info('HIP PoW module %s', 'built successfully' if ok else 'failed to build')
    return ok


class LogOutput(object):  # pylint: disable=too-few-public-methods
    """Capture file-descriptor-1 output of native code for the scope of a ``with`` block and
    log it line by line (reference ``LogOutput``, ``:27-69``; the reference wraps the C
    library call in it, ``:158``).  ``libbmpow_hip.so`` prints nothing, so the HIP path does
    not need it; it is kept for callers and tests of the reference interface."""

    def __init__(self, prefix='PoW'):
        self.prefix = prefix
        self._saved = None
        self._tmp = None

    def __enter__(self):
        try:
            sys.stdout.flush()
        except (AttributeError, ValueError, OSError):
            pass
        try:
            self._saved = os.dup(1)  # native code writes to fd 1 whatever sys.stdout is
        except OSError:
            return self  # no fd 1 (e.g. a windowed app): nothing to capture
        self._tmp = tempfile.TemporaryFile(mode='w+b')
        os.dup2(self._tmp.fileno(), 1)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        if self._saved is None:
            return False
        try:
            sys.stdout.flush()
        except (AttributeError, ValueError, OSError):
            pass
        os.dup2(self._saved, 1)
        os.close(self._saved)
        self._saved = None
        self._tmp.seek(0)
        for line in self._tmp.read().decode('utf-8', 'replace').splitlines():
            logger.info('%s: %s', self.prefix, line)
        self._tmp.close()
        return False


def _device_count():
    lib = _lib.get()
    ids = (ctypes.c_int * 64)()
    return lib.bmpow_get_devices(ids, 64)


def resetPoW():
    """Re-select devices and re-enable the backend after :func:`gpu_failed` (reference
    ``:328-330`` re-ran ``openclpow.initCL``, which re-reads the keys.dat ``opencl`` setting: the
    GPUs come back only when the configured vendor is this backend -- :func:`hippow.initCL` applies
    the last setting it was given)."""
    global _disabled
    _disabled = None
    _lib.reset()
    n = init()
    from . import hippow
    hippow.initCL()
    return n


def getPowType():
    """``"HIP"`` when the gfx950 engine is usable (reference ``:229-236`` returned
    ``"OpenCL"``/``"C"``/``"python"``); ``"none"`` otherwise -- no device, or disabled after a
    wrong answer (:func:`gpu_failed`; there is no CPU fallback)."""
    if _disabled is not None:
        return 'none'
    try:
        _lib.get()
        return 'HIP'
    except BmpowUnavailable:
        return 'none'


def estimate(difficulty, format=False):  # pylint: disable=redefined-builtin
    """Kept with the reference's exact semantics (``:197-226``, ``difficulty / 10`` and
    ``None`` when ``format`` is set) for API compatibility."""
    ret = difficulty / 10
    if ret < 1:
        ret = 1
    if format:
        ret = None
    return ret


def abort():
    """Make an in-flight device search return at its next step boundary (thread/signal safe)."""
    _lib.get().bmpow_abort()


def clear_abort():
    _lib.get().bmpow_clear_abort()
