"""GPU backend module -- stands in for the reference's ``src/openclpow.py``.

Same module surface as the reference (``initCL``, ``openclAvailable``, ``openclEnabled``,
``do_opencl_pow``, the ``gpus`` / ``enabledGpus`` / ``vendors`` lists) so callers that query GPU
status (``proofofwork.getPowType`` ``:232``, the Qt settings combo box
``bitmessageqt/settings.py:199-209,452-458``, ``support.py:143-146``) keep working, but the
device is a gfx950 MI355X driven through ``libbmpow_hip.so`` instead of a runtime-built OpenCL
kernel.

Differences from the reference, each a fix of an Appendix-B quirk:

* ``do_opencl_pow`` returns the ``_doSafePoW`` nonce (first ``n >= 1`` with ``trial <= target``),
  not the last racing writer's strict-``<`` nonce starting from 0 (``bitmsghash.cl:256-274``);
* the shutdown check reads ``state.shutdown`` live: the reference copies the flag at import
  (``openclpow.py:10``), so its loop (``:99,108``) can never see a shutdown;
* every enabled device is used (nonce-sharded), not only the context's first (``:53-54``).
"""
import ctypes
import logging

from . import _lib
from . import proofofwork
from . import state
from ._lib import BmpowUnavailable

logger = logging.getLogger('default')

#: vendor string a keys.dat ``opencl`` setting may name to select this backend; the reference
#: matches the setting against ``platform.vendor`` (``openclpow.py:45``)
VENDOR = 'Advanced Micro Devices, Inc.'
#: other accepted spellings of the backend in the ``opencl`` setting
ALIASES = ('HIP', 'hip', 'gfx950', 'MI355X', VENDOR)

gpus = []
enabledGpus = []
vendors = []
#: the keys.dat ``opencl`` value of the last :func:`initCL` call that named one; :func:`initCL`
#: without an argument (``proofofwork.resetPoW``) applies it again, as the reference's initCL re-reads
#: the setting from the config every time (``openclpow.py:45``)
_setting = None
_UNSET = object()

#: trials per bounded device call in ``do_opencl_pow`` (its shutdown-poll interval)
CALL_TRIALS = 1 << 30


class Device(object):
    """What the GUI reads from an OpenCL device object: ``.name`` (``proofofwork.py:178``)."""

    def __init__(self, ordinal):
        self.ordinal = ordinal
        self.name = 'AMD Instinct MI355X (gfx950) #%d' % ordinal

    def __repr__(self):
        return '<hippow.Device %s>' % self.name


def initCL(setting=_UNSET):
    """Discover gfx950 devices and enable them (reference ``initCL``, ``openclpow.py:31-64``).

    ``setting`` is the keys.dat ``[bitmessagesettings] opencl`` value; ``None`` or any of
    :data:`ALIASES` enables every visible device, another vendor name leaves them disabled
    (the reference enables only the platform whose vendor matches).  Omitted, the last setting
    given applies (``None`` before any)."""
    global _setting
    if setting is _UNSET:
        setting = _setting
    else:
        _setting = setting
    del enabledGpus[:]
    del vendors[:]
    del gpus[:]
    try:
        lib = _lib.get()
    except BmpowUnavailable as e:
        logger.info('No HIP GPUs found: %s', e)
        return
    ids = (ctypes.c_int * 64)()
    n = lib.bmpow_get_devices(ids, 64)
    gpus.extend(Device(ids[i]) for i in range(n))
    vendors.append(VENDOR)
    if setting is None or setting in ALIASES:
        enabledGpus.extend(gpus)
        logger.info('Loaded HIP PoW kernel on %d device(s)', len(enabledGpus))
    else:
        logger.info('HIP GPUs present but not selected (opencl=%r)', setting)


def openclAvailable():
    """Are there any gfx950 GPUs available? (``openclpow.py:67-69``)"""
    return bool(gpus)


def openclEnabled():
    """Is the GPU backend enabled (and available)? (``openclpow.py:72-74``)"""
    return bool(enabledGpus)


def do_opencl_pow(hash_, target):
    """Nonce for ``hash_`` (initialHash as hex, ``proofofwork.py:175``, any length) and ``target``
    (``openclpow.py:77-111``): the ``_doSafePoW`` nonce.  Returns 0 when no GPU is enabled, like
    the reference; raises ``Exception("Interrupted")`` when ``state.shutdown`` is set between
    bounded calls and ``ValueError`` on a negative target."""
    if not enabledGpus:
        return 0
    ih = proofofwork._ih_bytes(bytes.fromhex(hash_) if isinstance(hash_, str) else bytes(hash_))
    # a negative target is unsatisfiable (never wrapped into a u64, which would accept nonce 1);
    # the reference's numpy packing raises OverflowError on it or wraps it -- it never blocks
    target, satisfiable = proofofwork._clamp_target(target)
    if not satisfiable:
        raise ValueError('negative target: no nonce can satisfy it')
    lib = _lib.get()
    n, tv = ctypes.c_uint64(), ctypes.c_uint64()
    start = 1
    while True:
        if state.shutdown != 0:
            raise Exception('Interrupted')
        rc = _lib.check(lib, lib.bmpow_search_len(ih, len(ih), target, start, CALL_TRIALS, ctypes.byref(n),
                                                  ctypes.byref(tv)), 'bmpow_search_len')
        if rc == _lib.FOUND:
            return n.value
        if start > _lib.U64_MAX - CALL_TRIALS:
            raise Exception('nonce space exhausted')
        start += CALL_TRIALS
