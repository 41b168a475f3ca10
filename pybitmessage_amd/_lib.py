"""ctypes binding of ``libbmpow_hip.so`` (C ABI in ``include/bmpow.h``).

Loaded the way the reference loads its native PoW library
(``src/proofofwork.py:371-388``: ``ctypes.CDLL(codePath/bitmsghash/bitmsghash.so)``), but with
``argtypes``/``restype`` set for every entry point.  There is no CPU fallback: if the library
or a gfx950 device is missing, :func:`get` raises :class:`BmpowUnavailable`.
"""
import atexit
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_PATH = os.path.join(HERE, 'lib', 'libbmpow_hip.so')

NOT_FOUND = 0
FOUND = 1
E_NODEV = -1
E_HIP = -2
E_ARG = -3
E_ABORTED = -4
E_STATE = -5

PENDING = 0
DONE_FOUND = 1
DONE_EXHAUSTED = 2
PARKED = 3
FREE = 4
DONE_BADHASH = 5
SERVICE_VERIFY = 1

U64_MAX = (1 << 64) - 1
MAX_IH_LEN = 1 << 20  # BMPOW_MAX_IH_LEN: longest initialHash the library accepts


class BmpowError(RuntimeError):
    """A libbmpow_hip call failed (HIP error, bad argument, ...)."""

    def __init__(self, code, msg):
        RuntimeError.__init__(self, '%s (code %d)' % (msg, code))
        self.code = code


class BmpowUnavailable(BmpowError):
    """The HIP library is not built or no gfx950 device is visible."""


class BmpowStats(ctypes.Structure):
    _fields_ = [('launches', ctypes.c_uint64), ('trials', ctypes.c_uint64),
                ('kernel_ms', ctypes.c_double), ('max_shard_kernel_ms', ctypes.c_double),
                ('steps', ctypes.c_uint64), ('verify_launches', ctypes.c_uint64),
                ('verify_objects', ctypes.c_uint64), ('verify_blocks', ctypes.c_uint64),
                ('verify_kernel_ms', ctypes.c_double), ('addr_launches', ctypes.c_uint64),
                ('addr_tries', ctypes.c_uint64), ('addr_kernel_ms', ctypes.c_double),
                ('probe_trials', ctypes.c_uint64), ('probe_kernel_ms', ctypes.c_double),
                ('verify_host_build_ms', ctypes.c_double), ('verify_host_run_ms', ctypes.c_double),
                ('verify_host_verdict_ms', ctypes.c_double),
                ('cut_trials', ctypes.c_uint64),
                ('one_wait_spin_ms', ctypes.c_double), ('one_wait_sleep_ms', ctypes.c_double),
                ('past_window', ctypes.c_uint64), ('past_later', ctypes.c_uint64),
                ('past_split', ctypes.c_uint64), ('engine_hashed_est', ctypes.c_uint64),
                ('masked_streams', ctypes.c_uint64), ('run_streams', ctypes.c_uint64)]


class BmpowAddress(ctypes.Structure):
    """``bmpow_address`` (include/bmpow.h): one found try of the address search."""
    _fields_ = [('k', ctypes.c_uint64), ('ripe', ctypes.c_uint8 * 20), ('priv_signing', ctypes.c_uint8 * 32),
                ('priv_encryption', ctypes.c_uint8 * 32), ('pub_signing', ctypes.c_uint8 * 65),
                ('pub_encryption', ctypes.c_uint8 * 65)]


# (name, restype, argtypes) for every symbol include/bmpow.h declares
_u64, _p64, _pu8 = ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_pu32 = ctypes.POINTER(ctypes.c_uint32)
SIGNATURES = [
    ('bmpow_init', ctypes.c_int, []),
    ('bmpow_device_count', ctypes.c_int, []),
    ('bmpow_set_devices', ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ('bmpow_set_device_count', ctypes.c_int, [ctypes.c_int]),
    ('bmpow_get_devices', ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ('bmpow_device_pci_bus_id', ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    ('bmpow_get_shard_rates', ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ('bmpow_shutdown', None, []),
    ('bmpow_atexit', None, []),
    ('bmpow_last_error', ctypes.c_char_p, []),
    ('bmpow_version', ctypes.c_char_p, []),
    ('bmpow_abort', None, []),
    ('bmpow_clear_abort', None, []),
    ('bmpow_trials', ctypes.c_int, [ctypes.c_char_p, _p64, ctypes.c_size_t, _p64]),
    ('bmpow_trials_len', ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, _p64, ctypes.c_size_t, _p64]),
    ('bmpow_search', ctypes.c_int, [ctypes.c_char_p, _u64, _u64, _u64, _p64, _p64]),
    ('bmpow_search_len', ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, _u64, _u64, _u64, _p64, _p64]),
    ('bmpow_min_trial', ctypes.c_int, [ctypes.c_char_p, _u64, _u64, _p64, _p64]),
    ('bmpow_min_trial_batch', ctypes.c_int, [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _p64, _p64]),
    ('bmpow_min_trial_var', ctypes.c_int, [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _p64, _p64, _p64]),
    ('bmpow_search_batch', ctypes.c_int,
     [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _u64, _p64, _p64, _pu8]),
    ('bmpow_batch_create', _vp, [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64]),
    ('bmpow_batch_step', ctypes.c_int, [_vp, _u64]),
    ('bmpow_batch_results', ctypes.c_int, [_vp, _p64, _p64, _pu8, _p64]),
    ('bmpow_batch_reset', ctypes.c_int, [_vp, _p64]),
    ('bmpow_batch_set_pending', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]),
    ('bmpow_batch_add', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _pu32]),
    ('bmpow_batch_add_var', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _p64, _pu32]),
    ('bmpow_batch_take_done', ctypes.c_int, [_vp, ctypes.c_size_t, _pu32, _p64, _p64, _pu8]),
    ('bmpow_batch_destroy', None, [_vp]),
    ('bmpow_service_create', _vp, [_u64, ctypes.c_uint32]),
    ('bmpow_service_submit', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_char_p, _p64, _p64]),
    ('bmpow_service_submit_var', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _p64]),
    ('bmpow_service_poll', ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_int, _p64, _p64, _p64, _pu8]),
    ('bmpow_service_cancel', ctypes.c_int, [_vp]),
    ('bmpow_service_outstanding', ctypes.c_int, [_vp]),
    ('bmpow_service_stop', None, [_vp]),
    ('bmpow_service_destroy', None, [_vp]),
    ('bmpow_get_stats', ctypes.c_int, [ctypes.POINTER(BmpowStats)]),
    ('bmpow_reset_stats', None, []),
    ('bmpow_get_shard_stats', ctypes.c_int, [_p64, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ('bmpow_get_thread_info', ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ('bmpow_set_shard_throttle', ctypes.c_int, [ctypes.c_int, ctypes.c_double]),
    ('bmpow_set_run_split', ctypes.c_int, [ctypes.c_int]),
    ('bmpow_set_engine_split', ctypes.c_int, [ctypes.c_int]),
    ('bmpow_get_run_pieces', ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ('bmpow_get_step_trials', _u64, []),
    ('bmpow_set_step_trials', None, [_u64]),
    ('bmpow_pow_values', ctypes.c_int, [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64]),
    ('bmpow_verify_batch', ctypes.c_int,
     [ctypes.c_size_t, ctypes.c_char_p, _p64, _p64, _p64, ctypes.POINTER(ctypes.c_int64), _pu8]),
    ('bmpow_verify_batch_ptrs', ctypes.c_int,
     [ctypes.c_size_t, ctypes.c_void_p, _p64, _p64, _p64, ctypes.POINTER(ctypes.c_int64), _pu8]),
    ('bmpow_pow_sufficient', ctypes.c_int, [_u64, _u64, _u64, _u64, ctypes.c_int64, _u64]),
    ('bmpow_vbatch_create', _vp, [ctypes.c_size_t, ctypes.c_char_p, _p64]),
    ('bmpow_vbatch_run', ctypes.c_int, [_vp, _p64]),
    ('bmpow_vbatch_destroy', None, [_vp]),
    ('bmpow_pubkeys', ctypes.c_int, [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p]),
    ('bmpow_fe_probe', ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ('bmpow_address_search', ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_size_t, _u64, _u64, ctypes.c_int, ctypes.POINTER(BmpowAddress)]),
    ('bmpow_address_search_random', ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, _u64, _u64, ctypes.c_int, ctypes.POINTER(BmpowAddress)]),
    ('bmpow_addr_set_comb', ctypes.c_int, [ctypes.c_int]),
    ('bmpow_addr_last_comb', ctypes.c_int, []),
    ('BitmessagePOW', ctypes.c_ulonglong, [ctypes.c_char_p, ctypes.c_ulonglong]),
]

_lock = threading.Lock()
_lib = None
_exit_hooked = False


def lib_path():
    return os.environ.get('BMPOW_LIB', DEFAULT_PATH)


def load(path=None):
    """dlopen the library and bind every signature (no device access)."""
    path = path or lib_path()
    if not os.path.exists(path):
        raise BmpowUnavailable(E_NODEV, 'libbmpow_hip.so not built at %s (run __graft_entry__.build() '
                                        'or make -C pybitmessage_amd/csrc)' % path)
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if os.path.abspath(path) == os.path.abspath(DEFAULT_PATH):
                raise
            continue  # an A/B build of an earlier round (BMPOW_LIB) may lack later entry points
        fn.restype = res
        fn.argtypes = args
    return lib


def get():
    """The initialised library (devices selected).  Raises BmpowUnavailable."""
    global _lib, _exit_hooked
    with _lock:
        if _lib is None:
            lib = load()
            rc = lib.bmpow_init()
            if rc <= 0:
                raise BmpowUnavailable(rc, 'bmpow_init failed: %s' % lib.bmpow_last_error().decode())
            _lib = lib
            if not _exit_hooked:
                # release the devices (service threads, stepper threads, the streams kept for the
                # process) while the interpreter is still whole; the library's own C atexit hook then
                # finds nothing left to do
                atexit.register(_at_exit, lib)
                _exit_hooked = True
        return _lib


def _at_exit(lib):
    """Python's exit: ``bmpow_atexit`` (include/bmpow.h) before the HIP runtime's exit handlers."""
    fn = getattr(lib, 'bmpow_atexit', None)
    if fn is not None:
        fn()


def reset():
    """Forget the loaded handle's device selection (``resetPoW``)."""
    global _lib
    with _lock:
        if _lib is not None:
            _lib.bmpow_shutdown()
            _lib = None


def check(lib, rc, what):
    if rc < 0:
        msg = lib.bmpow_last_error().decode(errors='replace')
        if rc == E_NODEV:
            raise BmpowUnavailable(rc, '%s: %s' % (what, msg))
        raise BmpowError(rc, '%s: %s' % (what, msg))
    return rc


def u64_array(values):
    arr = (ctypes.c_uint64 * len(values))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr
