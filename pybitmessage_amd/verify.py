"""Batched receive-side PoW verification on the GPU.

The reference checks every received object with ``protocol.isProofOfWorkSufficient``
(``src/protocol.py:258-286``), one object and three SHA-512s at a time, from the network
thread (``network/bmobject.py:71-76``) and again at the recipient's difficulty in
``class_objectProcessor.py:624-629``.  Here a whole inventory flood is checked in one launch
of ``bv_pow_kernel`` (one object per lane, payload SHA-512 + the double hash of the trial
function) through ``bmpow_verify_batch``; the verdict uses the reference's exact IEEE-double
target arithmetic (host side of the C ABI).  No CPU fallback: without the HIP library the
calls raise :class:`BmpowUnavailable`.
"""
import ctypes
import os
import struct

import numpy as np

from . import _lib

P64 = ctypes.POINTER(ctypes.c_uint64)


def _pack(objects):
    """One concatenated buffer + byte offsets (the ABI's layout); bytes objects are not copied
    before the join."""
    objs = [o if type(o) is bytes else bytes(o) for o in objects]
    offsets = np.zeros(len(objs) + 1, dtype=np.uint64)
    np.cumsum(np.fromiter(map(len, objs), dtype=np.uint64, count=len(objs)), out=offsets[1:])
    return b''.join(objs), offsets, objs


def _per_object(value, n, dtype):
    if not np.ndim(value):
        return np.full(n, value, dtype=dtype)
    arr = np.asarray(value, dtype=dtype)
    if arr.shape != (n,):
        raise ValueError('expected a scalar or %d values' % n)
    return np.ascontiguousarray(arr)


def pow_values(objects):
    """``POW`` of each finished object (nonce || payload), ``protocol.py:280-282``."""
    data, offsets, objs = _pack(objects)
    n = len(objs)
    if n == 0:
        return []
    for o in objs:
        if len(o) < 8:
            raise struct.error('unpack requires a buffer of 8 bytes')
    lib = _lib.get()
    out = np.zeros(n, dtype=np.uint64)
    _lib.check(lib, lib.bmpow_pow_values(n, data, offsets.ctypes.data_as(P64), out.ctypes.data_as(P64)),
               'bmpow_pow_values')
    return [int(v) for v in out]


def _bytes_data_offset():
    """Offset of a CPython bytes object's data from its id() (the object's address): the header
    size, ``bytes.__basicsize__ - 1``.  Checked on a probe; None when the layout differs (then
    the pointers come from a ctypes array instead)."""
    off = bytes.__basicsize__ - 1
    probe = b'bmpow-probe-0123456789'
    try:
        if ctypes.string_at(id(probe) + off, len(probe)) == probe:
            return off
    except Exception:  # noqa: BLE001
        pass
    return None


_DATA_OFFSET = _bytes_data_offset()


def _pointers(objs):
    """Addresses of each object's bytes, without copying them (objs must stay alive)."""
    if _DATA_OFFSET is not None:
        return np.fromiter(map(id, objs), dtype=np.uint64, count=len(objs)) + np.uint64(_DATA_OFFSET)
    arr = (ctypes.c_char_p * len(objs))(*objs)
    return np.frombuffer(arr, dtype=np.uint64).copy()


def _load_fast():
    """The CPython marshalling module built beside the library (csrc/bmpow_pyext.c): walks a list of
    bytes in C and calls bmpow_verify_batch_ptrs with the GIL released.  None when not built (the
    numpy marshalling below is then used; the hashing is on the GPU either way)."""
    import glob
    import importlib.util
    for path in glob.glob(os.path.join(os.path.dirname(_lib.lib_path()), '_bmpow_fast*.so')):
        try:
            spec = importlib.util.spec_from_file_location('_bmpow_fast', path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            return mod
        except (ImportError, OSError):
            continue
    return None


_FAST = None
_FAST_TRIED = False


def _fast():
    global _FAST, _FAST_TRIED
    if not _FAST_TRIED:
        _FAST, _FAST_TRIED = _load_fast(), True
    return _FAST


def isProofOfWorkSufficient_batch(objects, nonceTrialsPerByte=0, payloadLengthExtraBytes=0, recvTime=0):
    """``[protocol.isProofOfWorkSufficient(o, nonceTrialsPerByte, payloadLengthExtraBytes,
    recvTime) for o in objects]`` with one GPU launch.  Each difficulty argument and
    ``recvTime`` may be a scalar or one value per object (``recvTime`` 0 = now, as in the
    reference).  An object shorter than 16 bytes raises ``struct.error`` as the reference's
    ``unpack('>Q', data[8:16])`` does.  The objects are read where they lie
    (``bmpow_verify_batch_ptrs``): no concatenation on the host."""
    objs = objects if type(objects) is list else list(objects)
    n = len(objs)
    if n == 0:
        return []
    fast = _fast()
    if fast is not None and not (np.ndim(nonceTrialsPerByte) or np.ndim(payloadLengthExtraBytes) or np.ndim(recvTime)):
        lib = _lib.get()
        addr = ctypes.cast(lib.bmpow_verify_batch_ptrs, ctypes.c_void_p).value
        args = (int(nonceTrialsPerByte), int(payloadLengthExtraBytes), int(recvTime))
        try:
            rc, ok = fast.verify_list(addr, objs, *args)
        except TypeError:  # bytearray / memoryview items: one bytes copy each
            objs = [o if type(o) is bytes else bytes(o) for o in objs]
            rc, ok = fast.verify_list(addr, objs, *args)
        _lib.check(lib, rc, 'bmpow_verify_batch_ptrs')
        if 2 in ok:
            raise struct.error('unpack requires a buffer of 8 bytes')
        return fast.verdicts(ok)
    if set(map(type, objs)) - {bytes}:  # bytearray / memoryview: one bytes copy each
        objs = [o if type(o) is bytes else bytes(o) for o in objs]
    ptrs = _pointers(objs)
    lens = np.fromiter(map(len, objs), dtype=np.uint64, count=n)
    ntpb = _per_object(nonceTrialsPerByte, n, np.uint64)
    extra = _per_object(payloadLengthExtraBytes, n, np.uint64)
    recv = _per_object([int(r) for r in recvTime] if np.ndim(recvTime) else int(recvTime), n, np.int64)
    lib = _lib.get()
    ok = np.zeros(n, dtype=np.uint8)
    _lib.check(lib, lib.bmpow_verify_batch_ptrs(n, ptrs.ctypes.data, lens.ctypes.data_as(P64),
                                                ntpb.ctypes.data_as(P64), extra.ctypes.data_as(P64),
                                                recv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))),
               'bmpow_verify_batch_ptrs')
    del objs  # the pointers were valid for the call
    if (ok == 2).any():
        raise struct.error('unpack requires a buffer of 8 bytes')
    return ok.astype(bool).tolist()


class VerifyBatch(object):
    """Objects padded, sorted and resident in HBM; :meth:`run` hashes all of them again
    (``bmpow_vbatch_*``, used by bench.py's verification leg)."""

    def __init__(self, objects):
        data, offsets, objs = _pack(objects)
        self.n = len(objs)
        self.lib = _lib.get()
        self.handle = self.lib.bmpow_vbatch_create(self.n, data, offsets.ctypes.data_as(P64))
        if not self.handle:
            raise _lib.BmpowError(_lib.E_HIP, 'bmpow_vbatch_create: %s' % self.lib.bmpow_last_error().decode())

    def run(self, want=True):
        out = np.zeros(self.n, dtype=np.uint64) if want else None
        _lib.check(self.lib, self.lib.bmpow_vbatch_run(self.handle, out.ctypes.data_as(P64) if want else None),
                   'bmpow_vbatch_run')
        return out

    def close(self):
        if self.handle:
            self.lib.bmpow_vbatch_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
