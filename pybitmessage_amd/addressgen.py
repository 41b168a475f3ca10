"""RIPE-prefix address search on the GPU -- the key-generation loops of
the reference's ``class_addressGenerator`` and the address/key formats either side of them.

The reference searches, one try at a time in Python with OpenSSL point multiplications, for a
key pair whose ``ripe = RIPEMD160(SHA512(pubSigningKey || pubEncryptionKey))`` starts with
``numberOfNullBytesDemandedOnFrontOfRipeHash`` zero bytes (1, or 2 for "shorter" addresses):

* deterministic addresses (``class_addressGenerator.py:238-271``; chans, ``getDeterministicAddress``):
  try k uses ``SHA512(passphrase || varint(2k))[:32]`` and ``... varint(2k+1)``, and the
  next address continues at k + 1 -- :func:`deterministic_addresses` returns the same
  addresses and keys (exact: the GPU search returns the first k);
* random addresses (``:130-148``): fixed signing key, fresh encryption keys --
  :func:`random_address` (any key pair meeting the prefix is valid).

The search itself runs through ``bmpow_address_search*`` in ``libbmpow_hip.so``; the formats
(``encodeVarint``, ``encodeAddress``, WIF) are restated from ``src/addresses.py`` and
``src/pyelliptic/arithmetic.py``.  No CPU fallback.
"""
import ctypes
import hashlib
import os
import struct

from . import _lib

ALPHABET = '123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
#: tries per bounded device call (the caller's shutdown-poll interval)
CALL_TRIES = 1 << 24


def encodeVarint(integer):
    """``addresses.encodeVarint`` (``src/addresses.py:66-79``)."""
    if integer < 0:
        raise ValueError('varint cannot be < 0')
    if integer < 253:
        return struct.pack('>B', integer)
    if integer < 65536:
        return struct.pack('>B', 253) + struct.pack('>H', integer)
    if integer < 4294967296:
        return struct.pack('>B', 254) + struct.pack('>I', integer)
    if integer < 18446744073709551616:
        return struct.pack('>B', 255) + struct.pack('>Q', integer)
    raise ValueError('varint cannot be >= 18446744073709551616')


def encodeBase58(num):
    """``addresses.encodeBase58`` (``src/addresses.py:16-33``)."""
    if num < 0:
        return None
    if num == 0:
        return ALPHABET[0]
    out = []
    while num:
        num, rem = divmod(num, 58)
        out.append(ALPHABET[rem])
    return ''.join(reversed(out))


def encodeAddress(version, stream, ripe):
    """``addresses.encodeAddress`` (``src/addresses.py:146-181``): strip the ripe's leading
    zero bytes (v2/v3: at most two; v4: all), append a double-SHA-512 checksum, base58."""
    if version >= 2 and version < 4:
        if len(ripe) != 20:
            raise ValueError('ripe must be 20 bytes')
        if ripe[:2] == b'\x00\x00':
            ripe = ripe[2:]
        elif ripe[:1] == b'\x00':
            ripe = ripe[1:]
    elif version == 4:
        if len(ripe) != 20:
            raise ValueError('ripe must be 20 bytes')
        ripe = ripe.lstrip(b'\x00')
    data = encodeVarint(version) + encodeVarint(stream) + ripe
    checksum = hashlib.sha512(hashlib.sha512(data).digest()).digest()[0:4]
    return 'BM-' + encodeBase58(int.from_bytes(data + checksum, 'big'))


def wif(privkey):
    """Wallet Import Format of a 32-byte private key as the reference stores it
    (``class_addressGenerator.py:169-178``: ``0x80 || key || sha256d[:4]``, base58)."""
    raw = b'\x80' + bytes(privkey)
    checksum = hashlib.sha256(hashlib.sha256(raw).digest()).digest()[0:4]
    return encodeBase58(int.from_bytes(raw + checksum, 'big'))


class Found(object):
    """One search result: the try index and everything derived from it."""
    __slots__ = ('k', 'ripe', 'priv_signing', 'priv_encryption', 'pub_signing', 'pub_encryption')

    def __init__(self, a):
        self.k = a.k
        self.ripe = bytes(a.ripe)
        self.priv_signing = bytes(a.priv_signing)
        self.priv_encryption = bytes(a.priv_encryption)
        self.pub_signing = bytes(a.pub_signing)
        self.pub_encryption = bytes(a.pub_encryption)


def pubkeys(privkeys):
    """``highlevelcrypto.pointMult`` for many 32-byte private keys at once (65-byte keys)."""
    keys = [bytes(k) for k in privkeys]
    for k in keys:
        if len(k) != 32:
            raise ValueError('private keys are 32 bytes')
    if not keys:
        return []
    lib = _lib.get()
    out = ctypes.create_string_buffer(65 * len(keys))
    _lib.check(lib, lib.bmpow_pubkeys(len(keys), b''.join(keys), out), 'bmpow_pubkeys')
    raw = out.raw
    return [raw[65 * i:65 * i + 65] for i in range(len(keys))]


def _interrupted():
    from . import state
    return getattr(state, 'shutdown', 0) != 0


def search_deterministic(passphrase, null_bytes=1, start=0, max_tries=None):
    """First try k >= start of the deterministic loop whose ripe meets the prefix, as a
    :class:`Found`; None when ``max_tries`` run out.  Bounded device calls; raises
    ``StopIteration('Interrupted')`` on ``state.shutdown`` between them."""
    if isinstance(passphrase, str):
        passphrase = passphrase.encode('utf-8')
    lib = _lib.get()
    out = _lib.BmpowAddress()
    k = start
    left = max_tries
    while left is None or left > 0:
        if _interrupted():
            raise StopIteration('Interrupted')
        n = CALL_TRIES if left is None else min(CALL_TRIES, left)
        rc = _lib.check(lib, lib.bmpow_address_search(passphrase, len(passphrase), k, n, null_bytes,
                                                      ctypes.byref(out)), 'bmpow_address_search')
        if rc == _lib.FOUND:
            return Found(out)
        k += n
        if left is not None:
            left -= n
    return None


def deterministic_addresses(passphrase, count=1, version=4, stream=1, null_bytes=1):
    """``createDeterministicAddresses`` / ``getDeterministicAddress`` key generation
    (``class_addressGenerator.py:232-300``): ``count`` addresses, each search continuing after
    the previous one's try.  Returns dicts with the address, ripe and WIF keys."""
    out = []
    k = 0
    for _ in range(count):
        f = search_deterministic(passphrase, null_bytes, k)
        out.append({'address': encodeAddress(version, stream, f.ripe), 'ripe': f.ripe, 'k': f.k,
                    'privSigningKey': wif(f.priv_signing), 'privEncryptionKey': wif(f.priv_encryption),
                    'pubSigningKey': f.pub_signing, 'pubEncryptionKey': f.pub_encryption})
        k = f.k + 1
    return out


def random_address(version=4, stream=1, null_bytes=1, priv_signing=None, seed=None):
    """``createRandomAddress`` key generation (``:130-148``): a random signing key kept fixed,
    encryption keys from a CSPRNG-seeded stream until the ripe meets the prefix."""
    priv_signing = bytes(priv_signing) if priv_signing is not None else os.urandom(32)
    seed = bytes(seed) if seed is not None else os.urandom(64)
    lib = _lib.get()
    out = _lib.BmpowAddress()
    k = 0
    while True:
        if _interrupted():
            raise StopIteration('Interrupted')
        rc = _lib.check(lib, lib.bmpow_address_search_random(priv_signing, seed, len(seed), k, CALL_TRIES,
                                                             null_bytes, ctypes.byref(out)),
                        'bmpow_address_search_random')
        if rc == _lib.FOUND:
            f = Found(out)
            return {'address': encodeAddress(version, stream, f.ripe), 'ripe': f.ripe, 'k': f.k,
                    'privSigningKey': wif(f.priv_signing), 'privEncryptionKey': wif(f.priv_encryption),
                    'pubSigningKey': f.pub_signing, 'pubEncryptionKey': f.pub_encryption}
        k += CALL_TRIES
