"""Target formulas and the receive-side PoW check -- the data format on either side of
the hot path.

All three reproduce the reference's float arithmetic exactly (IEEE double via Python 3 true
division, then ``int()`` truncation in ``proofofwork.run``); integer or rational arithmetic
would differ in the last unit for some inputs.
"""
import hashlib
import time
from struct import pack, unpack

#: ``src/defaults.py:20,24``
networkDefaultProofOfWorkNonceTrialsPerByte = 1000
networkDefaultPayloadLengthExtraBytes = 1000
#: ``src/defaults.py:7``
ridiculousDifficulty = 20000000


def object_target(payload_len, ttl, nonce_trials_per_byte=networkDefaultProofOfWorkNonceTrialsPerByte,
                  payload_length_extra_bytes=networkDefaultPayloadLengthExtraBytes):
    """Sender-side target: ``class_singleWorker._doPOWDefaults`` (``:222-230``) and the msg
    target (``:1256-1264``).  ``payload_len`` excludes the 8-byte nonce.  Returns the float
    the reference passes to ``proofofwork.run``."""
    ln = payload_len + 8 + payload_length_extra_bytes
    return 2 ** 64 / (nonce_trials_per_byte * (ln + ((ttl * ln) / (2 ** 16))))


def api_target(payload_len, nonce_trials_per_byte=networkDefaultProofOfWorkNonceTrialsPerByte,
               payload_length_extra_bytes=networkDefaultPayloadLengthExtraBytes):
    """``api.py:1288-1293`` / ``:1345-1347`` variant (no TTL term)."""
    return 2 ** 64 / ((payload_len + payload_length_extra_bytes + 8) * nonce_trials_per_byte)


def int_target(target):
    """``proofofwork.run``'s ``target = int(target)`` (``:293``)."""
    return int(target)


def pow_value(data):
    """POW of a finished object (nonce || rest): ``protocol.py:280-282``."""
    return unpack('>Q', hashlib.sha512(hashlib.sha512(
        data[:8] + hashlib.sha512(data[8:]).digest()).digest()).digest()[0:8])[0]


def isProofOfWorkSufficient(data, nonceTrialsPerByte=0, payloadLengthExtraBytes=0, recvTime=0):
    """Receive-side check, same semantics as ``protocol.isProofOfWorkSufficient``
    (``src/protocol.py:258-286``): difficulty clamped up to the network defaults, TTL from
    the object's expiry (bytes 8..16) clamped to >= 300 s, accept ``POW <= target``."""
    if nonceTrialsPerByte < networkDefaultProofOfWorkNonceTrialsPerByte:
        nonceTrialsPerByte = networkDefaultProofOfWorkNonceTrialsPerByte
    if payloadLengthExtraBytes < networkDefaultPayloadLengthExtraBytes:
        payloadLengthExtraBytes = networkDefaultPayloadLengthExtraBytes
    endOfLifeTime, = unpack('>Q', data[8:16])
    TTL = endOfLifeTime - (int(recvTime) if recvTime else int(time.time()))
    if TTL < 300:
        TTL = 300
    POW = pow_value(data)
    return POW <= 2 ** 64 / (
        nonceTrialsPerByte * (
            len(data) + payloadLengthExtraBytes
            + ((TTL * (len(data) + payloadLengthExtraBytes)) / (2 ** 16))))


def attach_nonce(nonce, payload):
    """``pack('>Q', nonce) + payload`` (``class_singleWorker.py:249,1290``)."""
    return pack('>Q', nonce) + payload
