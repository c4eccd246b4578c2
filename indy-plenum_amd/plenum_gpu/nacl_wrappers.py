"""Ed25519 key objects of stp_core/crypto/nacl_wrappers.py with a GPU backend.

Same classes, constructor checks, return values and exceptions as the
reference (VerifyKey :63-108, SigningKey :111-176, Signer :179-209,
Verifier :212-242), but every verification and signature is computed by the
HIP kernels in libplenum_verify.so:

  * VerifyKey.verify / crypto_sign_open   -> pv_verify_batch (batch of 1)
  * verify_signed_batch / Verifier.verify_batch -> one pv_verify_batch call
  * SigningKey / SigningKey.sign          -> pv_sign_batch

crypto_sign_open framing is applied on the host exactly as libsodium does it
(SURVEY.md App. C.1): sm = sig || msg; len(sm) < 64 rejects; otherwise the
kernel checks sm[:64] against sm[64:].  There is no CPU fallback.
"""
import binascii
import os

import numpy as np

from . import _native

SIGN_BYTES = 64
PUBLICKEY_BYTES = 32
SEED_BYTES = 32


class RawEncoder:
    @staticmethod
    def encode(data):
        return data

    @staticmethod
    def decode(data):
        return data


class HexEncoder:
    @staticmethod
    def encode(data):
        return binascii.hexlify(data)

    @staticmethod
    def decode(data):
        return binascii.unhexlify(data)


class Encodable:
    def encode(self, encoder=RawEncoder):
        return encoder.encode(bytes(self))


# ----------------------------------------------------------------- batch core
def verify_signed_batch(items):
    """crypto_sign_open verdicts for [(pk32, sm)] -> np.ndarray[bool].

    Entries with len(sm) < 64 are rejected on the host (libsodium's first
    check); every other entry is verified on the GPU in one launch sequence.
    """
    n = len(items)
    out = np.zeros(n, dtype=bool)
    idx, pks, sigs, msgs = [], [], [], []
    for k, (pk, sm) in enumerate(items):
        if len(pk) != PUBLICKEY_BYTES:
            raise ValueError('The key must be exactly %s bytes long' % PUBLICKEY_BYTES)
        if len(sm) < SIGN_BYTES:
            continue
        idx.append(k)
        pks.append(pk)
        sigs.append(sm[:SIGN_BYTES])
        msgs.append(sm[SIGN_BYTES:])
    if idx:
        blob, off = _native.pack_messages(msgs)
        pk_arr = np.frombuffer(b''.join(pks), np.uint8).reshape(-1, 32)
        sig_arr = np.frombuffer(b''.join(sigs), np.uint8).reshape(-1, 64)
        out[np.asarray(idx)] = _native.verify_batch_arrays(pk_arr, sig_arr, blob, off)
    return out


def cache_verkeys(keys):
    """Put 32-byte verifying keys a node already knows (node keys, client DIDs,
    NYM verkeys) in the persistent device key cache (pv_keycache_add): small
    host calls under them skip the decompression of A.  Verdicts are unchanged.
    No GPU work happens here; the keys are added by the next verify call."""
    for k in keys:
        k = bytes(k)
        if len(k) != PUBLICKEY_BYTES:
            raise ValueError('The key must be exactly %s bytes long' % PUBLICKEY_BYTES)
        _native.keycache_defer(k)


def crypto_sign_open(sm, pk):
    """libnacl.crypto_sign_open contract: the message, or ValueError."""
    if not verify_signed_batch([(bytes(pk), bytes(sm))])[0]:
        raise ValueError('Failed to validate message')
    return bytes(sm[SIGN_BYTES:])


def _sign(seed, msg):
    seeds = np.frombuffer(seed, np.uint8).reshape(1, 32)
    blob, off = _native.pack_messages([bytes(msg)])
    pk, sig = _native.sign_batch_arrays(seeds, blob, off)
    return pk[0].tobytes(), sig[0].tobytes()


def sign_batch(seeds, msgs):
    """[(seed32)], [msg] -> (pk (n,32) u8, sig (n,64) u8) via the GPU signer."""
    seeds = np.frombuffer(b''.join(seeds), np.uint8).reshape(-1, 32)
    blob, off = _native.pack_messages([bytes(m) for m in msgs])
    return _native.sign_batch_arrays(seeds, blob, off)


# --------------------------------------------------------------- key objects
class SignedMessage(bytes):
    @classmethod
    def _from_parts(cls, signature, message, combined):
        obj = cls(combined)
        obj._signature = signature
        obj._message = message
        return obj

    @property
    def signature(self):
        return self._signature

    @property
    def message(self):
        return self._message


class VerifyKey(Encodable):
    def __init__(self, key, encoder=RawEncoder):
        key = encoder.decode(key)
        if len(key) != PUBLICKEY_BYTES:
            raise ValueError('The key must be exactly %s bytes long' % PUBLICKEY_BYTES)
        self._key = key

    def __bytes__(self):
        return self._key

    def verify(self, smessage, signature=None, encoder=RawEncoder):
        if signature is not None:
            smessage = signature + smessage
        return crypto_sign_open(encoder.decode(smessage), self._key)


class SigningKey(Encodable):
    def __init__(self, seed, encoder=RawEncoder):
        seed = encoder.decode(seed)
        if len(seed) != SEED_BYTES:
            raise ValueError('The seed must be exactly %d bytes long' % SEED_BYTES)
        pk, _ = _sign(seed, b'')
        self._seed = seed
        self._signing_key = seed + pk
        self.verify_key = VerifyKey(pk)

    def __bytes__(self):
        return self._seed

    @classmethod
    def generate(cls):
        return cls(os.urandom(SEED_BYTES), encoder=RawEncoder)

    def sign(self, message, encoder=RawEncoder):
        _, sig = _sign(self._seed, message)
        signature = encoder.encode(sig)
        body = encoder.encode(message)
        combined = encoder.encode(sig + message)
        return SignedMessage._from_parts(signature, body, combined)


class Signer:
    def __init__(self, key=None):
        if key:
            if not isinstance(key, SigningKey):
                key = SigningKey(seed=key, encoder=RawEncoder if len(key) == 32 else HexEncoder)
        else:
            key = SigningKey.generate()
        self.key = key
        self.keyhex = key.encode(HexEncoder)
        self.keyraw = key.encode(RawEncoder)
        self.verhex = key.verify_key.encode(HexEncoder)
        self.verraw = key.verify_key.encode(RawEncoder)

    def sign(self, msg):
        return self.key.sign(msg)

    def signature(self, msg):
        return self.key.sign(msg).signature


class Verifier:
    """Bool-returning verifier; verify_batch checks many (signature, msg)
    pairs against this key in one GPU call."""

    def __init__(self, key=None):
        if key:
            if not isinstance(key, VerifyKey):
                key = VerifyKey(key, RawEncoder if len(key) == 32 else HexEncoder)
        self.key = key
        if isinstance(self.key, VerifyKey):
            self.keyhex = self.key.encode(HexEncoder)
            self.keyraw = self.key.encode(RawEncoder)
        else:
            self.keyhex = ''
            self.keyraw = ''

    def verify(self, signature, msg):
        if not self.key:
            return False
        try:
            self.key.verify(signature + msg)
        except ValueError:
            return False
        return True

    def verify_batch(self, pairs):
        """[(signature, msg)] -> np.ndarray[bool], same verdicts as verify()."""
        if not self.key:
            return np.zeros(len(pairs), dtype=bool)
        raw = bytes(self.key)
        return verify_signed_batch([(raw, bytes(sig) + bytes(msg)) for sig, msg in pairs])
