"""DID verifiers (plenum/common/verifier.py:10-54) on the GPU backend.

DidVerifier resolves the 32-byte Ed25519 key from its arguments exactly as the
reference does:
  * cryptonym: a 32-byte identifier with no verkey -> the identifier is the verkey
  * abbreviated verkey '~X'  -> b58(b58d(identifier) + b58d(X))
  * otherwise the verkey is taken as is
An empty verkey raises ValueError; a verkey that does not decode to 32 bytes
raises InvalidKey("verkey <as given>").  verify() is a bool; verify_batch()
checks many (signature, msg) pairs in one GPU call.
"""
from abc import abstractmethod

from .base58 import b58decode, b58encode
from .exceptions import InvalidKey
from .nacl_wrappers import Verifier as NaclVerifier
from .serialization import serialize_msg_for_signing


class Verifier:
    @abstractmethod
    def __init__(self, *args, **kwargs):
        pass

    @abstractmethod
    def verify(self, sig, msg) -> bool:
        pass

    def verifyMsg(self, sig, msg):
        return self.verify(sig, serialize_msg_for_signing(msg))


def resolve_verkey(verkey, identifier=None):
    """The full base58 verkey DidVerifier would use (may raise ValueError)."""
    if identifier:
        raw_idr = b58decode(identifier)
        if len(raw_idr) == 32 and not verkey:
            verkey = identifier
        if not verkey:
            raise ValueError("'verkey' should be a non-empty string")
        if verkey[0] == '~':
            verkey = b58encode(b58decode(identifier) + b58decode(verkey[1:])).decode('utf-8')
    return verkey


class DidVerifier(Verifier):
    def __init__(self, verkey, identifier=None):
        given = verkey
        self._verkey = None
        self._vr = None
        verkey = resolve_verkey(verkey, identifier)
        try:
            self.verkey = verkey
        except Exception as ex:
            raise InvalidKey('verkey {}'.format(given)) from ex

    @property
    def verkey(self):
        return self._verkey

    @verkey.setter
    def verkey(self, value):
        self._verkey = value
        self._vr = NaclVerifier(b58decode(value))

    @property
    def raw_verkey(self):
        """32-byte key bytes (used by the batch prefetch cache)."""
        return self._vr.keyraw if self._vr is not None else None

    def verify(self, sig, msg) -> bool:
        return self._vr.verify(sig, msg)

    def verify_batch(self, pairs):
        return self._vr.verify_batch(pairs)
