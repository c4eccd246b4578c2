"""ORACLE SHIM: plenum/common/util.py imports libnacl.secret; never used on the verify path."""


class SecretBox:
    def __init__(self, key=None):
        raise NotImplementedError('SecretBox is not available in the oracle shim')
