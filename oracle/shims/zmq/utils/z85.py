"""ORACLE SHIM: z85 is imported by plenum/common/util.py, unused on the verify path."""


def encode(b):
    raise NotImplementedError


def decode(s):
    raise NotImplementedError
