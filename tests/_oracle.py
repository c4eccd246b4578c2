"""ctypes access to the ORACLE (oracle/liboracle.so) — the checker, tests only."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, 'oracle', 'liboracle.so')
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            subprocess.run(['make', '-s', '-C', os.path.join(REPO, 'oracle')], check=True)
        _lib = ctypes.CDLL(SO)
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def padded(blob):
    return np.concatenate([np.asarray(blob, np.uint8), np.zeros(16, np.uint8)])


def verify_batch(pk, sig, blob, off):
    n = len(pk)
    v = np.zeros(n, np.uint8)
    if n:
        pk = np.ascontiguousarray(pk, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        b = padded(blob)
        off = np.ascontiguousarray(off, np.uint64)
        lib().oracle_verify_batch(_p(pk), _p(sig), _p(b), _p(off), ctypes.c_uint64(n), _p(v))
    return v.astype(bool)


def sign_open(sm, pk):
    return lib().oracle_sign_open(sm, ctypes.c_uint64(len(sm)), pk) == 0


def sign_batch(seeds, blob, off):
    n = len(seeds)
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    seeds = np.ascontiguousarray(seeds, np.uint8)
    b = padded(blob)
    off = np.ascontiguousarray(off, np.uint64)
    lib().oracle_sign_batch(_p(seeds), _p(b), _p(off), ctypes.c_uint64(n), _p(pk), _p(sig))
    return pk, sig


def sha512(m):
    out = ctypes.create_string_buffer(64)
    lib().oracle_sha512(m, ctypes.c_uint64(len(m)), out)
    return out.raw


def hram(sig, pk, m):
    out = ctypes.create_string_buffer(32)
    lib().oracle_hram(sig, pk, m, ctypes.c_uint64(len(m)), out)
    return out.raw
