"""ORACLE SHIM (test infrastructure, this container only).

Stand-in for libnacl 1.6.1 (absent here), used ONLY by oracle/gen_golden.py to
run the reference's own Plenum code against the libsodium 1.0.18 binary at
/opt/conda/lib/libsodium.so.23.  Restates libnacl 1.6.1's ctypes wrappers for
the functions the reference calls.
"""
import ctypes
import hashlib
import os

nacl = ctypes.CDLL('/opt/conda/lib/libsodium.so.23')
if nacl.sodium_init() < 0:
    raise RuntimeError('sodium_init failed')

crypto_sign_BYTES = nacl.crypto_sign_bytes()
crypto_sign_PUBLICKEYBYTES = nacl.crypto_sign_publickeybytes()
crypto_sign_SECRETKEYBYTES = nacl.crypto_sign_secretkeybytes()
crypto_sign_SEEDBYTES = nacl.crypto_sign_seedbytes()
crypto_box_PUBLICKEYBYTES = 32
crypto_box_SECRETKEYBYTES = 32
crypto_box_NONCEBYTES = 24
crypto_secretbox_KEYBYTES = 32
crypto_secretbox_NONCEBYTES = 24


class CryptError(Exception):
    pass


def randombytes(size):
    return os.urandom(size)


def randombytes_uniform(upper_bound):
    return nacl.randombytes_uniform(ctypes.c_uint32(upper_bound))


def crypto_sign_seed_keypair(seed):
    if len(seed) != crypto_sign_SEEDBYTES:
        raise ValueError('Invalid Seed')
    pk = ctypes.create_string_buffer(crypto_sign_PUBLICKEYBYTES)
    sk = ctypes.create_string_buffer(crypto_sign_SECRETKEYBYTES)
    if nacl.crypto_sign_seed_keypair(pk, sk, seed):
        raise CryptError('Failed to generate keypair')
    return pk.raw, sk.raw


def crypto_sign(msg, sk):
    if len(sk) != crypto_sign_SECRETKEYBYTES:
        raise ValueError('Invalid secret key')
    sig = ctypes.create_string_buffer(len(msg) + crypto_sign_BYTES)
    slen = ctypes.pointer(ctypes.c_ulonglong())
    if nacl.crypto_sign(sig, slen, msg, ctypes.c_ulonglong(len(msg)), sk):
        raise ValueError('Failed to sign message')
    return sig.raw


def crypto_sign_open(sig, vk):
    msg = ctypes.create_string_buffer(len(sig))
    msglen = ctypes.c_ulonglong()
    ret = nacl.crypto_sign_open(msg, ctypes.pointer(msglen), sig, ctypes.c_ulonglong(len(sig)), vk)
    if ret:
        raise ValueError('Failed to validate message')
    return msg.raw[:msglen.value]


def crypto_hash_sha256(msg):
    return hashlib.sha256(msg).digest()
