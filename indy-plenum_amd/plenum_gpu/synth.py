"""Deterministic synthetic workload.

Host restatement of the device generator (k_synth / k_synth_fill / k_tamper in
csrc/pv_kernels.hip) so tests can check the device output byte for byte on
small index ranges.  All hashes are SHA-512 over a single block:

    seed_i   = SHA-512("plenum-gpu/key"    || cfg || u64le(key_i))[0:32]
               key_i = i % key_mod if key_mod else i
    M_i      = SHA-512("plenum-gpu/msg"    || cfg || u64le(i) || u64le(c))  c = 0, 1, ...
               concatenated and truncated to mlen bytes
    tamper_i = u32le(SHA-512("plenum-gpu/tamper" || cfg || u64le(i))[0:4]) < 214748365   (~5.0 %)
    tamper kind (i mod 3): 0 flip bit (i mod 8) of M byte (i/3) mod len(M)
                           1 flip bit (i mod 8) of R byte (i/3) mod 32
                           2 flip bit (i mod 8) of S byte (i/3) mod 16
"""
import hashlib
import struct

import numpy as np

TAMPER_THRESHOLD = 214748365


def _h(tag, cfg, i, c=None):
    data = tag + bytes([cfg & 0xff]) + struct.pack('<Q', i)
    if c is not None:
        data += struct.pack('<Q', c)
    return hashlib.sha512(data).digest()


def seed(cfg, i, key_mod=0):
    return _h(b'plenum-gpu/key', cfg, i % key_mod if key_mod else i)[:32]


def message(cfg, i, mlen):
    out = b''
    c = 0
    while len(out) < mlen:
        out += _h(b'plenum-gpu/msg', cfg, i, c)
        c += 1
    return out[:mlen]


def tampered(cfg, i):
    return struct.unpack('<I', _h(b'plenum-gpu/tamper', cfg, i)[:4])[0] < TAMPER_THRESHOLD


def apply_tamper(i, msg, sig):
    """Return (msg, sig) with the spec's single-bit flip applied."""
    msg = bytearray(msg)
    sig = bytearray(sig)
    bit = 1 << (i % 8)
    kind = i % 3
    if kind == 0 and len(msg):
        msg[(i // 3) % len(msg)] ^= bit
    elif kind == 1 or (kind == 0 and not len(msg)):
        sig[(i // 3) % 32] ^= bit
    else:
        sig[32 + (i // 3) % 16] ^= bit
    return bytes(msg), bytes(sig)


def host_batch(cfg, first, n, mlen, key_mod=0):
    """seeds (n,32), msgs list, tamper (n,) for indices first..first+n-1 (unsigned)."""
    seeds = np.frombuffer(b''.join(seed(cfg, first + j, key_mod) for j in range(n)), np.uint8).reshape(n, 32)
    msgs = [message(cfg, first + j, mlen) for j in range(n)]
    tamper = np.array([tampered(cfg, first + j) for j in range(n)], dtype=bool)
    return seeds, msgs, tamper


# ---------------------------------------------------------------- C3 COMMITs
COMMIT_FMT = 'instId:0|op:COMMIT|ppSeqNo:{}|viewNo:0'


def commit_message(pp_seq_no):
    """serialize_msg_for_signing(Commit(0, 0, ppSeqNo))."""
    return COMMIT_FMT.format(pp_seq_no).encode()


def c3_invalid_count(b):
    """k_b = SHA-512("plenum-gpu/k" || u64le(b))[0] mod 13."""
    return hashlib.sha512(b'plenum-gpu/k' + struct.pack('<Q', b)).digest()[0] % 13
