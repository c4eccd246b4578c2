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

Layouts (csrc/pv_kernels.hip k_synth_len / k_synth / k_synth_fill):
    FIXED  (C2)  len(M_i) = mlen
    RANGE  (C4)  len(M_i) = lo + u32le(SHA-512("plenum-gpu/len" || cfg || u64le(i))[0:4]) mod (hi - lo + 1)
    COMMIT (C3)  signature i = the COMMIT vote in slot s = i mod n of 3PC batch b = i div n:
                 M = "instId:0|op:COMMIT|ppSeqNo:<b+1>|viewNo:0"
                 k_b  = SHA-512("plenum-gpu/k" || u64le(b))[0] mod 13    invalid votes in the batch
                 d    = SHA-512("plenum-gpu/c3" || 3 || u64le(b))
                 r_b  = d[0] mod n                                       first invalid slot (a run of k_b, cyclic)
                 dup  = u16le(d[1:3]) < 655 (~1 %): slot victim = d[3] mod n carries node
                        (victim + 1 + d[4] mod (n-1)) mod n's vote instead of its own
                 sender(b, s) signs with seed(3, sender); invalid slots get the tamper flip above.
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


FIXED, RANGE, COMMIT = 0, 1, 2


def msg_len(mode, cfg, i, lo, hi, n_nodes=25):
    if mode == FIXED:
        return lo
    if mode == COMMIT:
        return len(commit_message(i // n_nodes + 1))
    return lo + struct.unpack('<I', _h(b'plenum-gpu/len', cfg, i)[:4])[0] % (hi - lo + 1)


def c3_batch(b, n_nodes):
    """(r_b, k_b, dup_on, victim, dup) of 3PC batch b."""
    d = hashlib.sha512(b'plenum-gpu/c3' + bytes([3]) + struct.pack('<Q', b)).digest()
    k = c3_invalid_count(b)
    dup_on = n_nodes > 1 and (d[1] | (d[2] << 8)) < 655
    victim = d[3] % n_nodes
    dup = (victim + 1 + d[4] % (n_nodes - 1)) % n_nodes if n_nodes > 1 else 0
    return d[0] % n_nodes, k, dup_on, victim, dup


def c3_slots(b, n_nodes):
    """senders (n_nodes,) and invalid flags (n_nodes,) of batch b."""
    r, k, dup_on, victim, dup = c3_batch(b, n_nodes)
    senders = np.arange(n_nodes, dtype=np.uint32)
    if dup_on:
        senders[victim] = dup
    bad = ((np.arange(n_nodes) - r) % n_nodes) < k
    return senders, bad


def c3_expected(first_batch, n_batches, n_nodes, quorum):
    """votes (distinct valid senders) and quorum-reached per batch, from the spec alone."""
    votes = np.zeros(n_batches, np.uint32)
    for j in range(n_batches):
        senders, bad = c3_slots(first_batch + j, n_nodes)
        votes[j] = len(set(senders[~bad].tolist()))
    return votes, votes >= quorum


def host_batch_ex(mode, cfg, first, n, lo, hi=None, key_mod=0, n_nodes=25):
    """seeds, msgs, tamper, senders for signatures first..first+n-1 (unsigned) in any layout."""
    hi = lo if hi is None else hi
    seeds, msgs, tamper, senders = [], [], [], []
    for j in range(n):
        i = first + j
        if mode == COMMIT:
            b, s = divmod(i, n_nodes)
            snd, bad = c3_slots(b, n_nodes)
            senders.append(int(snd[s]))
            tamper.append(bool(bad[s]))
            seeds.append(seed(cfg, int(snd[s])))
            msgs.append(commit_message(b + 1))
        else:
            senders.append(0)
            tamper.append(tampered(cfg, i))
            seeds.append(seed(cfg, i, key_mod))
            msgs.append(message(cfg, i, msg_len(mode, cfg, i, lo, hi)))
    return (np.frombuffer(b''.join(seeds), np.uint8).reshape(n, 32), msgs, np.array(tamper, dtype=bool),
            np.array(senders, np.uint32))


# ---------------------------------------------------------------- C1 requests
def c1_identity(pk):
    """DidSigner(seed) identity for raw key pk: (identifier, abbreviated verkey)
    (plenum/common/signer_did.py: identifier = b58(vk[:16]), verkey = '~' + b58(vk[16:]))."""
    from .base58 import b58encode
    return b58encode(pk[:16]).decode(), '~' + b58encode(pk[16:]).decode()


def c1_requests(n, first=0, cfg=1):
    """BASELINE configs[0]: n signed write requests
    {'identifier', 'reqId', 'operation': {'type': 'buy', 'data': 256 chars a-z}, 'protocolVersion': 2}
    signed by DidSigner(seed_i) (GPU batch signer).  Returns (requests, [(identifier, verkey)])."""
    from .base58 import b58encode
    from .nacl_wrappers import sign_batch
    from .serialization import serialize_msg_for_signing
    seeds = [seed(cfg, first + j) for j in range(n)]
    pk, _ = sign_batch(seeds, [b''] * n)
    ids = [c1_identity(pk[j].tobytes()) for j in range(n)]
    reqs = []
    for j in range(n):
        data = ''.join(chr(97 + b % 26) for b in message(cfg, first + j, 256))
        reqs.append({'identifier': ids[j][0], 'reqId': first + j, 'operation': {'type': 'buy', 'data': data},
                     'protocolVersion': 2})
    _, sig = sign_batch(seeds, [serialize_msg_for_signing(r) for r in reqs])
    for j in range(n):
        reqs[j]['signature'] = b58encode(sig[j].tobytes()).decode()
    return reqs, ids
