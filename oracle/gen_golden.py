"""ORACLE — golden-fixture generator (TEST INFRASTRUCTURE, this container only).

Runs the REFERENCE's own Python (imported read-only from /root/reference through
the local shims in oracle/shims/) and the libsodium 1.0.18
binary (/opt/conda/lib/libsodium.so.23, the library libnacl 1.6.1 binds) to
produce the committed fixtures under tests/golden/.  Nothing here travels to or
runs on the GPU box; the fixtures it writes are plain data (JSON / npz without
pickles).

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

Fixtures
  kat.json              reference test KATs: DidVerifier abbreviated verkey
                        (plenum/test/common/test_verifier.py:6-28), signing
                        serializer (common/test/test_signing_serializer.py:8-38),
                        the PROPAGATE Ed25519 vector
                        (plenum/test/node_request/message_request/test_valid_message_request.py:86-91),
                        Quorums(n) (plenum/server/quorums.py:15-39)
  plenum_requests.json  C1-format requests through CoreAuthNr.authenticate
                        (plenum/server/client_authn.py:230-266) and
                        ReqAuthenticator.authenticate (plenum/server/req_authenticator.py:23-51):
                        result or exception class + str(), plus per-signature M/pk/sig
  raw_vectors.npz       random (pk, sig, M) with M in 0..4 KiB, ~5 % tampered,
                        verdict = libsodium crypto_sign_verify_detached
  adversarial.npz       SURVEY.md Appendix C.3 classes as sm = sig||M, verdict =
                        libsodium crypto_sign_open (framing included)
  tally.npz             25-node COMMIT batches: sender, verdict -> quorum bits via
                        the reference Commits/Quorums (plenum/server/models.py:91-114)
  merkle.json           Merkle Tree Hash roots (ledger/tree_hasher.py TreeHasher.hash_full_tree,
                        checked against CompactMerkleTree.extend) over leaves of every length
                        around the SHA-256 block boundaries, leaf and child hashes
  propagate.json        PROPAGATE f+1 quorums (row f4): streams of PROPAGATEs (re-sent,
                        duplicate and non-str senders, tampered and re-signed requests)
                        through the reference Requests.add_propagate /
                        req_with_acceptable_quorum (plenum/server/propagator.py:20-46,
                        111-134) with Quorums(n).propagate; a PROPAGATE reaches
                        add_propagate only if ReqAuthenticator.authenticate accepts its
                        request (Node.validateNodeMsg -> verifySignature, node.py:2624-2655)
  c1_10k.json           BASELINE configs[0] at full size: the 10,000 requests of
                        plenum_gpu.synth.c1_requests (seed / payload spec of SURVEY.md
                        8(d)), signed here by the reference DidSigner, with the
                        mutations tests/test_gpu_c1.py applies (reqId changed after
                        signing, a non-base58 character, a truncated signature,
                        identifiers never registered), through the reference
                        CoreAuthNr(['buy'], [], []).authenticate: every failure's
                        exception class + text, a digest of the successes, and a
                        digest of the request dicts (so the GPU-side regeneration is
                        checked to be the same input)
  ingress.json          one node service pass for the batched-ingestion path (f1):
                        client requests of every shape with the reference
                        Request(**req).key (plenum/common/request.py:82-120) and the
                        ReqAuthenticator outcome, PROPAGATE and BATCH wire dicts
                        (Propagate/Batch._asdict, plenum/common/messages/node_messages.py)

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py [fixture ...]   (default: all)
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, 'tests', 'golden')
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, 'shims'), '/root/reference']

import numpy as np  # noqa: E402

import base58  # noqa: E402  (shim)
import libnacl  # noqa: E402  (shim over libsodium 1.0.18)
from common.serializers.serialization import serialize_msg_for_signing  # noqa: E402
from plenum.common.messages.node_messages import Commit  # noqa: E402
from plenum.common.signer_did import DidSigner  # noqa: E402
from plenum.common.verifier import DidVerifier  # noqa: E402
from plenum.server.client_authn import CoreAuthNr  # noqa: E402
from plenum.server.models import Commits  # noqa: E402
from plenum.server.quorums import Quorums  # noqa: E402
from plenum.server.req_authenticator import ReqAuthenticator  # noqa: E402

NA = libnacl.nacl
NA.sodium_version_string.restype = ctypes.c_char_p
assert NA.sodium_version_string() == b'1.0.18'


def sodium_verify(sig64, msg, pk):
    return NA.crypto_sign_verify_detached(sig64, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def sodium_open(sm, pk):
    try:
        libnacl.crypto_sign_open(sm, pk)
        return True
    except ValueError:
        return False


def sodium_keypair(seed):
    return libnacl.crypto_sign_seed_keypair(seed)


def sodium_sign(msg, sk):
    return libnacl.crypto_sign(msg, sk)[:64]


# ----------------------------------------------- tiny Ed25519 for crafting
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def inv(x):
    return pow(x, P - 2, P)


def recover_x(y, sign):
    if y >= P:
        return None
    x2 = (y * y - 1) * inv(D * y * y + 1) % P
    if x2 == 0:
        return None if sign else 0
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P != 0:
        x = x * SQRTM1 % P
    if (x * x - x2) % P != 0:
        return None
    if (x & 1) != sign:
        x = P - x
    return x


def pt_add(p, q):
    (x1, y1), (x2, y2) = p, q
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + x2 * y1) * inv(1 + t) % P
    y3 = (y1 * y2 + x1 * x2) * inv(1 - t) % P
    return (x3, y3)


IDENT = (0, 1)


def pt_mul(p, k):
    r = IDENT
    while k:
        if k & 1:
            r = pt_add(r, p)
        p = pt_add(p, p)
        k >>= 1
    return r


def pt_neg(p):
    return ((-p[0]) % P, p[1])


def encode(p):
    x, y = p
    return (y | ((x & 1) << 255)).to_bytes(32, 'little')


def decode(s):
    v = int.from_bytes(s, 'little')
    y = v & ((1 << 255) - 1)
    x = recover_x(y, v >> 255)
    return None if x is None else (x, y)


BASE = decode(bytes.fromhex('58' + '66' * 31))
T8 = decode(bytes.fromhex('26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05'))
assert pt_mul(T8, 8) == IDENT and pt_mul(T8, 4) != IDENT


def h_int(R, A, M):
    return int.from_bytes(hashlib.sha512(R + A + M).digest(), 'little') % L


def secret_scalar(seed):
    h = bytearray(hashlib.sha512(seed).digest())
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    return int.from_bytes(h[:32], 'little'), bytes(h[32:])


# ------------------------------------------------------------------ helpers
def det_seed(tag, i):
    return hashlib.sha512(tag + struct.pack('<Q', i)).digest()[:32]


def det_bytes(tag, i, n):
    out = b''
    c = 0
    while len(out) < n:
        out += hashlib.sha512(tag + struct.pack('<QQ', i, c)).digest()
        c += 1
    return out[:n]


def exc_record(ex):
    return {'exc': type(ex).__name__, 'str': str(ex)}


class DictState:
    """Minimal stand-in for the domain state's get(key, is_committed)."""

    def __init__(self, nyms=None):
        self._d = {}
        for nym, verkey in (nyms or {}).items():
            key = hashlib.sha256(nym.encode()).digest()
            self._d[key] = json.dumps({'verkey': verkey}).encode()

    def get(self, key, isCommitted=True):
        return self._d.get(key)


# ------------------------------------------------------------------- KATs
def gen_kat():
    kat = {}
    # plenum/test/common/test_verifier.py:6-22
    v = DidVerifier('~8zH9ZSyZTFPGJ4ZPL5Rvxx', identifier='99BgFBg35BehzfSADV5nM4')
    kat['did_abbrev'] = {'verkey': '~8zH9ZSyZTFPGJ4ZPL5Rvxx', 'identifier': '99BgFBg35BehzfSADV5nM4',
                         'expected': v.verkey}
    try:
        DidVerifier('FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF')
        kat['did_odd'] = None
    except Exception as ex:
        kat['did_odd'] = {'verkey': 'FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF', **exc_record(ex)}
    # common/test/test_signing_serializer.py:8-38 (inputs restated as JSON-able cases)
    ser_cases = [1, 'aaa', None, {'1': 'a', '2': 'b'}, {'2': 'b', '1': 'a'}, [1, 5, 3, 4, 2],
                 {'1': 'a', '2': 'b', '3': [1, {'2': 'k'}]}, {'1': 'a', '2': 'b', '3': ['1', {'2': 'k'}]},
                 {'a': 1.5, 'b': True, 'c': [None, 'x', {'z': {'y': [1, 2]}}], 'd': {}},
                 {'signature': 'x', 'k': 'v'}]
    kat['serializer'] = [{'in': c, 'out': serialize_msg_for_signing(c).decode()} for c in ser_cases]
    kat['serializer_ignore'] = [{'in': {'signature': 'x', 'k': 'v', 'n': {'signature': 1}},
                                 'ignore': ['signature'],
                                 'out': serialize_msg_for_signing({'signature': 'x', 'k': 'v', 'n': {'signature': 1}},
                                                                  topLevelKeysToIgnore=['signature']).decode()}]
    # test_valid_message_request.py:86-91 : a real Ed25519 vector
    req = {'identifier': '5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC',
           'signature': 'ZbZG68WiaK67eU3CsgpVi85jpgCztW9Yqe7D5ezDUfWbKdiPPVbWq4Tb5m4Ur3jcR5wJ8zmBUZXZudjvMN63Aa9',
           'operation': {'amount': 62, 'type': 'buy'},
           'reqId': 1499782864169193}
    props = []
    for pv in (None, 1, 2):
        r = dict(req)
        if pv is not None:
            r['protocolVersion'] = pv
        to_ser = {k: vv for k, vv in r.items() if k not in ('signature', 'signatures', 'fees')}
        M = serialize_msg_for_signing(to_ser)
        pk = base58.b58decode(r['identifier'])
        sig = base58.b58decode(r['signature'])
        props.append({'request': r, 'M': M.hex(), 'pk': pk.hex(), 'sig': sig.hex(),
                      'verdict': sodium_open(sig + M, pk)})
    kat['propagate_vector'] = props
    kat['quorums'] = [{'n': n, 'f': Quorums(n).f, 'commit': Quorums(n).commit.value,
                       'prepare': Quorums(n).prepare.value, 'propagate': Quorums(n).propagate.value,
                       'weak': Quorums(n).weak.value, 'strong': Quorums(n).strong.value}
                      for n in range(1, 41)]
    pk = bytes.fromhex('58' + '66' * 31)
    kat['basepoint'] = pk.hex()
    return kat


# ------------------------------------------------------- Plenum requests
LETTERS = 'abcdefghijklmnopqrstuvwxyz'


def payload_chars(i, n=256):
    raw = det_bytes(b'plenum-gpu/c1data', i, n)
    return ''.join(LETTERS[b % 26] for b in raw)


def gen_plenum_requests(n_valid=320):
    rnd = random.Random(20261015)
    signers = [DidSigner(seed=det_seed(b'plenum-gpu/c1key', i)) for i in range(n_valid + 64)]
    registry = {}     # identifier -> verkey given to addIdr
    state_nyms = {}   # identifiers only present in the (uncommitted) state
    cases = []

    def base_req(i, s, data=None):
        return {'identifier': s.identifier, 'reqId': 1000 + i,
                'operation': {'type': 'buy', 'data': data if data is not None else payload_chars(i)},
                'protocolVersion': 2}

    for i in range(n_valid):
        s = signers[i]
        registry[s.identifier] = s.verkey
        r = base_req(i, s, payload_chars(i, rnd.choice([0, 1, 17, 256, 256, 256, 700])))
        r['signature'] = s.sign(r)
        kind = 'valid'
        roll = rnd.random()
        if roll < 0.08:
            r['reqId'] += 1
            kind = 'tampered_reqId'
        elif roll < 0.12:
            r['operation']['data'] = 'X' + r['operation']['data'][1:]
            kind = 'tampered_data'
        elif roll < 0.16:
            sig = bytearray(base58.b58decode(r['signature']))
            sig[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
            r['signature'] = base58.b58encode(bytes(sig)).decode()
            kind = 'tampered_sig'
        elif roll < 0.18:
            r['signature'] = r['signature'][:5] + rnd.choice('0OIl') + r['signature'][6:]
            kind = 'bad_base58'
        elif roll < 0.20:
            r['fees'] = [[['UUxx', 1, 3]], {'a': 1}]
            kind = 'fees_excluded'
        elif roll < 0.22:
            sig = base58.b58decode(r['signature'])
            r['signature'] = base58.b58encode(sig[:63]).decode()
            kind = 'sig_63B'
        elif roll < 0.24:
            sig = base58.b58decode(r['signature'])
            r['signature'] = base58.b58encode(sig + b'\x00').decode()
            kind = 'sig_65B'
        elif roll < 0.26:
            r['signature'] = signers[i + 1].sign(r)
            kind = 'wrong_key'
        cases.append({'kind': kind, 'req': r})

    j = n_valid
    # identifiers unknown to the registry but present in uncommitted state (full verkey)
    for _ in range(8):
        s = signers[j]; j += 1
        r = base_req(j, s)
        r['signature'] = s.sign(r)
        state_nyms[s.identifier] = s.full_verkey
        cases.append({'kind': 'state_verkey', 'req': r})
    # identifier nowhere -> CouldNotAuthenticate
    for _ in range(6):
        s = signers[j]; j += 1
        r = base_req(j, s)
        r['signature'] = s.sign(r)
        cases.append({'kind': 'unknown_idr', 'req': r})
    # cryptonym: 32-byte identifier registered with its full verkey
    for _ in range(6):
        s = signers[j]; j += 1
        cryptonym = s.full_verkey
        registry[cryptonym] = cryptonym
        r = {'identifier': cryptonym, 'reqId': 5000 + j,
             'operation': {'type': 'buy', 'data': payload_chars(j)}, 'protocolVersion': 2}
        M = serialize_msg_for_signing(r, topLevelKeysToIgnore=['signature'])
        r['signature'] = base58.b58encode(s.naclSigner.signature(M)).decode()
        cases.append({'kind': 'cryptonym', 'req': r})
    # odd-length verkey registered -> InvalidKey
    for _ in range(3):
        s = signers[j]; j += 1
        registry[s.identifier] = 'FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF'
        r = base_req(j, s)
        r['signature'] = s.sign(r)
        cases.append({'kind': 'invalid_key', 'req': r})
    # multi-signature requests ('signatures' field, no 'signature')
    for m in range(24):
        k = rnd.choice([2, 3, 4])
        group = [signers[rnd.randrange(n_valid)] for _ in range(k)]
        r = {'identifier': group[0].identifier, 'reqId': 9000 + m,
             'operation': {'type': 'buy', 'data': payload_chars(9000 + m, 64)}, 'protocolVersion': 2}
        sigs = {}
        for g in group:
            M = serialize_msg_for_signing(r, topLevelKeysToIgnore=['signature', 'signatures', 'fees'])
            sigs[g.identifier] = base58.b58encode(g.naclSigner.signature(M)).decode()
        kind = 'multi_valid'
        if m % 3 == 1:
            victim = rnd.choice(list(sigs))
            sb = bytearray(base58.b58decode(sigs[victim]))
            sb[0] ^= 0x40
            sigs[victim] = base58.b58encode(bytes(sb)).decode()
            kind = 'multi_one_bad'
        r['signatures'] = sigs
        threshold = None
        if m % 4 == 2:
            threshold = max(1, len(sigs) - 1)
            kind += '_threshold'
        if m % 8 == 7:
            threshold = len(sigs) + 1
            kind += '_threshold_too_high'
        cases.append({'kind': kind, 'req': r, 'threshold': threshold})
    # missing / empty signature, query and unknown types
    s0 = signers[0]
    r = base_req(0, s0)
    cases.append({'kind': 'missing_signature', 'req': dict(r)})
    r2 = dict(r); r2['signature'] = ''
    cases.append({'kind': 'empty_signature', 'req': r2})
    q = {'identifier': s0.identifier, 'reqId': 77, 'operation': {'type': 'get_x'}, 'protocolVersion': 2}
    q['signature'] = s0.sign(q)
    cases.append({'kind': 'query', 'req': q})
    u = {'identifier': s0.identifier, 'reqId': 78, 'operation': {'type': 'zzz'}, 'protocolVersion': 2}
    u['signature'] = s0.sign(u)
    cases.append({'kind': 'unknown_type', 'req': u})

    state = DictState(state_nyms)
    authnr = CoreAuthNr(['buy'], ['get_x'], [], state=state)
    for idr, vk in registry.items():
        authnr.addIdr(idr, vk)
    reqauth = ReqAuthenticator()
    reqauth.register_authenticator(authnr)

    for c in cases:
        req = c['req']
        try:
            res = authnr.authenticate(json.loads(json.dumps(req)), threshold=c.get('threshold'))
            c['core'] = {'result': list(res)}
        except Exception as ex:
            c['core'] = exc_record(ex)
        try:
            res = reqauth.authenticate(json.loads(json.dumps(req)), key='k%d' % id(c))
            c['reqauth'] = {'result': sorted(res)}
        except Exception as ex:
            c['reqauth'] = exc_record(ex)
        # the per-signature raw triples the verifier sees
        to_ser = {k: v for k, v in req.items() if k not in ('signature', 'signatures', 'fees')}
        M = serialize_msg_for_signing(to_ser)
        c['M'] = M.hex()
        sigmap = req.get('signatures') or ({req['identifier']: req['signature']} if req.get('signature') else {})
        raw = []
        for idr, sig in sigmap.items():
            vk = registry.get(idr) or state_nyms.get(idr)
            try:
                sig_b = base58.b58decode(sig)
                full = DidVerifier(vk, identifier=idr).verkey
                pk = base58.b58decode(full)
                raw.append({'idr': idr, 'pk': pk.hex(), 'sig': sig_b.hex(), 'verdict': sodium_open(sig_b + M, pk)})
            except Exception:
                continue
        c['raw'] = raw

    return {'registry': registry, 'state_nyms': state_nyms, 'write_types': ['buy'],
            'query_types': ['get_x'], 'action_types': [], 'cases': cases}


# ------------------------------------------------------------ raw vectors
def gen_raw(n=3000):
    rnd = random.Random(7)
    pks, sigs, msgs, verdicts, tampered = [], [], [], [], []
    for i in range(n):
        seed = det_seed(b'plenum-gpu/rawkey', i % 2500)  # some duplicate keys
        pk, sk = sodium_keypair(seed)
        ln = rnd.choice([0, 1, 31, 47, 48, 64, 111, 112, 175, 176, 200, 256, 256, 256, 300, 1000, 4096])
        if rnd.random() < 0.1:
            ln = rnd.randrange(0, 4097)
        M = det_bytes(b'plenum-gpu/rawmsg', i, ln)
        sig = bytearray(sodium_sign(M, sk))
        t = rnd.random() < 0.05
        if t:
            kind = i % 3
            if kind == 0 and ln:
                Mb = bytearray(M); Mb[(i // 3) % ln] ^= 1 << (i % 8); M = bytes(Mb)
            elif kind == 1:
                sig[rnd.randrange(32)] ^= 1 << rnd.randrange(8)
            else:
                sig[32 + rnd.randrange(16)] ^= 1 << rnd.randrange(8)
        sig = bytes(sig)
        pks.append(pk); sigs.append(sig); msgs.append(M); tampered.append(t)
        verdicts.append(sodium_verify(sig, M, pk))
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return dict(pk=np.frombuffer(b''.join(pks), np.uint8).reshape(n, 32),
                sig=np.frombuffer(b''.join(sigs), np.uint8).reshape(n, 64),
                blob=np.frombuffer(b''.join(msgs), np.uint8), off=off,
                verdict=np.array(verdicts, np.uint8), tampered=np.array(tampered, np.uint8))


# -------------------------------------------------------- adversarial set
SMALL_ORDER = [bytes(32), (1).to_bytes(32, 'little'),
               bytes.fromhex('26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05'),
               bytes.fromhex('c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a'),
               (P - 1).to_bytes(32, 'little'), P.to_bytes(32, 'little'), (P + 1).to_bytes(32, 'little')]


def gen_adversarial():
    rnd = random.Random(99)
    rows = []   # (label, pk, sm)

    def add(label, pk, sm):
        rows.append((label, bytes(pk), bytes(sm)))

    def honest(i, mlen=64):
        seed = det_seed(b'plenum-gpu/advkey', i)
        pk, sk = sodium_keypair(seed)
        M = det_bytes(b'plenum-gpu/advmsg', i, mlen)
        return pk, sk, M, sodium_sign(M, sk)

    pk, sk, M, sig = honest(0)
    add('valid', pk, sig + M)
    S = int.from_bytes(sig[32:], 'little')
    # canonical S
    for name, sv in [('S=L-1', L - 1), ('S=L', L), ('S=L+1', L + 1), ('S+L', S + L), ('S=2^253-1', 2 ** 253 - 1),
                     ('S=2^256-1', 2 ** 256 - 1), ('S=0', 0)]:
        add('canonical_' + name, pk, sig[:32] + sv.to_bytes(32, 'little') + M)
    # blocklist as R and as A, top bit 0/1
    for k, enc in enumerate(SMALL_ORDER):
        for top in (0, 1):
            e = bytearray(enc); e[31] = (e[31] & 0x7f) | (top << 7); e = bytes(e)
            add('blocklist_R_%d_%d' % (k, top), pk, e + sig[32:] + M)
            add('blocklist_A_%d_%d' % (k, top), e, sig + M)
    # near-blocklist (one bit off) must NOT be treated as small order
    for k, enc in enumerate(SMALL_ORDER):
        e = bytearray(enc); e[rnd.randrange(31)] ^= 1 << rnd.randrange(8)
        add('near_blocklist_A_%d' % k, bytes(e), sig + M)
    # A with y >= p (19 values), both sign bits
    for yv in range(P, 2 ** 255):
        for top in (0, 1):
            e = (yv | (top << 255)).to_bytes(32, 'little')
            add('A_y_ge_p_%d_%d' % (yv - P, top), e, sig + M)
    # R with y >= p (never matches)
    for yv in (P + 2, P + 5, 2 ** 255 - 1):
        add('R_y_ge_p_%d' % (yv - P), pk, yv.to_bytes(32, 'little') + sig[32:] + M)
    # non-square y for A
    cnt = 0
    while cnt < 24:
        yv = rnd.randrange(P)
        if recover_x(yv, 0) is None and yv not in (0,):
            top = cnt & 1
            add('A_nonsquare_%d' % cnt, (yv | (top << 255)).to_bytes(32, 'little'), sig + M)
            cnt += 1
    # A with x == 0 and sign bit 1 (y = 1 / p-1 are blocklisted) ; random sign flips
    for i in range(1, 9):
        pk_i, sk_i, M_i, sig_i = honest(i)
        flipped = bytearray(pk_i); flipped[31] ^= 0x80
        add('A_sign_flipped_%d' % i, bytes(flipped), sig_i + M_i)
    # mixed order: A' = aB + T, T of order 2/4/8; honest S over A' bytes
    torsion = [pt_mul(T8, k) for k in range(1, 8)]
    for ti, T in enumerate(torsion):
        for trial_target in ('accept', 'reject'):
            seed = det_seed(b'plenum-gpu/mixkey', ti * 2 + (trial_target == 'reject'))
            a, prefix = secret_scalar(seed)
            Ap = pt_add(pt_mul(BASE, a), T)
            Ab = encode(Ap)
            for ctr in range(400):
                Mx = det_bytes(b'plenum-gpu/mixmsg', ti * 1000 + ctr, 40)
                r = int.from_bytes(hashlib.sha512(prefix + Mx).digest(), 'little') % L
                Rb = encode(pt_mul(BASE, r))
                h = h_int(Rb, Ab, Mx)
                want = pt_mul(T, h) == IDENT
                if want == (trial_target == 'accept'):
                    Sv = (r + h * a) % L
                    add('mixed_A_T%d_%s' % (ti + 1, trial_target), Ab, Rb + Sv.to_bytes(32, 'little') + Mx)
                    break
    # mixed-order R with mixed-order A: R' = rB + Tc with Tc == -h*T  -> accept
    for ti, T in enumerate(torsion):
        seed = det_seed(b'plenum-gpu/mixRkey', ti)
        a, prefix = secret_scalar(seed)
        Ap = pt_add(pt_mul(BASE, a), T)
        Ab = encode(Ap)
        done = {'accept': False, 'reject': False}
        for ctr in range(2000):
            Mx = det_bytes(b'plenum-gpu/mixRmsg', ti * 10000 + ctr, 33)
            r = rnd.randrange(1, L)
            Tc = torsion[(ctr + ti) % 7]
            Rp = pt_add(pt_mul(BASE, r), Tc)
            Rb = encode(Rp)
            h = h_int(Rb, Ab, Mx)
            ok = pt_add(Tc, pt_mul(T, h)) == IDENT
            key = 'accept' if ok else 'reject'
            if not done[key]:
                Sv = (r + h * a) % L
                add('mixed_RA_T%d_%s' % (ti + 1, key), Ab, Rb + Sv.to_bytes(32, 'little') + Mx)
                done[key] = True
            if all(done.values()):
                break
    # mixed-order R with a prime-order A (always reject)
    for ti, T in enumerate(torsion[:3]):
        pk_i, sk_i, M_i, sig_i = honest(20 + ti)
        a, prefix = secret_scalar(det_seed(b'plenum-gpu/advkey', 20 + ti))
        r = rnd.randrange(1, L)
        Rb = encode(pt_add(pt_mul(BASE, r), T))
        h = h_int(Rb, pk_i, M_i)
        Sv = (r + h * a) % L
        add('mixed_R_T%d' % (ti + 1), pk_i, Rb + Sv.to_bytes(32, 'little') + M_i)
    # torsion-only A that is NOT blocklisted? (all 8-torsion encodings are in the list; T of order 2 = p-1)
    # h == 0 mod L is infeasible; S = 0 with R = -hA: craft R so encode(-hA) == R
    for i in range(3):
        pk_i, sk_i, M_i, sig_i = honest(40 + i)
        a, _ = secret_scalar(det_seed(b'plenum-gpu/advkey', 40 + i))
        # S = 0 is canonical; R' = -h A depends on R (through h): pick R random, check reject
        add('S_zero_%d' % i, pk_i, sig_i[:32] + bytes(32) + M_i)
    # duplicate keys: same pk, many messages, one bad
    pk_d, sk_d, _, _ = honest(60)
    for i in range(6):
        Mi = det_bytes(b'plenum-gpu/dupmsg', i, 50 + i)
        si = bytearray(sodium_sign(Mi, sk_d))
        if i == 3:
            si[40] ^= 2
        add('dup_key_%d' % i, pk_d, bytes(si) + Mi)
    # signature length quirks through the sig||msg concatenation
    pk_s, sk_s, M_s, sig_s = honest(70, 80)
    for sl in (0, 1, 63, 65, 96):
        if sl <= 64:
            sm = (sig_s + M_s)[:sl] if sl < 64 else sig_s + M_s
        else:
            sm = sig_s + bytes(sl - 64) + M_s
        add('siglen_%d' % sl, pk_s, sm)
    # crafted: a valid signature over M' where sig||M' == sig65||M  (shifted byte)
    add('siglen_shift_valid', pk_s, sig_s + M_s)
    # message lengths at the SHA-512 block boundaries of R||A||M and large messages
    for i, ml in enumerate([0, 1, 47, 48, 49, 111, 112, 175, 176, 177, 239, 240, 4096, 65536, 131072]):
        pk_i, sk_i, M_i, sig_i = honest(100 + i, ml)
        add('mlen_%d' % ml, pk_i, sig_i + M_i)
        if ml:
            Mb = bytearray(M_i); Mb[-1] ^= 1
            add('mlen_%d_tampered' % ml, pk_i, sig_i + bytes(Mb))
    labels, pks, sms = zip(*rows)
    verdict = [sodium_open(sm, pkk) for _, pkk, sm in rows]
    off = np.zeros(len(rows) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in sms])
    return dict(label=np.array(labels), pk=np.frombuffer(b''.join(pks), np.uint8).reshape(-1, 32),
                sm_blob=np.frombuffer(b''.join(sms), np.uint8), sm_off=off,
                verdict=np.array(verdict, np.uint8))


# ------------------------------------------------------------------- tally
def gen_tally(n_batches=500, n_nodes=25):
    quorums = Quorums(n_nodes)
    keys = [sodium_keypair(det_seed(b'plenum-gpu/node', j)) for j in range(n_nodes)]
    names = ['Node%d' % (j + 1) for j in range(n_nodes)]
    rnd = random.Random(3)
    senders, pks, sigs, msgs, verdicts, batch_off = [], [], [], [], [], [0]
    commit_reached, prepare_reached, vote_count = [], [], []
    for b in range(n_batches):
        commit = Commit(0, 0, b + 1)
        M = serialize_msg_for_signing(dict(commit.items()) | {'op': 'COMMIT'})
        assert M == b'instId:0|op:COMMIT|ppSeqNo:%d|viewNo:0' % (b + 1)
        k_b = hashlib.sha512(b'plenum-gpu/k' + struct.pack('<Q', b)).digest()[0] % 13
        order = list(range(n_nodes))
        rnd.shuffle(order)
        bad = set(order[:k_b])
        slots = list(range(n_nodes))
        if rnd.random() < 0.05:       # one duplicate sender replaces another node's message
            victim, dup = rnd.sample(range(n_nodes), 2)
            slots[victim] = dup
        commits = Commits()
        for j in slots:
            pk, sk = keys[j]
            sig = bytearray(sodium_sign(M, sk))
            if j in bad:
                sig[rnd.randrange(64)] ^= 1 << rnd.randrange(8)
            sig = bytes(sig)
            v = sodium_verify(sig, M, pk)
            if v:
                commits.addVote(commit, names[j])
            senders.append(j); pks.append(pk); sigs.append(sig); msgs.append(M); verdicts.append(v)
        batch_off.append(len(senders))
        vote_count.append(commits._votes_count(commit))
        commit_reached.append(commits.hasQuorum(commit, quorums.commit.value))
        prepare_reached.append(commits.hasQuorum(commit, quorums.prepare.value))
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return dict(n_nodes=np.array(n_nodes), commit_quorum=np.array(quorums.commit.value),
                prepare_quorum=np.array(quorums.prepare.value),
                sender=np.array(senders, np.uint32), batch_off=np.array(batch_off, np.uint64),
                pk=np.frombuffer(b''.join(pks), np.uint8).reshape(-1, 32),
                sig=np.frombuffer(b''.join(sigs), np.uint8).reshape(-1, 64),
                blob=np.frombuffer(b''.join(msgs), np.uint8), off=off,
                verdict=np.array(verdicts, np.uint8), vote_count=np.array(vote_count, np.uint32),
                commit_reached=np.array(commit_reached, np.uint8),
                prepare_reached=np.array(prepare_reached, np.uint8))


def gen_ingress(n=48):
    """One service pass: client requests (single/multi signature, optional
    protocolVersion/taaAcceptance/endorser, tampered, unknown identifier), the
    reference Request.key of each, the reference ReqAuthenticator outcome, and
    PROPAGATE / BATCH wire dicts carrying some of them."""
    from plenum.common.messages.node_messages import Batch, Propagate
    from plenum.common.request import Request
    rnd = random.Random(4242)
    signers = [DidSigner(seed=det_seed(b'plenum-gpu/ingress', i)) for i in range(n + 8)]
    authnr = CoreAuthNr(['buy'], [], [])
    registry = {}
    for s in signers[:n]:
        authnr.addIdr(s.identifier, s.verkey)
        registry[s.identifier] = s.verkey
    ra = ReqAuthenticator()
    ra.register_authenticator(authnr)
    cases = []
    for i in range(n):
        s = signers[i]
        req = {'identifier': s.identifier, 'reqId': 5000 + i,
               'operation': {'type': 'buy', 'data': payload_chars(9000 + i, 40 + i)}, 'protocolVersion': 2}
        kind = ['single', 'single', 'taa', 'endorser', 'multi', 'tampered', 'unknown', 'single'][i % 8]
        if kind == 'taa':
            req['taaAcceptance'] = {'mechanism': 'x', 'taaDigest': hashlib.sha256(b'taa%d' % i).hexdigest(),
                                    'time': 1600000000 + 86400 * i}
        if kind == 'endorser':
            req['endorser'] = signers[(i + 1) % n].identifier
        if kind == 'unknown':
            s = signers[n + (i % 8)]
            req['identifier'] = s.identifier
        if kind in ('multi', 'endorser'):
            other = signers[(i + 1) % n] if kind == 'endorser' else signers[(i + 3) % n]
            sigs = {}
            for sg in (s, other):
                sigs[sg.identifier] = sg.sign(req)
            req['signatures'] = sigs
        else:
            req['signature'] = s.sign(req)
        if kind == 'tampered':
            req['reqId'] += 1
        key = Request(**req).key
        try:
            out = {'result': sorted(ra.authenticate(json.loads(json.dumps(req)), key=key))}
        except Exception as ex:
            out = exc_record(ex)
        cases.append({'kind': kind, 'req': req, 'key': key, 'reqauth': out})
    props = []
    for i in range(0, n, 3):
        props.append(json.loads(json.dumps(Propagate(cases[i]['req'], 'Client%d' % i)._asdict())))
    batches = []
    for j in range(0, len(props) - 2, 4):
        msgs = [json.dumps(props[j + k]) for k in range(3)]
        batches.append(json.loads(json.dumps(Batch(msgs, None)._asdict())))
    rnd.shuffle(props)
    return {'registry': registry, 'write_types': ['buy'], 'cases': cases, 'propagates': props, 'batches': batches}


def gen_propagate():
    """PROPAGATE streams through the reference Requests store.  Per stream:
    events [sender, case index] in arrival order (sender a node name, or a
    bytes name — the non-str sender the reference filters out), the
    per-request outcome: Requests.votes (every sender), the str-sender count
    and whether req_with_acceptable_quorum(Quorums(n).propagate) returns a
    request (and which sender's copy)."""
    from plenum.common.request import Request
    from plenum.server.propagator import Requests
    rnd = random.Random(777)
    n_clients = 40
    signers = [DidSigner(seed=det_seed(b'plenum-gpu/propagate', i)) for i in range(n_clients)]
    authnr = CoreAuthNr(['buy'], [], [])
    registry = {}
    for sg in signers:
        authnr.addIdr(sg.identifier, sg.verkey)
        registry[sg.identifier] = sg.verkey
    ra = ReqAuthenticator()
    ra.register_authenticator(authnr)
    cases = []
    for i in range(n_clients):
        sg = signers[i]
        req = {'identifier': sg.identifier, 'reqId': 7000 + i,
               'operation': {'type': 'buy', 'data': payload_chars(12000 + i, 24 + i % 17)}, 'protocolVersion': 2}
        req['signature'] = sg.sign(req)
        kind = 'valid'
        if i % 5 == 3:      # tampered in transit: the signature no longer verifies
            req['operation']['data'] += 'x'
            kind = 'tampered'
        cases.append({'kind': kind, 'req': req})
        if i % 7 == 2:      # the client re-signs a second operation under the same reqId
            req2 = {'identifier': sg.identifier, 'reqId': 7000 + i,
                    'operation': {'type': 'buy', 'data': payload_chars(13000 + i, 30)}, 'protocolVersion': 2}
            req2['signature'] = sg.sign(req2)
            cases.append({'kind': 'resigned', 'req': req2})
    for c in cases:
        c['key'] = Request(**c['req']).key
        try:
            ra.authenticate(json.loads(json.dumps(c['req'])))
            c['valid'] = True
        except Exception:
            c['valid'] = False
    streams = []
    for n in (4, 7, 25):
        quorums = Quorums(n)
        names = ['Node%d' % (j + 1) for j in range(n)]
        events = []
        for ci in range(len(cases)):
            # how many distinct nodes propagate this request: around the f+1 boundary
            k = max(0, min(n, quorums.propagate.value + rnd.choice([-2, -1, -1, 0, 0, 1, 3])))
            for j in rnd.sample(range(n), k):
                events.append([names[j], ci])
            if rnd.random() < 0.3:          # a node re-sends its PROPAGATE
                events.append([names[rnd.randrange(n)], ci])
            if rnd.random() < 0.2:          # a non-str (bytes) sender name
                events.append([{'bytes': names[rnd.randrange(n)]}, ci])
        rnd.shuffle(events)
        store = Requests()
        order = []
        for snd, ci in events:
            c = cases[ci]
            if not c['valid']:
                continue                     # verifySignature rejected the PROPAGATE
            sender = snd['bytes'].encode() if isinstance(snd, dict) else snd
            req = Request(**json.loads(json.dumps(c['req'])))
            if req.key not in store:
                order.append(req.key)
            store.add_propagate(req, sender)
        outcome = {}
        for key in order:
            state = store[key]
            got = state.req_with_acceptable_quorum(quorums.propagate)
            str_senders = [s for s in state.propagates if isinstance(s, str)]
            outcome[key] = {'votes': store.votes(state.request), 'str_votes': len(str_senders),
                            'reached': got is not None,
                            'finalised_by': (str_senders[quorums.propagate.value - 1] if got is not None else None)}
            if got is not None:
                assert got is state.propagates[outcome[key]['finalised_by']]
        streams.append({'n': n, 'f': quorums.f, 'quorum': quorums.propagate.value, 'events': events,
                        'order': order, 'outcome': outcome})
    return {'registry': registry, 'write_types': ['buy'], 'cases': cases, 'streams': streams}


def gen_merkle():
    """Merkle Tree Hash roots from the reference ledger/tree_hasher.py TreeHasher
    (and CompactMerkleTree for the incremental form) over deterministic leaves of
    every length around the SHA-256 block boundaries."""
    from ledger.compact_merkle_tree import CompactMerkleTree
    from ledger.tree_hasher import TreeHasher
    th = TreeHasher()
    lens = [0, 1, 2, 31, 32, 54, 55, 56, 62, 63, 64, 65, 118, 119, 120, 127, 128, 129, 255, 256, 1000, 4097]
    leaves = [det_bytes(b'plenum-gpu/merkle', i, lens[i % len(lens)]) for i in range(1030)]
    trees = []
    for size in list(range(0, 70)) + [127, 128, 129, 1000, 1030]:
        cmt = CompactMerkleTree(hasher=th)
        cmt.extend(leaves[:size])
        root = th.hash_full_tree(leaves[:size])
        assert cmt.root_hash == root
        trees.append({'size': size, 'root': root.hex()})
    return {'leaves': [lf.hex() for lf in leaves], 'trees': trees,
            'leaf_hashes': [th.hash_leaf(lf).hex() for lf in leaves[:70]],
            'children': [th.hash_children(leaves[i][:32].ljust(32, b'x'), leaves[i + 1][:32].ljust(32, b'y')).hex()
                         for i in range(0, 20, 2)]}

# ------------------------------------------------------- C1 at 10k (configs[0])
C1_MUTATIONS = {'reqId_plus_1': 'k % 41 == 0', 'bad_base58_first_char': 'k % 173 == 7',
                'sig_minus_3_chars': 'k % 211 == 11', 'never_registered': 'k % 997 == 5'}


def c1_mutate(reqs):
    """tests/test_gpu_c1.py's mutations, in its order"""
    n = len(reqs)
    for k in range(0, n, 41):
        reqs[k]['reqId'] += 1
    for k in range(7, n, 173):
        reqs[k]['signature'] = '0' + reqs[k]['signature'][1:]
    for k in range(11, n, 211):
        reqs[k]['signature'] = reqs[k]['signature'][:-3]
    return reqs


def c1_digest(obj):
    return hashlib.sha256(json.dumps(obj, sort_keys=True, separators=(',', ':')).encode()).hexdigest()


def gen_c1(n=10_000):
    sys.path.insert(0, os.path.join(REPO, 'indy-plenum_amd'))
    from plenum_gpu import synth   # pure seed / payload spec (no GPU)
    reqs, ids = [], []
    for j in range(n):
        sgn = DidSigner(seed=synth.seed(1, j))
        ids.append((sgn.identifier, sgn.verkey))
        data = ''.join(chr(97 + b % 26) for b in synth.message(1, j, 256))
        r = {'identifier': sgn.identifier, 'reqId': j, 'operation': {'type': 'buy', 'data': data},
             'protocolVersion': 2}
        r['signature'] = sgn.sign(r)
        reqs.append(r)
    c1_mutate(reqs)
    authnr = CoreAuthNr(['buy'], [], [])
    for k, (idr, vk) in enumerate(ids):
        if k % 997 != 5:
            authnr.addIdr(idr, vk)
    fails, ok = {}, []
    for k, r in enumerate(reqs):
        try:
            ok.append([k, list(authnr.authenticate(r))])
        except Exception as ex:  # noqa: BLE001 - the outcome is the fixture
            fails[str(k)] = [type(ex).__name__, str(ex)]
    return {'n': n, 'spec': 'plenum_gpu.synth.c1_requests(n) (cfg 1), signed by the reference DidSigner; '
                            'mutations then CoreAuthNr([\'buy\'], [], []).authenticate',
            'mutations': C1_MUTATIONS, 'identities_digest': c1_digest(ids), 'requests_digest': c1_digest(reqs),
            'failures': fails, 'ok_count': len(ok), 'ok_digest': c1_digest(ok)}


GENERATORS = ['kat', 'plenum_requests', 'raw_vectors', 'adversarial', 'tally', 'ingress', 'merkle', 'propagate', 'c1']


def main(which=None):
    which = which or GENERATORS
    os.makedirs(OUT, exist_ok=True)
    if 'kat' in which:
        with open(os.path.join(OUT, 'kat.json'), 'w') as fh:
            json.dump(gen_kat(), fh, indent=1, sort_keys=True)
    if 'plenum_requests' in which:
        with open(os.path.join(OUT, 'plenum_requests.json'), 'w') as fh:
            json.dump(gen_plenum_requests(), fh, indent=0)  # keep dict order: the signature loop order matters
    if 'raw_vectors' in which:
        np.savez_compressed(os.path.join(OUT, 'raw_vectors.npz'), **gen_raw())
    if 'adversarial' in which:
        np.savez_compressed(os.path.join(OUT, 'adversarial.npz'), **gen_adversarial())
    if 'tally' in which:
        np.savez_compressed(os.path.join(OUT, 'tally.npz'), **gen_tally())
    if 'merkle' in which:
        with open(os.path.join(OUT, 'merkle.json'), 'w') as fh:
            json.dump(gen_merkle(), fh, indent=0)
    if 'propagate' in which:
        with open(os.path.join(OUT, 'propagate.json'), 'w') as fh:
            json.dump(gen_propagate(), fh, indent=0)
    if 'c1' in which:
        with open(os.path.join(OUT, 'c1_10k.json'), 'w') as fh:
            json.dump(gen_c1(), fh, indent=0, sort_keys=True)
    if 'ingress' in which:
        with open(os.path.join(OUT, 'ingress.json'), 'w') as fh:
            json.dump(gen_ingress(), fh, indent=0)
    for fn in sorted(os.listdir(OUT)):
        print(fn, os.path.getsize(os.path.join(OUT, fn)))


if __name__ == '__main__':
    main(sys.argv[1:] or None)
