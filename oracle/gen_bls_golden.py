"""ORACLE -- BLS COMMIT-check fixture generator (TEST INFRASTRUCTURE, this
container only; nothing here travels to the GPU box, only the JSON it writes).

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_bls_golden.py

Writes tests/golden/bls.json:
  generator       the reference's G2 generator string
                  (crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:19) and its bytes
  msv             MultiSignatureValue(...).as_single_value() of the REFERENCE
                  (crypto/bls/bls_multi_signature.py:48, msgpack of the sorted
                  dict) -- the message every COMMIT's BLS signature covers
                  (plenum/bls/bls_bft_replica_plenum.py:194-210)
  keys            synthetic node keys: sk (32-byte big-endian), pk = sk * g (128 B)
  cases           (signature bytes, message, key index or raw pk bytes, verdict,
                  label): valid signatures and every rejection class the
                  restated decoding has (wrong message / key, bit flips, the point
                  at infinity, x or y >= p, unknown prefixes, compressed forms with
                  both parities, bad lengths, negated points, off-twist keys)

PARITY UNPINNED: the verdicts come from tests/_bn254_py.py's NAIVE pairing
(generic Fp12 arithmetic, one pow by (p^12-1)/r) -- a restatement of python-ursa
0.1.1 / Milagro AMCL BN254, which are absent here; no reference vector exists
for any BLS signature.  Only the generator and the message bytes come from the
reference itself."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, 'shims'), '/root/reference', os.path.join(REPO, 'tests')]

import base58  # noqa: E402  (shim)
from crypto.bls.bls_multi_signature import MultiSignatureValue  # noqa: E402  (reference)

import _bn254_py as bn  # noqa: E402

G_STR = ('3LHpUjiyFC2q2hD7MnwwNmVXiuaFbQx2XkAFJWzswCjgN1utjsCeLzHsKk1nJvFEaS4fcrUmVAkdhtPCYbrVyATZcmzwJReTcJqwqBCPTm'
         'TQ9uWPwz6rEncKb2pYYYFcdHa8N17HzVyTqKfgPi4X9pMetfT3A5xCHq54R2pDNYWVLDX')


def sk_of(i):
    return int.from_bytes(hashlib.sha256(b'plenum-gpu/bls-key' + i.to_bytes(8, 'little')).digest(), 'big') % bn.R


def root(tag, i):
    return base58.b58encode(hashlib.sha256(tag + i.to_bytes(8, 'little')).digest()).decode()


def main():
    gb = base58.b58decode(G_STR)
    g = bn.g2_from_bytes(gb)
    assert g is not None and bn.g2_mul(g, bn.R) is None
    # messages: the reference's MultiSignatureValue serialisation
    msv = []
    for i in range(6):
        v = MultiSignatureValue(ledger_id=i % 4, state_root_hash=root(b'state', i),
                                pool_state_root_hash=root(b'pool', i), txn_root_hash=root(b'txn', i),
                                timestamp=1600000000 + 17 * i)
        msv.append({'ledger_id': v.ledger_id, 'state_root_hash': v.state_root_hash,
                    'pool_state_root_hash': v.pool_state_root_hash, 'txn_root_hash': v.txn_root_hash,
                    'timestamp': v.timestamp, 'single_value': v.as_single_value().hex()})
    msgs = [bytes.fromhex(m['single_value']) for m in msv] + [b'', b'Hello!', bytes(range(256)) * 4]
    keys = []
    for i in range(4):
        sk = sk_of(i)
        keys.append({'sk': sk.to_bytes(32, 'big').hex(), 'pk': bn.g2_to_bytes(bn.g2_mul(g, sk)).hex()})
    pks = [bytes.fromhex(k['pk']) for k in keys]

    def sign(ki, m):
        return bn.g1_to_bytes(bn.g1_mul(bn.hash_to_g1(m), sk_of(ki)))

    cases = []

    def add(label, sig, m, key):
        pk = pks[key] if isinstance(key, int) else key
        verdict = bn.verify_sig(sig, m, pk, gb)
        c = {'label': label, 'sig': sig.hex(), 'msg': m.hex(), 'verdict': verdict}
        if isinstance(key, int):
            c['key'] = key
        else:
            c['pk'] = key.hex()
        cases.append(c)
        print(label, verdict, flush=True)

    for j, m in enumerate(msgs):
        add('valid/msg{}'.format(j), sign(j % 4, m), m, j % 4)
    s0 = sign(0, msgs[0])
    add('wrong_message', s0, msgs[1], 0)
    add('wrong_key', s0, msgs[0], 1)
    add('other_signer_same_message', sign(2, msgs[0]), msgs[0], 0)
    flip = bytearray(s0)
    flip[20] ^= 4
    add('x_bit_flip', bytes(flip), msgs[0], 0)
    flip = bytearray(s0)
    flip[50] ^= 1
    add('y_bit_flip', bytes(flip), msgs[0], 0)
    x, y = bn.g1_from_bytes(s0)
    add('negated', bn.g1_to_bytes((x, (-y) % bn.P)), msgs[0], 0)
    add('zero_bytes_is_infinity', bytes(128), msgs[0], 0)
    add('x_ge_p', b'\x04' + (bn.P + 5).to_bytes(32, 'big') + s0[33:], msgs[0], 0)
    add('y_ge_p', s0[:33] + (y + bn.P).to_bytes(32, 'big') + s0[65:], msgs[0], 0)
    add('prefix_05', b'\x05' + s0[1:], msgs[0], 0)
    par = y & 1
    add('compressed_right_parity', bytes([2 | par]) + s0[1:33] + bytes(95), msgs[0], 0)
    add('compressed_wrong_parity', bytes([2 | (1 - par)]) + s0[1:33] + bytes(95), msgs[0], 0)
    add('trailing_bytes_ignored', s0[:65] + bytes(range(63)), msgs[0], 0)
    add('length_127', s0[:127], msgs[0], 0)
    add('length_129', s0 + b'\x00', msgs[0], 0)
    off_twist = bytearray(pks[0])
    off_twist[127] ^= 1
    add('off_twist_key_valid_sig', s0, msgs[0], bytes(off_twist))
    add('off_twist_key_infinity_sig', bytes(128), msgs[0], bytes(off_twist))
    # a compressed x whose x^3 + 2 is not a square
    xx = 5
    while bn.is_qr(xx ** 3 + 2):
        xx += 1
    add('compressed_nonsquare', b'\x02' + xx.to_bytes(32, 'big') + bytes(95), msgs[0], 0)
    out = {'generator': G_STR, 'generator_hex': gb.hex(), 'msv': msv, 'keys': keys, 'cases': cases,
           'source': 'oracle/gen_bls_golden.py (verdicts: tests/_bn254_py.py naive pairing; parity unpinned)'}
    path = os.path.join(REPO, 'tests', 'golden', 'bls.json')
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(path, len(cases), 'cases')


if __name__ == '__main__':
    main()
