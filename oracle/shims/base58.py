"""ORACLE SHIM (test infrastructure): base58 2.x semantics (Bitcoin alphabet,
leading zero bytes <-> leading '1', b58decode strips trailing whitespace,
ValueError on an invalid character).  base58 is unpinned by the reference
(setup.py:98-99) and absent here; restated from its published behaviour."""
BITCOIN_ALPHABET = b'123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
alphabet = BITCOIN_ALPHABET
_MAP = {c: i for i, c in enumerate(BITCOIN_ALPHABET)}


def _scrub(v):
    if isinstance(v, str):
        v = v.encode('ascii')
    return bytes(v)


def b58encode_int(i, default_one=True, alphabet=BITCOIN_ALPHABET):
    if not i and default_one:
        return alphabet[0:1]
    out = b''
    while i:
        i, idx = divmod(i, 58)
        out = alphabet[idx:idx + 1] + out
    return out


def b58encode(v, alphabet=BITCOIN_ALPHABET):
    v = _scrub(v)
    n0 = len(v) - len(v.lstrip(b'\0'))
    acc = int.from_bytes(v, 'big')
    return alphabet[0:1] * n0 + b58encode_int(acc, default_one=False, alphabet=alphabet)


def b58decode_int(v, alphabet=BITCOIN_ALPHABET):
    v = _scrub(v.rstrip() if isinstance(v, (str, bytes)) else v)
    acc = 0
    for ch in v:
        try:
            acc = acc * 58 + _MAP[ch]
        except KeyError:
            raise ValueError('Invalid character {!r}'.format(chr(ch))) from None
    return acc


def b58decode(v, alphabet=BITCOIN_ALPHABET):
    v = v.rstrip()
    v = _scrub(v)
    n0 = len(v) - len(v.lstrip(alphabet[0:1]))
    acc = b58decode_int(v[n0:], alphabet=alphabet)
    out = []
    while acc > 0:
        acc, mod = divmod(acc, 256)
        out.append(mod)
    return b'\0' * n0 + bytes(reversed(out))
