"""base58 (Bitcoin alphabet) with the base58 2.x behaviour Plenum relies on.

The reference leaves base58 unpinned (setup.py:98-99) and ships no source, so
this restates its published contract: leading zero bytes <-> leading '1',
b58decode strips trailing whitespace, an invalid character raises ValueError,
both functions accept str or bytes and return bytes.
"""
ALPHABET = b'123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz'
_INDEX = {c: i for i, c in enumerate(ALPHABET)}


def _as_bytes(v):
    if isinstance(v, str):
        v = v.encode('ascii')
    return bytes(v)


def _py_b58encode(v):
    raw = _as_bytes(v)
    stripped = raw.lstrip(b'\0')
    zeros = len(raw) - len(stripped)
    num = int.from_bytes(stripped, 'big')
    digits = bytearray()
    while num:
        num, rem = divmod(num, 58)
        digits.append(ALPHABET[rem])
    return b'1' * zeros + bytes(reversed(digits))


def _py_b58decode(v):
    text = _as_bytes(v.rstrip())
    body = text.lstrip(b'1')
    zeros = len(text) - len(body)
    num = 0
    for ch in body:
        d = _INDEX.get(ch)
        if d is None:
            raise ValueError('Invalid character {!r}'.format(chr(ch)))
        num = num * 58 + d
    out = num.to_bytes((num.bit_length() + 7) // 8, 'big') if num else b''
    return b'\0' * zeros + out


# Native implementations (csrc/pv_host.cpp); inputs the
# restatement treats specially or rejects take the Python path above, so
# results and exceptions are identical.
try:
    from . import _host
    NATIVE = True
except ImportError:  # not built yet: the restatement alone (host preprocessing, not the verify path)
    _host = None
    NATIVE = False


def b58encode(v):
    if _host is not None:
        try:
            return _host.b58encode(v)
        except _host.Fallback:
            pass
    return _py_b58encode(v)


def b58decode(v):
    if _host is not None:
        try:
            return _host.b58decode(v)
        except _host.Fallback:
            pass
    return _py_b58decode(v)
