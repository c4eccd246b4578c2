"""Native host preprocessing (csrc/pv_host.cpp -> plenum_gpu._host, SURVEY.md
§8 f2) is byte-identical to the base58 / signing-serializer restatements,
including every rejected input (same exception type and text)."""
import random

import pytest

from plenum_gpu import base58, serialization


def _outcome(fn, *a):
    try:
        return ('ok', fn(*a))
    except Exception as ex:  # noqa: BLE001 - comparing exact exceptions
        return ('err', type(ex), str(ex))


def test_native_module_loaded():
    import sys
    sys.path.insert(0, serialization.__file__.rsplit('/', 2)[0])
    import build
    build.build_host()
    import importlib
    importlib.reload(base58)
    importlib.reload(serialization)
    assert base58.NATIVE and serialization._host is not None


def test_base58_roundtrip_random():
    rng = random.Random(7)
    alpha = base58.ALPHABET.decode()
    for n in range(0, 130):
        for _ in range(20):
            raw = bytes(rng.choice([0, 0, 1, 255, rng.randrange(256)]) for _ in range(n))
            e = base58.b58encode(raw)
            assert e == base58._py_b58encode(raw)
            assert base58.b58decode(e) == raw == base58.b58decode(e.decode())
            s = ''.join(rng.choice(alpha) for _ in range(n))
            assert base58.b58decode(s) == base58._py_b58decode(s)


@pytest.mark.parametrize('v', ['0abc', 'abcI', 'abcl', 'é', 'ab c', b'abc\x1f', 'abc\x1c', 'zz\n\t ', b'11', '',
                               3, memoryview(b'abc'), bytearray(b'3yZe7d'), None, ['a']])
def test_base58_decode_edges_identical(v):
    assert _outcome(base58.b58decode, v) == _outcome(base58._py_b58decode, v)


@pytest.mark.parametrize('v', [b'', b'\0\0', 'abc', 'é', 3, memoryview(b'\0ab'), bytearray(b'\0\1'), [1, 2], None])
def test_base58_encode_edges_identical(v):
    assert _outcome(base58.b58encode, v) == _outcome(base58._py_b58encode, v)


class _IntSub(int):
    def __str__(self):
        return 'sub'


class _DictSub(dict):
    pass


CASES = [
    {'a': 1, 'b': [1, 2, {'x': None, 'y': 1.5}], 'c': 'é€😀', 'd': True, 'e': False},
    {'z': {}, 'y': [], 'x': ''}, 'abc', 5, -7, 1e300, float('nan'), None, [1, 'a', None, [2, [3]]],
    {'signature': 'x', 'k': 1, 'signatures': {'a': 'b'}}, {1: 'a', 2: 'b', -1: 'c'}, {'a': (1, 2)},
    {'a': object()}, {1: 'a', 'b': 2}, {'a': {'b': {'c': [[], [None], 'q']}}}, {'a': _IntSub(3)},
    _DictSub(b=1, a=2), {'a': _DictSub(x=1)}, {'a': '\ud800'}, {'a': b'bytes'}, {'a': {1, 2}},
    {'operation': {'type': 'buy', 'data': 'x' * 300}, 'reqId': 12, 'identifier': 'Id', 'protocolVersion': 2},
]


@pytest.mark.parametrize('case', range(len(CASES)))
@pytest.mark.parametrize('ignore', [None, [], ['signature'], {'k', 'signatures'}, ('a',)])
def test_serializer_identical(case, ignore):
    obj = CASES[case]
    want = _outcome(serialization.signing_serializer.serialize, obj, 0, None, ignore)
    got = _outcome(serialization.serialize_msg_for_signing, obj, ignore)
    if want[0] == 'ok' and isinstance(obj, float) and obj != obj:
        assert got == want
    assert got == want


def test_pack_matches_python_packer():
    """plenum_gpu._host.pack (csrc/pv_host.cpp) == the Python packer for lists and
    tuples of bytes-like items (bytes, bytearray, memoryview, contiguous numpy);
    anything else raises Fallback so pack_messages keeps the Python behaviour."""
    import numpy as np
    from plenum_gpu import _host, _native as nat

    def py_pack(msgs):
        n = len(msgs)
        off = np.zeros(n + 1, np.uint64)
        if n:
            off[1:] = np.cumsum([len(m) for m in msgs])
        return np.frombuffer(b''.join(msgs), np.uint8), off

    rng = np.random.default_rng(5)
    cases = [[], [b''], [b'abc'], (b'q', b'', b'zz'),
             [b'a', bytearray(b'xyz'), memoryview(b'12345'), np.arange(7, dtype=np.uint8)],
             [rng.bytes(int(k)) for k in rng.integers(0, 600, 500)]]
    for c in cases:
        b1, o1 = nat.pack_messages(c)
        b2, o2 = py_pack([bytes(m) for m in c])
        assert o1.dtype == np.uint64 and (o1 == o2).all() and (b1 == b2).all()
    for bad in ([1, 2], [b'a', 'str'], [np.arange(6, dtype=np.uint8)[::2]], iter([b'a'])):
        with pytest.raises(_host.Fallback):
            _host.pack(bad)


def test_verify_batch_call_path_passes_buffers_and_falls_back():
    """_host.verify_batch (the wrapper's native call path into pv_verify_batch):
    the five buffers reach the C function unchanged, n = the verdict length, the
    mask / flags pass through, and a missing address or an unwritable verdict
    buffer raises Fallback (the ctypes path then runs).  A stand-in C function
    with pv_verify_batch's signature checks the arguments (no GPU)."""
    import ctypes
    import numpy as np
    from plenum_gpu import _host
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32)
    seen = {}

    def fake(pk, sig, blob, off, n, verdict, mask, flags):
        seen.update(pk=pk, sig=sig, blob=blob, off=off, n=n, verdict=verdict, mask=mask, flags=flags)
        ctypes.memset(verdict, 1, n)
        return 7

    cb = proto(fake)
    addr = ctypes.cast(cb, ctypes.c_void_p).value
    pk, sig = np.zeros((3, 32), np.uint8), np.zeros((3, 64), np.uint8)
    blob, off = np.zeros(100, np.uint8), np.array([0, 10, 20, 30], np.uint64)
    v = np.zeros(3, np.uint8)
    rc = _host.verify_batch(addr, pk, sig, blob, off, v, 5, 2)
    assert rc == 7 and (v == 1).all()
    assert seen['pk'] == pk.ctypes.data and seen['sig'] == sig.ctypes.data and seen['blob'] == blob.ctypes.data
    assert seen['off'] == off.ctypes.data and seen['verdict'] == v.ctypes.data
    assert (seen['n'], seen['mask'], seen['flags']) == (3, 5, 2)
    with pytest.raises(_host.Fallback):
        _host.verify_batch(0, pk, sig, blob, off, v, 0, 0)
    ro = np.zeros(3, np.uint8)
    ro.flags.writeable = False
    with pytest.raises(_host.Fallback):
        _host.verify_batch(addr, pk, sig, blob, off, ro, 0, 0)
    # undersized inputs: ValueError before the C function is reached
    seen.clear()
    for args in ((pk[:2], sig, blob, off), (pk, sig[:2], blob, off), (pk, sig, blob, off[:3]),
                 (pk, sig, blob[:29], off)):
        with pytest.raises(ValueError):
            _host.verify_batch(addr, *args, v, 0, 0)
    assert not seen
