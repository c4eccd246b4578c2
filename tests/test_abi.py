"""The C-ABI library builds, loads on a CPU-only host, exports exactly what
include/plenum_verify.h declares, and fails loudly without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, 'include', 'plenum_verify.h')


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char \*)\s*\**\s*(pv_\w+)\s*\(', text, re.M)))


@pytest.fixture(scope='module')
def native():
    import sys
    sys.path.insert(0, PKG)
    import build as pkg_build
    pkg_build.build()
    from plenum_gpu import _native
    return _native


def test_exports_every_declared_symbol(native):
    names = declared()
    assert len(names) >= 12
    out = subprocess.run(['nm', '-D', '--defined-only', native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r' T (pv_\w+)', out))
    assert set(names) <= exported, set(names) - exported
    lib = native.load()
    for n in names:
        assert getattr(lib, n) is not None


def test_python_binding_matches_header(native):
    assert sorted(n for n, _, _ in native.SIGNATURES) == declared()


def test_library_is_gfx950(native):
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '--notes', native.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(native.LIB_PATH, 'rb').read()
    assert b'gfx950' in blob


def _gpu_present(native):
    rc = native.load().pv_init(0)
    if rc == 0:
        native.load().pv_shutdown()
        return True
    return False


def test_fails_loudly_without_gpu(native):
    if _gpu_present(native):
        pytest.skip('a GPU is present; the no-GPU contract is exercised on CPU hosts')
    lib = native.load()
    assert lib.pv_init(0) == -19  # PV_ENODEV
    assert lib.pv_last_error()
    n = 1
    buf = np.zeros(64, np.uint8)
    off = np.zeros(2, np.uint64)
    v = np.zeros(1, np.uint8)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    assert lib.pv_verify_batch(p(buf), p(buf), p(buf), p(off), n, p(v), 0, 0) == -77  # PV_ENOTINIT
    with pytest.raises(native.PlenumGpuError):
        native.verify_batch_arrays(np.zeros((1, 32), np.uint8), np.zeros((1, 64), np.uint8),
                                   np.zeros(0, np.uint8), np.zeros(2, np.uint64))
    # the key cache: nothing to prepare it on
    assert lib.pv_keycache_add(p(buf), 1) == -77   # PV_ENOTINIT
    c = ctypes.c_uint64(5)
    assert lib.pv_keycache_size(ctypes.byref(c)) == 0 and c.value == 0
    assert lib.pv_keycache_clear() == 0
    # keys registered without a GPU are only queued (SimpleAuthNr.addIdr must not raise)
    from plenum_gpu.client_authn import SimpleAuthNr
    from plenum_gpu import base58
    SimpleAuthNr().addIdr('did', base58.b58encode(bytes(range(32))).decode())
    assert native._pending_keys
    native.keycache_clear()
    assert not native._pending_keys


def test_no_cpu_fallback_in_product_package():
    """The product package never imports the oracle or the host build."""
    pkg = os.path.join(PKG, 'plenum_gpu')
    for fn in os.listdir(pkg):
        if fn.endswith('.py'):
            src = open(os.path.join(pkg, fn)).read()
            assert 'oracle' not in src.lower().replace('libsodium', ''), fn
            assert 'hostcheck' not in src, fn
            assert 'libsodium.so' not in src, fn


def test_library_reads_no_environment(native):
    """pv_init reads no environment: the library imports no
    getenv, and the schedule knobs are one explicit pv_tuning struct whose
    defaults, validation and round trip are checked here (no GPU needed)."""
    out = subprocess.run(['nm', '-D', '--undefined-only', native.LIB_PATH], capture_output=True, text=True).stdout
    assert not re.search(r'\bgetenv\b|secure_getenv', out)
    d = native.get_tuning()
    assert d == {'curve_mode': 0, 'lat_max': 32768, 'lat_keyed_max': 8192, 'small_zc_max': 2048, 'lat_kernel': 0,
                 'host_fused': 1, 'host_staging': 0, 'host_chunks': 8, 'host_first_pct': 50, 'host_copy_threads': 8,
                 'host_ramp': 32768, 'host_pin_max_mb': 512, 'host_trace': 0,
                 'bls_quad_max': 32768, 'bls_oct_max': 4096}
    os.environ['PV_CURVE_MODE'] = 'full'        # ignored by the library itself
    try:
        assert native.get_tuning()['curve_mode'] == 0
        for bad in ({'curve_mode': 3}, {'host_chunks': 0}, {'host_ramp': 5},
                    {'host_pin_max_mb': 8}, {'lat_max': (1 << 20) + 1},
                    {'bls_quad_max': (1 << 20) + 1}, {'bls_oct_max': (1 << 20) + 1}):
            with pytest.raises(native.PlenumGpuError):
                native.set_tuning(**bad)
            assert native.get_tuning() == d
        prev = native.set_tuning(curve_mode=2, lat_max=0, host_trace=1)
        assert native.get_tuning() == dict(d, curve_mode=2, lat_max=0, host_trace=1)
        native.set_tuning(**prev)
        assert native.get_tuning() == d
        assert native.tuning_from_env({'PV_CURVE_MODE': 'grouped', 'PV_HOST_CHUNKS': '4'}) == \
            {'curve_mode': 2, 'host_chunks': 4}
        native.set_tuning(curve_mode=0, host_chunks=8)
        with pytest.raises(ValueError):
            native.tuning_from_env({'PV_CURVE_MODE': 'fast'})
        t = native.Tuning(struct_size=ctypes.sizeof(native.Tuning) - 4)
        assert native.load().pv_get_tuning(ctypes.byref(t)) == -22
    finally:
        del os.environ['PV_CURVE_MODE']


def test_tuning_struct_has_no_test_fields(native):
    """The node-facing pv_tuning carries schedule knobs only:
    the duplicate-device test mode is its own test-only entry point,
    pv_test_init_dup, which refuses bad counts before touching a device."""
    names = [f for f, _ in native.Tuning._fields_]
    assert not [f for f in names if f.startswith('test') or 'dup' in f], names
    hdr = open(os.path.join(REPO, 'include', 'plenum_verify.h')).read()
    body = hdr[hdr.index('typedef struct pv_tuning'):hdr.index('} pv_tuning;')]
    assert 'test' not in body and 'dup' not in body
    assert 'int pv_test_init_dup(uint32_t k);' in hdr
    for bad in (0, 1, 9):
        assert native.load().pv_test_init_dup(bad) == -22

