"""ctypes binding of libplenum_verify.so (include/plenum_verify.h).

This is the ONLY way the package reaches the verifier: there is no CPU
fallback.  If the shared library is missing, or no GPU is present when a
compute entry point is called, the call raises — loudly — instead of silently
verifying on the host.
"""
import ctypes
import logging
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PLENUM_GPU_LIB', os.path.join(os.path.dirname(_HERE), 'lib', 'libplenum_verify.so'))

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p

# (name, restype, argtypes) exactly as declared in include/plenum_verify.h
SIGNATURES = [
    ('pv_init', ctypes.c_int, [ctypes.c_uint32]),
    ('pv_shutdown', None, []),
    ('pv_test_init_dup', ctypes.c_int, [ctypes.c_uint32]),
    ('pv_test_set_spin_ns', ctypes.c_int, [ctypes.c_int64]),
    ('pv_last_error', ctypes.c_char_p, []),
    ('pv_device_count', ctypes.c_int, []),
    ('pv_verify_batch', ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, ctypes.c_uint32]),
    ('pv_verify_batch_device', ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_tally', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    ('pv_tally_device', ctypes.c_int,
     [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_tally_votes', ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    ('pv_tally_votes_device', ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_tally_votes_device_async', ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_sign_batch', ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    ('pv_sign_batch_device', ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_synth_device', ctypes.c_int,
     [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp,
      _vp, ctypes.c_int, _vp]),
    ('pv_synth_layout_device', ctypes.c_int,
     [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
      ctypes.c_uint32, _vp, ctypes.c_int, _vp]),
    ('pv_synth_fill_device', ctypes.c_int,
     [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp,
      _vp, _vp, _vp, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_keys_prepare_device', ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp]),
    ('pv_verify_batch_device_async', ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    ('pv_verify_keyed_device_async', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    ('pv_keys_prepare_device_async', ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    ('pv_keys_prepare_wide_device', ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp]),
    ('pv_keys_prepare_wide_device_async', ctypes.c_int,
     [_vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    ('pv_verify_keyed_wide_device', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_verify_keyed_wide_device_async', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    ('pv_verify_keys_device_async', ctypes.c_int,
     [_vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, ctypes.c_int, _vp,
      ctypes.c_int]),
    ('pv_sha256_batch', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int32, _vp]),
    ('pv_sha256_batch_device', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int32, _vp, ctypes.c_int, _vp]),
    ('pv_merkle_root', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    ('pv_merkle_root_device', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_verify_keyed_device', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp]),
    ('pv_time_verify_keyed_device', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int,
      ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    ('pv_time_verify_device', ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_int, _vp, ctypes.c_int,
      ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    ('pv_curve_stats', ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)]),
    ('pv_get_tuning', ctypes.c_int, [_vp]),
    ('pv_set_tuning', ctypes.c_int, [_vp]),
    ('pv_keycache_add', ctypes.c_int, [_vp, ctypes.c_uint64]),
    ('pv_keycache_clear', ctypes.c_int, []),
    ('pv_keycache_size', ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    ('pv_bls_set_keys', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_add_keys', ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    ('pv_bls_keyset_info', ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.POINTER(ctypes.c_uint64)]),
    ('pv_bls_verify_batch', ctypes.c_int,
     [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_verify_batch_device', ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp]),
    ('pv_bls_sign_batch_device', ctypes.c_int,
     [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int, _vp]),
    ('pv_bls_sign_batch', ctypes.c_int,
     [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_verify_multi_batch', ctypes.c_int,
     [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_aggregate_sigs', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_pubkeys', ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    ('pv_bls_kernel_ms', ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    ('pv_bls_last_error', ctypes.c_char_p, []),
    ('pv_bls_shutdown', None, []),
    ('pv_kernel_timing', ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
      ctypes.POINTER(ctypes.c_uint64)]),
    ('pv_kernel_timing_sha', ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_float)]),
]


def kernel_timing(device, enable):
    """Start (enable=True) or stop live HIP-event timing of the verify launches on
    `device` (pv_kernel_timing); stopping returns (hash_ms, curve_ms, launches) summed."""
    h, c, k = ctypes.c_float(), ctypes.c_float(), ctypes.c_uint64()
    _check('pv_kernel_timing', load().pv_kernel_timing(device, 1 if enable else 0, ctypes.byref(h), ctypes.byref(c),
                                                       ctypes.byref(k)))
    return h.value, c.value, k.value

def kernel_timing_sha(device):
    """Summed ms of the SHA-512 stage (pre-checks + k_hash) of the verify launches
    timed since kernel_timing(device, True) (pv_kernel_timing_sha)."""
    v = ctypes.c_float()
    _check('pv_kernel_timing_sha', load().pv_kernel_timing_sha(device, ctypes.byref(v)))
    return v.value


class Tuning(ctypes.Structure):
    """struct pv_tuning (include/plenum_verify.h): the schedule knobs.  pv_init
    reads no environment; tests and tools set these explicitly."""
    _fields_ = [('struct_size', ctypes.c_uint32), ('curve_mode', ctypes.c_uint32), ('lat_max', ctypes.c_uint64),
                ('lat_keyed_max', ctypes.c_uint64), ('small_zc_max', ctypes.c_uint64), ('lat_kernel', ctypes.c_uint32),
                ('host_fused', ctypes.c_uint32), ('host_staging', ctypes.c_uint32), ('host_chunks', ctypes.c_uint32),
                ('host_first_pct', ctypes.c_uint32), ('host_copy_threads', ctypes.c_uint32),
                ('host_ramp', ctypes.c_uint64), ('host_pin_max_mb', ctypes.c_uint32), ('host_trace', ctypes.c_uint32),
                ('bls_quad_max', ctypes.c_uint32), ('bls_oct_max', ctypes.c_uint32), ('reserved', ctypes.c_uint32)]


CURVE_MODES = {0: 'half', 1: 'full', 2: 'grouped'}   # PV_CURVE_HALF / _FULL / _GROUPED
LAT_KERNELS = {'quad': 0, 'pair': 1}                 # PV_LAT_QUAD / PV_LAT_PAIR
STAGING_MODES = {0: 'pinned', 1: 'pageable'}         # PV_STAGING_PINNED / _PAGEABLE
LAT_MAX_DEFAULT = 32768                              # defaults of pv_tuning (csrc/pv_api.cpp)
LAT_KEYED_MAX_DEFAULT = 8192


def get_tuning():
    """The current pv_tuning as a dict (names of include/plenum_verify.h)."""
    t = Tuning(struct_size=ctypes.sizeof(Tuning))
    _check('pv_get_tuning', load().pv_get_tuning(ctypes.byref(t)))
    return {f: getattr(t, f) for f, _ in Tuning._fields_ if f not in ('struct_size', 'reserved')}


def set_tuning(**kw):
    """Change pv_tuning fields (the others keep their values); validated as a
    whole by pv_set_tuning, applied to initialised devices and later pv_init.
    Returns the previous values of the changed fields (to restore them)."""
    cur = get_tuning()
    bad = set(kw) - set(cur)
    if bad:
        raise KeyError('unknown tuning field(s): {}'.format(sorted(bad)))
    t = Tuning(struct_size=ctypes.sizeof(Tuning), **{**cur, **kw})
    _check('pv_set_tuning', load().pv_set_tuning(ctypes.byref(t)))
    return {k: cur[k] for k in kw}


# environment names of the tuning fields, for the A/B tools only (tuning_from_env)
ENV_TUNING = {'PV_CURVE_MODE': ('curve_mode', {v: k for k, v in CURVE_MODES.items()}.get),
              'PV_LAT_MAX': ('lat_max', int), 'PV_LAT_KEYED_MAX': ('lat_keyed_max', int),
              'PV_SMALL_ZC_MAX': ('small_zc_max', int), 'PV_LAT_KERNEL': ('lat_kernel', LAT_KERNELS.get),
              'PV_HOST_FUSED': ('host_fused', int),
              'PV_HOST_STAGING': ('host_staging', {v: k for k, v in STAGING_MODES.items()}.get),
              'PV_HOST_CHUNKS': ('host_chunks', int), 'PV_HOST_FIRST_PCT': ('host_first_pct', int),
              'PV_HOST_COPY_THREADS': ('host_copy_threads', int), 'PV_HOST_RAMP': ('host_ramp', int),
              'PV_HOST_PIN_MAX_MB': ('host_pin_max_mb', int), 'PV_HOST_TRACE': ('host_trace', int),
              'PV_BLS_QUAD_MAX': ('bls_quad_max', int), 'PV_BLS_OCT_MAX': ('bls_oct_max', int)}


def tuning_from_env(environ=None):
    """Explicit opt-in for A/B tools and bench experiments: apply the PV_* tuning
    variables that are set in `environ` (default os.environ).  The library itself
    never reads the environment.  Returns the fields changed."""
    environ = os.environ if environ is None else environ
    kw = {}
    for var, (field, conv) in ENV_TUNING.items():
        if var in environ:
            v = conv(environ[var])
            if v is None:
                raise ValueError('{}={!r} is not a valid value'.format(var, environ[var]))
            kw[field] = v
    if kw:
        set_tuning(**kw)
    return kw


def set_curve_mode(name):
    """Curve-stage schedule of generic batches ('half', 'full', 'grouped')."""
    set_tuning(curve_mode={v: k for k, v in CURVE_MODES.items()}[name])


def set_lat_max(max_signatures):
    """Largest generic batch that runs the latency-mode curve kernel (8 lanes
    per signature); 0 disables."""
    set_tuning(lat_max=int(max_signatures))


def set_lat_keyed_max(max_signatures):
    """Largest keyed batch (prepared keys) that runs the keyed latency kernel; 0 disables."""
    set_tuning(lat_keyed_max=int(max_signatures))


def keycache_add(keys):
    """Add 32-byte verifying keys (an (k, 32) u8 array or an iterable of bytes)
    to the persistent device key cache (pv_keycache_add); cached keys are skipped."""
    ensure_init()
    if not isinstance(keys, np.ndarray):
        keys = [bytes(k) for k in keys]
        if any(len(k) != 32 for k in keys):
            raise ValueError('verifying keys are 32 bytes')
        keys = np.frombuffer(b''.join(keys), np.uint8) if keys else np.zeros(0, np.uint8)
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
    if keys.shape[0]:
        _check('pv_keycache_add', load().pv_keycache_add(_ptr(keys), keys.shape[0]))
        with _lock:
            _cached_keys.update(keys[i].tobytes() for i in range(keys.shape[0]))


_pending_keys = {}   # keys registered before / between GPU calls (keycache_defer), insertion-ordered, unique
_cached_keys = set()  # keys this process has handed to the device cache (tracked here: no library call)


def keycache_defer(raw):
    """Queue a 32-byte key for the device key cache; it is added by the next
    host-buffer verify call.  No GPU work and no library call here (addIdr may
    run before pv_init, or on the Looper thread while another thread holds the
    library in a verify call): the cap counts this process's own bookkeeping."""
    global _cache_dropped
    raw = bytes(raw)
    if len(raw) == 32:
        with _lock:
            if raw in _pending_keys or raw in _cached_keys:
                return
            if len(_cached_keys) + len(_pending_keys) >= KEYCACHE_MAX:
                _cache_dropped += 1          # over the cap: verified uncached
                return
            _pending_keys[raw] = None


KEYCACHE_MAX = 1 << 18   # keys queued for the device cache at most (9,344 B each on every device)
_cache_dropped = 0


def _flush_keycache():
    """Add the queued keys to the device cache.  Best effort: the cache only
    speeds verification up (uncached keys take the generic kernels), so a
    failure here (e.g. the cache cannot grow) is counted and the keys are
    dropped, never raised into the verify call that triggered the flush."""
    global _cache_dropped
    if _pending_keys:
        with _lock:
            keys = list(_pending_keys)
            _pending_keys.clear()
        try:
            keycache_add(keys)
            with _lock:
                _cached_keys.update(keys)
        except PlenumGpuError as e:
            _cache_dropped += len(keys)
            logging.getLogger(__name__).warning('device key cache: %d keys not cached (%s)', len(keys), e)


def keycache_clear():
    with _lock:
        _pending_keys.clear()
        _cached_keys.clear()
    if _inited_mask is not None:
        _check('pv_keycache_clear', load().pv_keycache_clear())


def keycache_size():
    c = ctypes.c_uint64()
    _check('pv_keycache_size', load().pv_keycache_size(ctypes.byref(c)))
    return c.value


def set_lat_kernel(name):
    """Latency kernel: 'quad' (default, lane quads per point) or 'pair' (A/B)."""
    set_tuning(lat_kernel=LAT_KERNELS[name])


def set_host_fused(enable):
    """Host-buffer chunks: one fused launch per chunk + a deferred pass (True,
    default) or the hash / lattice / curve launches per chunk."""
    set_tuning(host_fused=1 if enable else 0)


def set_host_staging(name, copy_threads=0, chunks=0):
    """Host-buffer staging of pv_verify_batch ('pinned' / 'pageable'); copy_threads
    / chunks 0 keep the current values."""
    kw = {'host_staging': {v: k for k, v in STAGING_MODES.items()}[name]}
    if copy_threads:
        kw['host_copy_threads'] = int(copy_threads)
    if chunks:
        kw['host_chunks'] = int(chunks)
    set_tuning(**kw)


def curve_stats(device=0):
    """(mode name, deferred count of the last generic batch) on `device` (pv_curve_stats)."""
    mode, nd = ctypes.c_uint32(), ctypes.c_uint64()
    _check('pv_curve_stats', load().pv_curve_stats(device, ctypes.byref(mode), ctypes.byref(nd)))
    return CURVE_MODES[mode.value], nd.value


class PlenumGpuError(RuntimeError):
    """A C-ABI call returned a negative code (message from pv_last_error)."""

    def __init__(self, fn, code, msg):
        super().__init__('{} failed ({}): {}'.format(fn, code, msg))
        self.code = code


_lib = None
_lock = threading.Lock()
_inited_mask = None   # None = nothing initialised; 0 = every visible device


def _bind_runtime_first():
    """One HIP runtime per process.  PyTorch-ROCm ships its own
    libamdhip64.so.7 (same soname as /opt/rocm's); whichever is loaded first
    serves every later NEEDED entry.  Loading torch's copy first keeps torch
    usable in processes that also call this library (bench, multi-GPU ranks,
    the device-pointer entry points); without torch, /opt/rocm's is used."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load():
    """Load the shared library (raises OSError if it was not built)."""
    global _lib
    if _lib is None:
        _bind_runtime_first()
        if not os.path.exists(LIB_PATH):
            raise OSError('libplenum_verify.so not found at {} — build it with '
                          '`python indy-plenum_amd/build.py` (there is no CPU fallback)'.format(LIB_PATH))
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _check(fn, rc):
    if rc != 0:
        raise PlenumGpuError(fn, rc, load().pv_last_error().decode(errors='replace'))


def ensure_init(device_mask=0):
    """pv_init for the devices in device_mask (0 = all visible) unless already
    initialised; raises PlenumGpuError when no GPU is usable."""
    global _inited_mask
    with _lock:
        if _inited_mask == 0 or (_inited_mask is not None and device_mask and
                                 (device_mask & _inited_mask) == device_mask):
            return
        _check('pv_init', load().pv_init(device_mask))
        _inited_mask = 0 if device_mask == 0 else (device_mask | (_inited_mask or 0))


def test_init_dup(k):
    """TEST ONLY: pv_test_init_dup -- k engine devices on HIP device 0 (the
    multi-device paths on a one-GPU box); nothing may be initialised yet."""
    global _inited_mask
    with _lock:
        _check('pv_test_init_dup', load().pv_test_init_dup(int(k)))
        _inited_mask = 0


def test_set_spin_ns(ns):
    """TEST ONLY: pv_test_set_spin_ns -- the completion-word spin budget of
    zero-copy small calls (0: every such call takes the synchronize fallback)."""
    _check('pv_test_set_spin_ns', load().pv_test_set_spin_ns(int(ns)))


def shutdown():
    global _inited_mask
    with _lock:
        _cached_keys.clear()
        # pv_bls_shutdown releases every device key set: the content index must go too
        _bls_sets.clear()
        if _lib is not None:
            _lib.pv_shutdown()
            _lib.pv_bls_shutdown()
        _inited_mask = None


def _ptr(a):
    """address of a contiguous array's data, for a c_void_p argument (None if empty).
    The buffer-protocol form costs ~0.8 us against ~2 us for `a.ctypes.data`, which
    matters at five pointers per latency call; read-only arrays take the slow path."""
    if a is None or not a.size:
        return None
    try:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError, BufferError):
        return a.ctypes.data


try:  # native host preprocessing (csrc/pv_host.cpp); the Python packer covers its Fallback cases
    from . import _host
except ImportError:
    _host = None


def pack_messages(msgs):
    """list[bytes] -> (blob uint8, off uint64[n+1]).  Native single pass
    (plenum_gpu._host.pack) for lists/tuples of bytes-like items; anything else
    takes the Python packer below."""
    if _host is not None and type(msgs) in (list, tuple):
        try:
            blob, off = _host.pack(msgs)
            return np.frombuffer(blob, np.uint8), np.frombuffer(off, np.uint64)
        except _host.Fallback:
            pass
    n = len(msgs)
    off = np.zeros(n + 1, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=n))
    blob = np.frombuffer(b''.join(msgs), dtype=np.uint8) if n else np.zeros(0, np.uint8)
    return blob, off


PV_FLAG_DEDUP_KEYS = 1
PV_KEY_WORDS = 2336
PV_KEY_WORDS_WIDE = 33056


def verify_batch_arrays(pk, sig, blob, off, device_mask=0, dedup_keys=True):
    """pk (n,32) u8, sig (n,64) u8, blob u8, off (n+1) u64 -> verdict (n,) bool.

    dedup_keys: let the library prepare each distinct key once when keys repeat
    (PV_FLAG_DEDUP_KEYS; same verdicts)."""
    ensure_init()
    pk = np.ascontiguousarray(pk, dtype=np.uint8)
    sig = np.ascontiguousarray(sig, dtype=np.uint8)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = pk.shape[0]
    if sig.shape[0] != n or off.shape[0] != n + 1 or (n and pk.shape[1] != 32) or (n and sig.shape[1] != 64):
        raise ValueError('shape mismatch: pk {}, sig {}, off {}'.format(pk.shape, sig.shape, off.shape))
    if n and int(off[-1]) > blob.size:
        raise ValueError('msg_off exceeds blob size')
    if n == 0:
        return np.zeros(0, dtype=bool)
    verdict = np.empty(n, dtype=np.uint8)   # every entry written by the library (0 / 1)
    _flush_keycache()
    flags = PV_FLAG_DEDUP_KEYS if dedup_keys else 0
    rc = None
    if _host is not None and blob.size:
        # the native call path (pv_host.cpp verify_batch): ~3 us less than five
        # ctypes pointer conversions on a ~80 us lone verify
        try:
            rc = _host.verify_batch(_verify_batch_addr(), pk, sig, blob, off, verdict, device_mask, flags)
        except _host.Fallback:
            rc = None
    if rc is None:
        rc = load().pv_verify_batch(_ptr(pk), _ptr(sig), _ptr(blob), _ptr(off), n, _ptr(verdict), device_mask, flags)
    _check('pv_verify_batch', rc)
    return verdict.view(np.bool_)


_vb_addr = None


def _verify_batch_addr():
    global _vb_addr
    if _vb_addr is None:
        _vb_addr = ctypes.cast(load().pv_verify_batch, ctypes.c_void_p).value
    return _vb_addr


def tally_arrays(verdict, sender, batch_off, n_nodes, quorum):
    ensure_init()
    verdict = np.ascontiguousarray(verdict, dtype=np.uint8)
    sender = np.ascontiguousarray(sender, dtype=np.uint32)
    batch_off = np.ascontiguousarray(batch_off, dtype=np.uint64)
    nb = batch_off.shape[0] - 1
    votes = np.zeros(max(nb, 0), dtype=np.uint32)
    reached = np.zeros(max(nb, 0), dtype=np.uint8)
    if nb <= 0:
        return votes, reached.astype(bool)
    _check('pv_tally_votes', load().pv_tally_votes(_ptr(verdict), _ptr(sender), _ptr(batch_off), nb, n_nodes,
                                                    quorum, _ptr(votes), _ptr(reached)))
    return votes, reached.astype(bool)


def tally_bits_arrays(verdict_bits, n_nodes, quorum, dup_mask=None):
    """pv_tally: verdict_bits / dup_mask (n_batches, ceil(n_nodes/32))
    uint32 node-indexed voter bitmaps -> reached (n_batches,) bool."""
    ensure_init()
    w = (int(n_nodes) + 31) // 32
    bits = np.ascontiguousarray(verdict_bits, dtype=np.uint32).reshape(-1, w)
    nb = bits.shape[0]
    dup = None
    if dup_mask is not None:
        dup = np.ascontiguousarray(dup_mask, dtype=np.uint32).reshape(-1, w)
        if dup.shape != bits.shape:
            raise ValueError('dup_mask shape {} != verdict_bits shape {}'.format(dup.shape, bits.shape))
    reached = np.zeros(nb, dtype=np.uint8)
    if nb:
        _check('pv_tally', load().pv_tally(_ptr(bits), _ptr(dup) if dup is not None else None, nb, int(n_nodes),
                                            int(quorum), _ptr(reached)))
    return reached.astype(bool)


def sign_batch_arrays(seeds, blob, off):
    ensure_init()
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = seeds.shape[0]
    pk = np.zeros((n, 32), dtype=np.uint8)
    sig = np.zeros((n, 64), dtype=np.uint8)
    if n:
        _check('pv_sign_batch', load().pv_sign_batch(_ptr(seeds), _ptr(blob), _ptr(off), n, _ptr(pk), _ptr(sig)))
    return pk, sig


# ---------------------------------------------------------------- BLS COMMIT check (row f4)
BLS_KEY_OK, BLS_KEY_INFINITY, BLS_KEY_NOT_IN_G2 = 0, 1, 2


def _bls_check(fn, rc):
    if rc != 0:
        raise PlenumGpuError(fn, rc, load().pv_bls_last_error().decode(errors='replace'))


class _BlsKeySet:
    """What the device's key set holds (its content, not who asked for it):
    the generator bytes, key bytes -> index, and each key's status."""
    __slots__ = ('gen', 'index', 'status')

    def __init__(self, gen):
        self.gen = gen
        self.index = {}
        self.status = []


_bls_sets = {}   # device -> _BlsKeySet of the set pv_bls_set_keys / pv_bls_add_keys built there


def bls_set_keys(gen, pks, device=0):
    """pv_bls_set_keys: the generator (128 B) and k keys (k x 128) -> status (k,) u8
    (0 = in G2, 1 = off the twist, 2 = outside the order-r subgroup).  The device
    holds ONE key set; it replaces whatever was there."""
    ensure_init()
    _bls_sets.pop(device, None)
    gen = np.ascontiguousarray(np.frombuffer(bytes(gen), np.uint8))
    if gen.size != 128:
        raise ValueError('the generator representation is 128 bytes')
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 128)
    st = np.zeros(pks.shape[0], np.uint8)
    _bls_check('pv_bls_set_keys', load().pv_bls_set_keys(_ptr(gen), _ptr(pks), pks.shape[0], _ptr(st), device))
    ks = _BlsKeySet(gen.tobytes())
    for i in range(pks.shape[0]):
        ks.index.setdefault(pks[i].tobytes(), i)
    ks.status = [int(x) for x in st]
    _bls_sets[device] = ks
    return st


def bls_add_keys(pks, device=0):
    """pv_bls_add_keys: append k keys (k x 128) to the device's key set without
    re-preparing it -> (first index, status (k,) u8)."""
    ensure_init()
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 128)
    st = np.zeros(pks.shape[0], np.uint8)
    first = ctypes.c_uint64()
    _bls_check('pv_bls_add_keys', load().pv_bls_add_keys(_ptr(pks), pks.shape[0], _ptr(st), ctypes.byref(first),
                                                         device))
    return first.value, st


def bls_keyset_info(device=0):
    """(keys in the device's set, points k_bls_lines prepared for it so far)"""
    n, pts = ctypes.c_uint64(), ctypes.c_uint64()
    _bls_check('pv_bls_keyset_info', load().pv_bls_keyset_info(device, ctypes.byref(n), ctypes.byref(pts)))
    return n.value, pts.value


def bls_key_indices(gen, pks, device=0):
    """Indices of 128-byte keys in the device's key set for generator `gen`,
    keyed by content: keys already there are reused, new ones appended (one
    k_bls_lines launch for all of them, pv_bls_add_keys); a set built for
    another generator is replaced.  -> (indices list, status list of the set)."""
    gen = bytes(gen)
    with _lock:
        ks = _bls_sets.get(device)
    if ks is not None and ks.gen == gen and bls_keyset_info(device)[0] < len(ks.status):
        ks = None   # the device set was released behind this index (pv_bls_shutdown): rebuild it
    if ks is None or ks.gen != gen:
        new = list(dict.fromkeys(pks))
        bls_set_keys(gen, np.frombuffer(b''.join(new), np.uint8) if new else np.zeros((0, 128), np.uint8),
                     device=device)
        ks = _bls_sets[device]
    else:
        new = [b for b in dict.fromkeys(pks) if b not in ks.index]
        if new:
            first, st = bls_add_keys(np.frombuffer(b''.join(new), np.uint8), device=device)
            for i, b in enumerate(new):
                ks.index[b] = first + i
            ks.status.extend(int(x) for x in st)
    return [ks.index[b] for b in pks], ks.status


def bls_verify_arrays(sig, blob, off, msg_idx, key_idx, sig_len=None, device=0):
    """pv_bls_verify_batch over host arrays: sig (n,128) u8, messages (blob, off),
    msg_idx / key_idx (n,) u32 -> verdict (n,) bool."""
    ensure_init()
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 128)
    n = sig.shape[0]
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    msg_idx = np.ascontiguousarray(msg_idx, dtype=np.uint32)
    key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
    if msg_idx.shape != (n,) or key_idx.shape != (n,):
        raise ValueError('msg_idx / key_idx must have one entry per signature')
    sl = None if sig_len is None else np.ascontiguousarray(sig_len, dtype=np.uint64)
    if sl is not None and sl.shape != (n,):
        raise ValueError('sig_len must have one entry per signature')
    verdict = np.zeros(n, np.uint8)
    if n:
        _bls_check('pv_bls_verify_batch', load().pv_bls_verify_batch(
            _ptr(sig), _ptr(sl) if sl is not None else None, _ptr(blob), _ptr(off), off.shape[0] - 1, _ptr(msg_idx),
            _ptr(key_idx), n, _ptr(verdict), device))
    return verdict.astype(bool)


def bls_verify_multi_arrays(gen, sig, blob, off, msg_idx, pks, pk_off, sig_len=None, device=0):
    """pv_bls_verify_multi_batch: check j = (sig j (n,128) u8, message msg_idx[j] of
    (blob, off), the sum of keys pks[pk_off[j]:pk_off[j+1]] ((k,128) u8)) against
    the generator `gen` -> verdict (n,) bool.  The key set of bls_set_keys is kept."""
    ensure_init()
    gen = np.ascontiguousarray(np.frombuffer(bytes(gen), np.uint8))
    if gen.size != 128:
        raise ValueError('the generator representation is 128 bytes')
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 128)
    n = sig.shape[0]
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    msg_idx = np.ascontiguousarray(msg_idx, dtype=np.uint32)
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 128)
    pk_off = np.ascontiguousarray(pk_off, dtype=np.uint64)
    if msg_idx.shape != (n,) or pk_off.shape != (n + 1,):
        raise ValueError('msg_idx needs n entries and pk_off n + 1')
    if n and int(pk_off[-1]) > pks.shape[0]:
        raise ValueError('pk_off exceeds the key array')
    sl = None if sig_len is None else np.ascontiguousarray(sig_len, dtype=np.uint64)
    if sl is not None and sl.shape != (n,):
        raise ValueError('sig_len must have one entry per signature')
    verdict = np.zeros(n, np.uint8)
    if n:
        _bls_check('pv_bls_verify_multi_batch', load().pv_bls_verify_multi_batch(
            _ptr(gen), _ptr(sig), _ptr(sl) if sl is not None else None, _ptr(blob), _ptr(off), off.shape[0] - 1,
            _ptr(msg_idx), _ptr(pks), _ptr(pk_off), n, _ptr(verdict), device))
    return verdict.astype(bool)


def bls_aggregate_sigs(sigs, set_off, device=0):
    """pv_bls_aggregate_sigs: the G1 sum of sigs[set_off[j]:set_off[j+1]] ((k,128) u8)
    for every set j -> (m, 128) u8 representations (MultiSignature.new)."""
    ensure_init()
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(-1, 128)
    set_off = np.ascontiguousarray(set_off, dtype=np.uint64)
    m = set_off.shape[0] - 1
    if m > 0 and int(set_off[-1]) > sigs.shape[0]:
        raise ValueError('set_off exceeds the signature array')
    out = np.zeros((max(m, 0), 128), np.uint8)
    if m > 0:
        _bls_check('pv_bls_aggregate_sigs', load().pv_bls_aggregate_sigs(_ptr(sigs), _ptr(set_off), m, _ptr(out),
                                                                          device))
    return out


def bls_sign_arrays(sks, blob, off, msg_idx, key_idx, device=0):
    """pv_bls_sign_batch: sig j = sk[key_idx[j]] * H(message msg_idx[j]) -> (n, 128) u8 (data generation)."""
    ensure_init()
    sks = np.ascontiguousarray(sks, dtype=np.uint8).reshape(-1, 32)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    msg_idx = np.ascontiguousarray(msg_idx, dtype=np.uint32)
    key_idx = np.ascontiguousarray(key_idx, dtype=np.uint32)
    n = msg_idx.shape[0]
    out = np.zeros((n, 128), np.uint8)
    if n:
        _bls_check('pv_bls_sign_batch', load().pv_bls_sign_batch(
            _ptr(sks), sks.shape[0], _ptr(blob), _ptr(off), off.shape[0] - 1, _ptr(msg_idx), _ptr(key_idx), n,
            _ptr(out), device))
    return out


def bls_pubkeys(gen, sks, device=0):
    """pv_bls_pubkeys: pk = sk * g for k 32-byte big-endian secret scalars (data generation)."""
    ensure_init()
    gen = np.ascontiguousarray(np.frombuffer(bytes(gen), np.uint8))
    sks = np.ascontiguousarray(sks, dtype=np.uint8).reshape(-1, 32)
    out = np.zeros((sks.shape[0], 128), np.uint8)
    _bls_check('pv_bls_pubkeys', load().pv_bls_pubkeys(_ptr(gen), _ptr(sks), sks.shape[0], _ptr(out), device))
    return out


def bls_kernel_ms(device=0):
    """(hash_ms, verify_ms) of the last BLS verify call on `device` (HIP events)."""
    h, v = ctypes.c_float(), ctypes.c_float()
    _bls_check('pv_bls_kernel_ms', load().pv_bls_kernel_ms(device, ctypes.byref(h), ctypes.byref(v)))
    return h.value, v.value
