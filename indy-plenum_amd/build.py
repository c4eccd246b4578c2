"""Build libplenum_verify.so (HIP, gfx950) in-tree.

    python indy-plenum_amd/build.py            # build if sources changed
    python indy-plenum_amd/build.py --force

Output: indy-plenum_amd/lib/libplenum_verify.so (git-ignored, travels to the
GPU box with the gpurun snapshot).  Compiles on a CPU-only host: hipcc
cross-compiles gfx950 code objects.
"""
import argparse
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, 'lib')
LIB = os.path.join(LIBDIR, 'libplenum_verify.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
SOURCES = ['pv_kernels.hip', 'pv_bls.hip', 'pv_api.cpp']
COMMON = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH, '-Wall', '-Wno-unused-function',
          '-Wno-unused-variable', '-I' + os.path.join(REPO, 'include')]


def _digest():
    h = hashlib.sha256()
    for fn in sorted(os.listdir(CSRC)):
        with open(os.path.join(CSRC, fn), 'rb') as fh:
            h.update(fn.encode() + fh.read())
    with open(os.path.join(REPO, 'include', 'plenum_verify.h'), 'rb') as fh:
        h.update(fh.read())
    h.update(' '.join(COMMON).encode())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('build failed:\n' + ' '.join(cmd) + '\n' + r.stdout + r.stderr)
    return r.stdout + r.stderr


def build_host(force=False):
    """plenum_gpu/_host (CPython extension, g++): native base58 + signing serializer."""
    import sysconfig
    src = os.path.join(CSRC, 'pv_host.cpp')
    out = os.path.join(HERE, 'plenum_gpu', '_host' + sysconfig.get_config_var('EXT_SUFFIX'))
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    tmp = out + '.tmp'
    _run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-Wall', '-I' + sysconfig.get_paths()['include'], src,
          '-o', tmp])
    os.replace(tmp, out)
    return out


def build(force=False, verbose=False, defines=(), lib=None):
    """Compile the library; `defines`/`lib` build named variants for A/B timing."""
    os.makedirs(LIBDIR, exist_ok=True)
    lib = lib or LIB
    extra = ['-D' + d for d in defines]
    stamp = lib + '.stamp'
    dig = _digest() + ' '.join(extra)
    if not force and os.path.exists(lib) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == dig:
                return lib
    objs = []
    cmds = []
    for src in SOURCES:
        obj = os.path.join(LIBDIR, os.path.basename(lib) + '.' + src + '.o')
        lang = ['-x', 'hip'] if src.endswith('.hip') else []
        cmds.append([HIPCC] + COMMON + extra + lang + ['-c', os.path.join(CSRC, src), '-o', obj])
        objs.append(obj)
    with ThreadPoolExecutor(len(cmds)) as ex:
        for out in ex.map(_run, cmds):
            if verbose and out.strip():
                print(out)
    tmp = lib + '.tmp'
    _run([HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', tmp] + objs)
    os.replace(tmp, lib)
    with open(stamp, 'w') as fh:
        fh.write(dig)
    return lib


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-v', '--verbose', action='store_true')
    ap.add_argument('-D', dest='defines', action='append', default=[], help='extra -D for a variant build')
    ap.add_argument('-o', dest='lib', default=None, help='output .so for a variant build')
    a = ap.parse_args()
    if not a.lib:
        print(build_host(force=a.force))
    print(build(force=a.force, verbose=a.verbose, defines=a.defines, lib=a.lib))
    sys.exit(0)
