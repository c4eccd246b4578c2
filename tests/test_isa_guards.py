"""ISA guards on the built gfx950 code object (CPU only: llvm-objdump of the
library's offload bundle).

Round 3's scalar-cache variant of the BLS Miller loop (line coefficients read
with SMEM through readfirstlane'd pointers) faulted with an illegal memory
access on its first GPU run.  Its object files are still in
indy-plenum_amd/lib (sload.so.*.o); their disassembly shows correct addresses
and offsets, and ONE pattern no shipped build has: the base SGPR pair of an
SMEM load is overwritten 1-3 instructions after issue by the carry-out of a
v_mad_u64_u32 inside the generated inline-asm MAD chains (csrc/pv_bn254_asm.h),
which hipcc schedules as opaque statements and pads no hazards for
(cdna_hip_programming.md §5.7).  DESIGN.md §8 item 7 has the analysis.  The
shipped kernels read line coefficients with vector loads only; this test keeps
that pattern out of every kernel of the library."""
import os
import re
import subprocess

import pytest

from conftest import PKG

LLVM = '/opt/rocm/lib/llvm/bin'
LIB = os.path.join(PKG, 'lib', 'libplenum_verify.so')


@pytest.fixture(scope='module')
def disasm(tmp_path_factory):
    """Disassembly of every gfx950 code object in the library (the .hip_fatbin
    section holds one offload bundle per .hip source, concatenated)."""
    import sys
    sys.path.insert(0, PKG)
    import build as pkg_build
    pkg_build.build()
    d = tmp_path_factory.mktemp('isa')
    fat = str(d / 'fat.bin')
    subprocess.run([os.path.join(LLVM, 'llvm-objcopy'), '--dump-section=.hip_fatbin=' + fat, LIB, str(d / 'lib.so')],
                   check=True)
    blob = open(fat, 'rb').read()
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
    lines = []
    for k, a in enumerate(starts):
        part, co = str(d / 'b{}.bin'.format(k)), str(d / 'b{}.co'.format(k))
        with open(part, 'wb') as fh:
            fh.write(blob[a:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        subprocess.run([os.path.join(LLVM, 'clang-offload-bundler'), '--unbundle', '--type=o', '--input=' + part,
                        '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', '--output=' + co], check=True)
        lines += subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--no-show-raw-insn', co],
                                capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(starts) >= 2    # pv_kernels.hip and pv_bls.hip
    return lines


def _pair(tok):
    m = re.match(r's\[(\d+):(\d+)\]', tok)
    return (int(m.group(1)), int(m.group(2))) if m else None


def test_no_smem_base_rewritten_by_valu_right_after_issue(disasm):
    """No SMEM whose base SGPR pair a VALU overwrites within the next 3
    instructions (the faulting build did so 2 instructions after issue, from
    inline asm; compiler-scheduled code keeps >= 4 instructions between, e.g.
    pv::k_scan_sums)."""
    funcs = sum(1 for ln in disasm if re.match(r'^[0-9a-f]+ <', ln))
    assert funcs > 20
    bad = []
    for i, ln in enumerate(disasm):
        m = re.search(r'\ss_load_dword\w*\s+[^,]+,\s+(s\[\d+:\d+\])', ln)
        if not m:
            continue
        base = _pair(m.group(1))
        for j in range(i + 1, min(i + 4, len(disasm))):
            # VALU writes of an SGPR pair: the carry-out of VOP3b ops, a VOPC e64 mask
            w = (re.match(r'\s+v_(?:mad_[iu]64_[iu]32|add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co|div_scale)'
                          r'\w*\s+[^,]+,\s+(s\[\d+:\d+\])', disasm[j])
                 or re.match(r'\s+v_cmpx?_\w+_e64\s+(s\[\d+:\d+\])', disasm[j]))
            if w and _pair(w.group(1)) == base:
                bad.append((i + 1, ln.strip()[:60], disasm[j].strip()[:60]))
    assert not bad, bad[:5]


def test_bls_check_kernel_reads_lines_with_vector_loads(disasm):
    """k_bls_verify and the bn:: functions it calls read the wave-uniform line
    rows through EXEC-masked vector loads (staged in LDS), never SMEM: the only
    SMEM left there are the kernel-argument loads of the prologue."""
    fn = [i for i, ln in enumerate(disasm) if re.match(r'^[0-9a-f]+ <', ln)]
    bodies = {}
    for k, i in enumerate(fn):
        name = disasm[i].split('<')[1].rstrip('>:')
        bodies[name] = disasm[i:fn[k + 1] if k + 1 < len(fn) else len(disasm)]
    verify = [n for n in bodies if 'k_bls_verify' in n]
    assert len(verify) == 3    # the lane-pair, lane-quad and lane-octet check kernels
    for v in verify:
        smem = [ln for ln in bodies[v] if re.search(r'\ss_load_', ln)]
        assert smem and len(smem) <= 16, smem
        assert all(re.search(r's_load_\w+\s+[^,]+,\s+s\[(0:1|[2-9]:\d+|1\d:\d+)\],\s+0x[0-9a-f]+', ln) for ln in smem)
        assert [ln for ln in bodies[v] if re.search(r'\s(global|flat)_load_', ln)]
    for n, body in bodies.items():
        if n.startswith('_ZN2bn'):
            assert not [ln for ln in body if re.search(r'\ss_load_', ln)], n
