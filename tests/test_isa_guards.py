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

import _isa_hazards
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
    """No SMEM whose base SGPR pair a v_mad_*64_*32 carry-out overwrites within
    the next 3 instructions (the faulting round-3 build did so 2 instructions
    after issue, from inline asm).  The v_mad carry-out is the only SGPR write
    our inline asm emits (csrc/pv_madchains.h, pv_bn254_asm.h); the compiler's
    own scheduling does place other SGPR writes there (a v_cmp_*_e64 mask or a
    v_readfirstlane over the kernarg pointer, 0-2 instructions after an s_load
    from it -- k_hash, k_verify_quad_keyed, the BLS quad / octet kernels), which
    _isa_hazards.py records as smem_base_war without a bound: SMEM reads its
    SGPR operands at issue."""
    funcs = sum(1 for ln in disasm if re.match(r'^[0-9a-f]+ <', ln))
    assert funcs > 20
    bad = []
    for i, ln in enumerate(disasm):
        m = re.search(r'\ss_load_dword\w*\s+[^,]+,\s+(s\[\d+:\d+\])', ln)
        if not m:
            continue
        base = _pair(m.group(1))
        for j in range(i + 1, min(i + 4, len(disasm))):
            w = re.match(r'\s+v_mad_[iu]64_[iu]32\w*\s+[^,]+,\s+(s\[\d+:\d+\])', disasm[j])
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


def test_documented_wait_states_hold_in_every_kernel(disasm):
    """every producer/consumer pair of the ISA's software
    wait-state rules (tests/_isa_hazards.py: VALU SGPR write -> VMEM / lane
    select, VALU VGPR write -> DPP / v_readlane / v_permlane, VALU EXEC write ->
    DPP, wide VMEM store -> overwrite of its data) has its wait states, in
    compiler code and inside the generated asm chains alike: the scan covers all
    pairs of the code object, a superset of those with an end inside an asm
    string.  LDS reads of a just-written VGPR (ds_swizzle exchanges, LDS
    addresses) are hardware-interlocked and only counted."""
    bad, counts, lds = _isa_hazards.scan(disasm)
    documented = [b for b in bad if b[0] in _isa_hazards.REQUIRED]
    assert not documented, documented[:5]
    assert counts['valu_vgpr_dpp'] > 100 and counts['store_data_war'] > 100 and counts['valu_vgpr_readlane'] > 10
    assert lds > 100
    # the recorded SMEM pattern occurs only where the compiler put it (a readfirstlane or a
    # v_cmp mask over the kernarg pointer), never from an asm chain's v_mad carry-out (the
    # round-3 fault's form; the only SGPR write inline asm emits here)
    war = [b for b in bad if b[0] == 'smem_base_war']
    assert war and not [b for b in war if 'v_mad_' in b[3]], war


SNIPPETS = {
    'valu_sgpr_vmem': ['v_add_co_u32_e64 v1, s[4:5], v2, v3', 'global_load_dword v6, v[2:3], s[4:5]'],
    'valu_sgpr_lanesel': ['v_cmp_eq_u32_e64 s[8:9], v1, v2', 'v_readlane_b32 s10, v3, s8'],
    'valu_vgpr_dpp': ['v_add_u32_e32 v5, v1, v2', 'v_mov_b32_dpp v6, v5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf'],
    'valu_exec_dpp': ['v_cmpx_eq_u32_e32 v1, v2', 'v_mov_b32_dpp v6, v7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf'],
    'valu_vgpr_readlane': ['v_mad_u64_u32 v[4:5], vcc, v1, v2, v[4:5]', 'v_readfirstlane_b32 s3, v4'],
    'valu_vgpr_permlane': ['v_add_u32_e32 v8, v1, v2', 'v_permlane32_swap_b32 v8, v9'],
    'store_data_war': ['global_store_dwordx4 v[0:1], v[4:7], off', 'v_mov_b32_e32 v6, 0'],
}


@pytest.mark.parametrize('rule', sorted(SNIPPETS))
def test_scanner_flags_each_rule_and_accepts_the_padded_form(rule):
    """each rule on a two-instruction stream: flagged back to back, accepted
    with exactly the required s_nop in between (s_nop N = N + 1 states)"""
    need = _isa_hazards.REQUIRED[rule]
    p, c = SNIPPETS[rule]
    head = ['0000000000001000 <k>:']
    bad, counts, _ = _isa_hazards.scan(head + ['\t' + p, '\t' + c])
    assert [b[0] for b in bad] == [rule] and counts[rule] == 1
    short = ['\ts_nop {}'.format(need - 2)] if need >= 2 else []
    bad, _, _ = _isa_hazards.scan(head + ['\t' + p] + short + ['\t' + c])
    assert [b[0] for b in bad] == [rule]
    bad, _, _ = _isa_hazards.scan(head + ['\t' + p, '\ts_nop {}'.format(need - 1), '\t' + c])
    assert not bad

