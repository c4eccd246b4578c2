"""Software wait-state check over a gfx950 disassembly (tests/test_isa_guards.py).

hipcc pads the hazards of the code it schedules, but treats an inline-asm
statement as opaque: nothing inside the string is padded and only a fixed one-
state pad follows `;;#ASMEND` (cdna_hip_programming.md §5.7 item 2).  The
generated MAD chains (csrc/pv_madchains.h, csrc/pv_bn254_asm.h) write the VCC
carry-out of every v_mad_*64_*32 and feed DPP / ds_swizzle exchanges and memory
addresses in the quad, pair and octet kernels.  This scanner checks EVERY
producer/consumer pair of the rules below in the whole code object -- compiler
code and asm alike (a superset of the pairs with an end inside an asm string) --
so it needs no asm markers and runs on llvm-objdump output.

Rules (CDNA3/CDNA4 ISA "manually inserted wait states"; states = instructions
between producer and consumer, s_nop N counting N + 1):
  valu_sgpr_vmem     VALU writes an SGPR (VOP3b carry-out, v_cmp_e64 / v_cmp_e32
                     VCC, v_readlane / v_readfirstlane) -> VMEM reads it
                     (saddr / srsrc / soffset)                               5
  valu_sgpr_lanesel  same producer -> v_readlane / v_writelane lane select   4
  valu_vgpr_dpp      VALU writes a VGPR -> a DPP op reads it as src0         2
  valu_exec_dpp      VALU writes EXEC (v_cmpx) -> any DPP op                 5
  valu_vgpr_readlane VALU writes a VGPR -> v_readlane / v_readfirstlane
                     reads it                                                1
  valu_vgpr_permlane VALU writes a VGPR -> v_permlane*_swap reads it         2
  store_data_war     VMEM store of > 64 data bits -> a VALU overwrites one
                     of its data VGPRs                                       1
Recorded, not bounded (no documented wait state):
  smem_base_war      an in-flight SMEM's base / offset SGPRs overwritten by a
                     VALU within 3 instructions of the SMEM -- the round-3
                     faulting build's pattern (a v_mad carry-out 2 after issue).
                     The shipped library has it too, in compiler-scheduled code
                     that runs in every GPU test (v_readfirstlane_b32 s0
                     overwriting the kernarg pointer s[0:1] 0-2 instructions
                     after an s_load from it, k_hash and the BLS quad / octet
                     kernels): SMEM reads its SGPR operands at issue, so this is
                     not the hazard that faulted.
LDS instructions (ds_read / ds_write / ds_swizzle / ds_bpermute) reading a
VGPR a VALU just wrote are interlocked by the hardware (no software wait
state): the scanner records those pairs (`lds_after_valu`) without a bound.
"""
import re

REQUIRED = {'valu_sgpr_vmem': 5, 'valu_sgpr_lanesel': 4, 'valu_vgpr_dpp': 2, 'valu_exec_dpp': 5,
            'valu_vgpr_readlane': 1, 'valu_vgpr_permlane': 2, 'store_data_war': 1}
RECORDED = {'smem_base_war': 3}   # window of the recorded (unbounded) pattern
LOOKAHEAD = 6   # largest requirement + 1: a consumer further away is always padded

_INSN = re.compile(r'^\s+([a-z_][a-z0-9_]*)\s*(.*?)\s*(?://.*)?$')
_VCOP3B = re.compile(r'^v_(?:mad_[iu]64_[iu]32|add_co_u32|sub_co_u32|subrev_co_u32|addc_co_u32|subb_co_u32|'
                     r'subbrev_co_u32|div_scale_f\d+)')
_STOP = ('s_branch', 's_setpc_b64', 's_swappc_b64', 's_endpgm', 's_trap', 's_rfe_b64')


def _regs(tok, kind):
    """register numbers of `kind` ('v' / 's') named by one operand token"""
    tok = tok.strip()
    m = re.match(r'^' + kind + r'\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'^' + kind + r'(\d+)$', tok)
    if m:
        return {int(m.group(1))}
    if kind == 's' and tok.startswith('vcc'):
        return {106, 107} if tok == 'vcc' else ({106} if tok == 'vcc_lo' else {107})
    if kind == 's' and tok.startswith('exec'):
        return {126, 127}
    return set()


def _operands(rest):
    # operands before the first modifier word (offset:, quad_perm:, row_..., off, glc ...)
    out = []
    for t in re.split(r',\s*', rest):
        t = t.strip()
        if not t:
            continue
        out.append(t.split()[0])
    return out


class Insn:
    __slots__ = ('op', 'ops', 'rest', 'line', 'dpp')

    def __init__(self, op, rest, line):
        self.op, self.rest, self.line = op, rest, line
        self.ops = _operands(rest)
        self.dpp = op.endswith('_dpp') or 'quad_perm:' in rest or 'row_' in rest or 'wave_' in rest

    def is_valu(self):
        return self.op.startswith('v_') and not self.op.startswith(('v_accvgpr',))

    def valu_sgpr_writes(self):
        if not self.is_valu():
            return set()
        if _VCOP3B.match(self.op) and len(self.ops) > 1:
            return _regs(self.ops[1], 's')
        if self.op.startswith(('v_cmp_', 'v_cmpx_', 'v_cmps_', 'v_cmpsx_')):
            if self.op.endswith('_e64') and self.ops:
                return _regs(self.ops[0], 's')
            return {106, 107}
        if self.op.startswith(('v_readlane', 'v_readfirstlane')) and self.ops:
            return _regs(self.ops[0], 's')
        if self.op.startswith(('v_add_co', 'v_sub_co', 'v_subrev_co', 'v_addc_co', 'v_subb_co')):
            return {106, 107}   # e32 forms: VCC
        return set()

    def valu_exec_write(self):
        return self.is_valu() and self.op.startswith(('v_cmpx', 'v_cmpsx'))

    def valu_vgpr_writes(self):
        if not self.is_valu() or not self.ops:
            return set()
        if self.op.startswith(('v_readlane', 'v_readfirstlane', 'v_cmp')):
            return set()
        w = _regs(self.ops[0], 'v')
        if self.op.startswith('v_permlane') and len(self.ops) > 1:
            w |= _regs(self.ops[1], 'v')   # the swaps write both operands
        return w

    def vmem(self):
        return self.op.startswith(('global_', 'buffer_', 'flat_', 'scratch_'))

    def smem(self):
        return self.op.startswith(('s_load_', 's_buffer_load_', 's_scratch_load', 's_dcache'))

    def sgpr_reads(self):
        out = set()
        for t in self.ops[1:] if (self.vmem() and 'store' not in self.op) or self.smem() else self.ops:
            out |= _regs(t, 's')
        return out

    def store_data(self):
        """data VGPRs of a VMEM store wider than 64 bits"""
        if not self.vmem() or 'store' not in self.op or not re.search(r'dwordx[34]|b96|b128', self.op):
            return set()
        # global/flat/scratch: store vaddr, vdata, ...; buffer: store vdata, vaddr, ...
        idx = 0 if self.op.startswith('buffer_') else 1
        return _regs(self.ops[idx], 'v') if len(self.ops) > idx else set()


def parse(lines):
    """[(function name, [Insn])] from llvm-objdump -d --no-show-raw-insn output"""
    funcs, cur = [], None
    for ln in lines:
        m = re.match(r'^[0-9a-f]+ <(.+)>:', ln)
        if m:
            cur = (m.group(1), [])
            funcs.append(cur)
            continue
        if cur is None:
            continue
        m = _INSN.match(ln)
        if m and not ln.strip().startswith(('//', ';')):
            cur[1].append(Insn(m.group(1), m.group(2), ln))
    return funcs


def _states(insns, i, j):
    n = 0
    for k in range(i + 1, j):
        m = re.match(r'^s_nop$', insns[k].op)
        n += (int(insns[k].ops[0], 0) + 1) if m and insns[k].ops else 1
    return n


def scan(lines):
    """-> (violations [(rule, function, producer line, consumer line, states, required)]
           -- RECORDED rules' hits included --, counts {rule: pairs checked (REQUIRED) or
           hits (RECORDED)}, lds_after_valu pairs)"""
    bad, counts, lds_pairs = [], dict.fromkeys(list(REQUIRED) + list(RECORDED), 0), 0
    for name, insns in parse(lines):
        for i, p in enumerate(insns):
            sw, vw = p.valu_sgpr_writes(), p.valu_vgpr_writes()
            xw = p.valu_exec_write()
            sd = p.store_data()
            sm = p.sgpr_reads() if p.smem() else set()
            if not (sw or vw or xw or sd or sm):
                continue
            for j in range(i + 1, min(i + 1 + LOOKAHEAD, len(insns))):
                c = insns[j]
                st = _states(insns, i, j)
                hits = []
                if sw and c.vmem() and sw & c.sgpr_reads():
                    hits.append('valu_sgpr_vmem')
                if sw and c.op.startswith(('v_readlane', 'v_writelane')) and len(c.ops) > 2 and sw & _regs(c.ops[2], 's'):
                    hits.append('valu_sgpr_lanesel')
                if vw and c.dpp and len(c.ops) > 1 and vw & _regs(c.ops[1], 'v'):
                    hits.append('valu_vgpr_dpp')
                if xw and c.dpp:
                    hits.append('valu_exec_dpp')
                if vw and c.op.startswith(('v_readlane', 'v_readfirstlane')) and len(c.ops) > 1 and \
                        vw & _regs(c.ops[1], 'v'):
                    hits.append('valu_vgpr_readlane')
                if vw and c.op.startswith('v_permlane') and vw & (set().union(*[_regs(t, 'v') for t in c.ops[:2]])):
                    hits.append('valu_vgpr_permlane')
                if sd and c.is_valu() and sd & c.valu_vgpr_writes():
                    hits.append('store_data_war')
                if sm and c.valu_sgpr_writes() & sm:
                    hits.append('smem_base_war')
                if vw and c.op.startswith('ds_') and vw & set().union(*[_regs(t, 'v') for t in c.ops]):
                    lds_pairs += 1
                for h in hits:
                    need = REQUIRED.get(h, RECORDED.get(h))
                    if h in RECORDED and st >= need:
                        continue
                    counts[h] += 1
                    if st < need:
                        bad.append((h, name, p.line.strip()[:70], c.line.strip()[:70], st, need))
                if c.op.startswith(_STOP):
                    break
    return bad, counts, lds_pairs
