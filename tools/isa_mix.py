"""Instruction mix per basic block of one kernel in a hipcc -S listing.

    python tools/isa_mix.py k.s k_curve_half [--top 12]

Prints, for the largest blocks (by instruction count), the number of
instructions per class: MAD (v_mad_u64_u32), 64-bit VALU, other VALU, VMEM,
SALU, waitcnt, nop.  Used to read where the non-MAD issue cycles of the field
code go."""
import re
import sys
from collections import Counter

def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index('--top') + 1]) if '--top' in sys.argv else 12
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + name + r'\S*:', l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    blocks, cur, label = [], [], 'entry'
    for l in lines[start + 1:end]:
        s = l.strip()
        if re.match(r'^\.?L?\w+:', s) and not s.startswith(';'):
            blocks.append((label, cur))
            label, cur = s.split(':')[0], []
            continue
        if not s or s.startswith(';') or s.startswith('.'):
            continue
        cur.append(s.split()[0])
    blocks.append((label, cur))
    def cls(op):
        if op == 'v_mad_u64_u32': return 'mad'
        if op.startswith('v_mul_lo_u32'): return 'mul_lo'
        if re.search(r'_(b|u|i)64', op) or op.startswith('v_lshl_add_u64'): return 'valu64'
        if op.startswith('v_cndmask'): return 'cndmask'
        if op.startswith(('v_accvgpr', 'v_mov')): return 'mov'
        if op.startswith('v_'): return 'valu32'
        if op.startswith(('global_', 'buffer_', 'scratch_', 'flat_')): return 'vmem'
        if op.startswith('ds_'): return 'lds'
        if op.startswith('s_waitcnt'): return 'waitcnt'
        if op.startswith('s_nop'): return 'nop'
        if op.startswith('s_'): return 'salu'
        return 'other'
    tot = Counter()
    for _, ins in blocks:
        tot.update(cls(o) for o in ins)
    print('kernel total', sum(tot.values()), dict(tot))
    for label, ins in sorted(blocks, key=lambda b: -len(b[1]))[:top]:
        c = Counter(cls(o) for o in ins)
        print('{:>14} {:6d} {}'.format(label, len(ins), dict(c.most_common())))

if __name__ == '__main__':
    main()
