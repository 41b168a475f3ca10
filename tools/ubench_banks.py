"""Generates tools/ubench_banks.hip: issue rate of 3-source VALU ops vs the VGPR banks of their
operands (explicit registers in inline asm, 8 independent chains, dst = src0)."""
import os

def chains3(op, x, y, z, tail=''):
    """8 chains, chain c: A = bitop3(A, B, C) with A, B, C its own registers in banks x, y, z."""
    regs = [(8 + 12 * c + x, 8 + 12 * c + 4 + y, 8 + 12 * c + 8 + z) for c in range(8)]
    return [op + ' v%d, v%d, v%d, v%d' % (a, a, b, cc) + tail for a, b, cc in regs]


def seq_sigma(banks_ok):
    """Sigma-like: per chain r1..r3 = alignbit(x, x2, n); x = bitop3(r1, r2, r3)."""
    out = []
    for c in range(8):
        base = 8 + 12 * c
        x, x2 = base, base + 1
        r = [base + 5, base + 6, base + 7] if banks_ok else [base + 4, base + 8, base + 4 + 4 * 0 + 0]
        if not banks_ok:
            r = [base + 4, base + 8, base + 0 + 0]  # all bank 0 (the last one overwrites x's bank)
            r = [base + 4, base + 8, base + 2]
        out.append((c, x, x2, r))
    lines = []
    for c, x, x2, r in out:
        lines += ['v_alignbit_b32 v%d, v%d, v%d, %d' % (r[0], x, x2, 7),
                  'v_alignbit_b32 v%d, v%d, v%d, %d' % (r[1], x2, x, 13),
                  'v_alignbit_b32 v%d, v%d, v%d, %d' % (r[2], x, x2, 19)]
    for c, x, x2, r in out:
        lines.append('v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96' % (x, r[0], r[1], r[2]))
    return lines


def mixed(second, group):
    """8 chains of alignbit (own registers, banks 0/1) and 8 of `second` (banks 1/2/3), issued in
    groups of `group` instructions of each kind."""
    al = ['v_alignbit_b32 v%d, v%d, v%d, 7' % (8 + 12 * c, 8 + 12 * c, 9 + 12 * c) for c in range(8)]
    if second == 'xor':
        sc = ['v_xor_b32 v%d, v%d, v%d' % (13 + 12 * c, 13 + 12 * c, 14 + 12 * c) for c in range(8)]
    else:
        sc = ['v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96' % (13 + 12 * c, 13 + 12 * c, 14 + 12 * c, 15 + 12 * c)
              for c in range(8)]
    out = []
    for g in range(0, 8, group):
        out += al[g:g + group] + sc[g:g + group]
    return out


PATS = []
PATS.append(('bitop3 banks 012, 4 waves/SIMD', chains3('v_bitop3_b32', 0, 1, 2, tail=' bitop3:0x96'), 1, 0))
PATS.append(('alignbit banks 01', [l.rsplit(',', 1)[0] + ', 7' for l in chains3('v_alignbit_b32', 0, 1, 2)], 1, 0))
PATS.append(('mad_u64_u32 (per instr)', ['v_mad_u64_u32 v[%d:%d], s[44:45], v%d, v%d, v[%d:%d]' % (8 + 12 * c, 9 + 12 * c, 12 + 12 * c, 13 + 12 * c, 8 + 12 * c, 9 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('mul_lo_u32', ['v_mul_lo_u32 v%d, v%d, v%d' % (8 + 12 * c, 8 + 12 * c, 13 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('mul_hi_u32', ['v_mul_hi_u32 v%d, v%d, v%d' % (8 + 12 * c, 8 + 12 * c, 13 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('fma_f64', ['v_fma_f64 v[%d:%d], v[%d:%d], v[%d:%d], v[%d:%d]' % (8 + 12 * c, 9 + 12 * c, 8 + 12 * c, 9 + 12 * c, 14 + 12 * c, 15 + 12 * c, 16 + 12 * c, 17 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('add_co_u32 e32 (vcc)', ['v_add_co_u32_e32 v%d, vcc, v%d, v%d' % (8 + 12 * c, 8 + 12 * c, 13 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('addc_co_u32 e32 (vcc in/out)', ['v_addc_co_u32_e32 v%d, vcc, v%d, v%d, vcc' % (8 + 12 * c, 8 + 12 * c, 13 + 12 * c) for c in range(8)], 1, 0))
PATS.append(('add_co_u32 e64 (sgpr carry)', ['v_add_co_u32_e64 v%d, s[%d:%d], v%d, v%d' % (8 + 12 * c, 46 + 2 * (c % 4), 47 + 2 * (c % 4), 8 + 12 * c, 13 + 12 * c) for c in range(8)], 1, 0))

CLOB = ', '.join('"v%d"' % i for i in range(112)) + ', "s40", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "vcc"'


def body(lines, reps):
    reps = reps or 2
    return '\\n\\t'.join(lines * (64 // (len(lines) * 1) if reps == 1 else 2))


def main():
    src = ['#define CLOB_ALL ' + ', '.join('"v%d"' % i for i in range(112))]
    src += [open(os.path.join(os.path.dirname(__file__), 'ubench_banks_head.hip')).read()]
    for i, (name, lines, reps, occ) in enumerate(PATS):
        src.append('template <> __device__ __forceinline__ void step<%d>() { asm volatile("%s" ::: %s); }'
                   % (i, body(lines, reps), CLOB))
    src.append('int main() {\n  SETUP();')
    for i, (name, lines, reps, occ) in enumerate(PATS):
        n = len(body(lines, reps).split('\\n\\t'))
        bar = int(name[4:name.index(' ')]) if name.startswith('SYNC') else -1
        src.append('  rc |= run<%d, %d>("%s", %d, %s, dout, dclk);' % (i, bar, name, n, 'blocks' if not occ else 'p.multiProcessorCount * %d' % occ))
    src.append('  return rc;\n}')
    open(os.path.join(os.path.dirname(__file__), 'ubench_banks.hip'), 'w').write('\n'.join(src) + '\n')


if __name__ == '__main__':
    main()
