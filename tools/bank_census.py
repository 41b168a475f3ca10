#!/usr/bin/env python3
"""VGPR bank census of v_bitop3_b32 in a kernel's hot loop (hipcc -save-temps .s).

    python tools/bank_census.py <file.s> [kernel_substring]

gfx950 co-issues two waves' v_bitop3_b32 in one quad-cycle only when an instruction's three
source VGPRs are not all in one bank (bank = register number mod 4; profiles/r01_ubench_coissue.json:
'banks 000' / '222' run at the single-issue rate, every other pattern at twice it).  Counts the
bitop3 whose sources share one bank, per pattern.
"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
import isa_census as ic  # noqa: E402


def loop_body(path, name):
    body = ic.kernel_lines(path, name)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.match(r'^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)', l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < i:
                sp = (labels[t], i)
                if best is None or sp[1] - sp[0] > best[1] - best[0]:
                    best = sp
    return body[best[0]:best[1] + 1]


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else 'bm_search_kernel'
    pats = collections.Counter()
    total = 0
    for l in loop_body(path, name):
        m = re.match(r'^\s+v_bitop3_b32\s+(.*)', l)
        if not m:
            continue
        ops = [o.strip() for o in m.group(1).split(';')[0].split(',')]
        srcs = ops[1:4]
        regs = [int(m2.group(1)) for m2 in (re.match(r'v(\d+)\b', o) for o in srcs) if m2]
        total += 1
        if len(regs) < 3:
            pats['non-vgpr source'] += 1
            continue
        banks = tuple(r % 4 for r in regs)
        kind = 'all three in one bank' if len(set(banks)) == 1 else ('two share a bank' if len(set(banks)) == 2 else 'three banks')
        pats[kind] += 1
    print('%s: %d v_bitop3_b32 in the loop' % (path, total))
    for k, v in pats.most_common():
        print('  %-24s %5d  (%.1f %%)' % (k, v, 100.0 * v / max(total, 1)))


if __name__ == '__main__':
    main()
