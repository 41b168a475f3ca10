#!/usr/bin/env python3
"""Instruction census of a kernel's hot loop in a hipcc -save-temps .s file.

    python tools/isa_census.py <file.s> [kernel_substring]

Finds the kernel's body, locates the largest basic-block range that ends in a backward
branch (the nonce loop), and counts instructions by mnemonic class.  Used to check what
the compiler emitted per trial (issued VALU ops per trial vs the 8,288-op
algorithmic count).
"""
import collections
import re
import sys


def kernel_lines(path, name):
    lines = open(path).read().split('\n')
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r'^_\w*%s\w*:\s*(;.*)?$' % re.escape(name), l):
            start = i
        elif start is not None and l.strip().startswith('.Lfunc_end'):
            return lines[start:i]
    raise SystemExit('kernel %s not found' % name)


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else 'bm_search_kernel'
    body = kernel_lines(path, name)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.match(r'^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)', l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                span = (labels[tgt], i)
                if best is None or span[1] - span[0] > best[1] - best[0]:
                    best = span
    if best is None:
        raise SystemExit('no loop found')
    cnt = collections.Counter()
    for l in body[best[0]:best[1] + 1]:
        m = re.match(r'^\s+([vsdgb][a-z0-9_]+)', l)
        if m:
            cnt[m.group(1)] += 1
    valu = sum(v for k, v in cnt.items() if k.startswith('v_'))
    salu = sum(v for k, v in cnt.items() if k.startswith('s_'))
    print('loop lines %d..%d  VALU=%d  SALU=%d' % (best[0], best[1], valu, salu))
    for k, v in cnt.most_common(40):
        print('  %-28s %d' % (k, v))


if __name__ == '__main__':
    main()
