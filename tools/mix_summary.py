#!/usr/bin/env python3
"""profiles/mix_ceiling.json from a tools/ubench_mix run (JSON lines): the best VALU issue rate per
SIMD per quad-cycle of the kernel's dependence-free mix at the kernel's own occupancy, and the table
of every variant.

    python tools/mix_summary.py profiles/r04/ubench_mix.jsonl [waves=5]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    waves = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = [json.loads(l) for l in open(src) if l.strip()]
    head = rows[0]
    runs = [r for r in rows[1:] if 'variant' in r]
    table = {}
    for r in runs:
        key = '%s_w%d' % (r['variant'], r['waves_per_simd'])
        table[key] = max(table.get(key, 0.0), r['valu_per_simd_quadcycle'])
    # the free-running streams (no barrier); the phased ones are reported apart
    free = {k: v for k, v in table.items() if not k.startswith('phased')}
    at = {k: v for k, v in free.items() if k.endswith('_w%d' % waves)}
    out = {'source': os.path.relpath(src, ROOT), 'device': head.get('device'), 'mix': head.get('mix'),
           'valu_per_iter': head.get('valu_per_iter'), 'waves_per_simd': waves,
           'ceiling_valu_per_simd_quadcycle': round(max(at.values()), 4),
           'best_variant': max(at, key=at.get),
           'max_over_every_occupancy': round(max(free.values()), 4),
           'table_valu_per_simd_quadcycle': {k: round(v, 4) for k, v in sorted(table.items())}}
    if 'phased_w4' in table:
        # every bitop3 of the iteration first, the waves of a SIMD meeting at a barrier before them
        out['phased_valu_per_simd_quadcycle'] = round(table['phased_w4'], 4)
        out['phased_nobar_valu_per_simd_quadcycle'] = round(table.get('phased_nobar_w4', 0.0), 4)
    with open(os.path.join(ROOT, 'profiles', 'mix_ceiling.json'), 'w') as f:
        json.dump(out, f, indent=1)
        f.write('\n')
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
