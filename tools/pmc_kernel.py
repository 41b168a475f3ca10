#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (one counter group per pass directory).

    python tools/pmc_kernel.py ROOT KERNEL_SUBSTRING [--units N] [--out FILE]

Sums every dispatch of the kernel in each pass and divides by the dispatch count (per launch).
Derived as in tools/pmc_summary.py (MI355X_MICROARCH.md conventions): SIMD quad-cycles =
1,024 x GRBM_GUI_ACTIVE / 8 / 4; VALU issue utilisation = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) /
quad-cycles; instructions per SIMD quad-cycle = ACTIVE_INST_VALU / quad-cycles; HBM bytes =
2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; FETCH_SIZE counts half of a wide stream's bytes on gfx950).
--units: work units in the whole profiled run (objects, tries) for per-unit figures."""
import argparse
import collections
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('root')
    ap.add_argument('kernel')
    ap.add_argument('--units', type=float, default=0)
    ap.add_argument('--out')
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    launches, ns = {}, {}
    for p in sorted(os.listdir(a.root)):
        path = os.path.join(a.root, p, 'run_counter_collection.csv')
        if not os.path.exists(path):
            continue
        disp = set()
        with open(path) as f:
            for row in csv.DictReader(f):
                if a.kernel not in row['Kernel_Name']:
                    continue
                tot[row['Counter_Name']] += float(row['Counter_Value'])
                if row['Dispatch_Id'] not in disp:
                    disp.add(row['Dispatch_Id'])
                    ns[p] = ns.get(p, 0) + int(row['End_Timestamp']) - int(row['Start_Timestamp'])
        launches[p] = len(disp)
    n = max(launches.values()) if launches else 0
    if not n or len(set(launches.values())) != 1:
        raise SystemExit('dispatch counts differ between passes: %s' % launches)
    raw = {k: v / n for k, v in tot.items()}
    out = {'kernel': a.kernel, 'launches': n, 'kernel_ns_per_launch': sum(ns.values()) / len(ns) / n, 'raw': raw}
    d = {}
    g = raw.get('GRBM_GUI_ACTIVE')
    if g and raw.get('SQ_ACTIVE_INST_VALU') is not None:
        quad = 1024 * g / 8 / 4
        d['eff_clock_ghz'] = g / 8 / out['kernel_ns_per_launch']
        d['valu_instr_per_simd_quad_cycle'] = raw['SQ_ACTIVE_INST_VALU'] / quad
        if raw.get('SQ_ACTIVE_INST_VALU2') is not None:
            d['valu_issue_util'] = (raw['SQ_ACTIVE_INST_VALU'] - raw['SQ_ACTIVE_INST_VALU2']) / quad
            d['dual_issue_share'] = raw['SQ_ACTIVE_INST_VALU2'] / raw['SQ_ACTIVE_INST_VALU']
        if raw.get('SQ_BUSY_CU_CYCLES') is not None:
            d['simd_busy_frac'] = raw['SQ_BUSY_CU_CYCLES'] / quad
    if raw.get('FETCH_SIZE') is not None and raw.get('WRITE_SIZE') is not None:
        d['hbm_bytes_per_launch'] = (2 * raw['FETCH_SIZE'] + raw['WRITE_SIZE']) * 1024
    if a.units and raw.get('SQ_INSTS_VALU'):
        d['units'] = a.units
        d['valu_lane_instr_per_unit'] = raw['SQ_INSTS_VALU'] * n * 64 / a.units
        if 'hbm_bytes_per_launch' in d:
            d['hbm_bytes_per_unit'] = d['hbm_bytes_per_launch'] * n / a.units
    out['derived'] = d
    s = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(s + '\n')
    print(s)


if __name__ == '__main__':
    main()
