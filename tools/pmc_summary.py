#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output for bm_search_kernel (per launch, averaged).

    python tools/pmc_summary.py gpurun_out/pmc_r01 [trials_per_launch]

Derived (MI355X_MICROARCH.md conventions):
  * issued VALU instructions per trial = SQ_INSTS_VALU x 64 / trials
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (sum over XCDs)
  * VALU busy = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (256 CUs x GRBM_GUI_ACTIVE / 8)  [per-CU share]
  * HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE reads half the bytes of wide streams
    on gfx950 (guide §HBM); this kernel's reads are scalar/64-bit, so the doubled figure is an upper bound.
"""
import collections
import csv
import json
import os
import sys

KERNEL = 'bm_search_kernel'


def load(path):
    per = collections.defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL not in row['Kernel_Name']:
                continue
            d = per[int(row['Dispatch_Id'])]
            d[row['Counter_Name']] = d.get(row['Counter_Name'], 0.0) + float(row['Counter_Value'])
            d['_ns'] = int(row['End_Timestamp']) - int(row['Start_Timestamp'])
    return per


def avg(per, name):
    vals = [d[name] for d in per.values() if name in d]
    return sum(vals) / len(vals) if vals else None


def main():
    root = sys.argv[1]
    trials = float(sys.argv[2]) if len(sys.argv) > 2 else float(1 << 28)
    out = {'trials_per_launch': trials}
    for p in ['instr', 'busy', 'valu', 'fetch', 'write']:
        path = os.path.join(root, p, 'run_counter_collection.csv')
        if not os.path.exists(path):
            continue
        per = load(path)
        out[p + '_launches'] = len(per)
        for name in sorted({k for d in per.values() for k in d if not k.startswith('_')}):
            out[name] = avg(per, name)
        out[p + '_ns'] = avg(per, '_ns')
    res = {}
    if out.get('SQ_INSTS_VALU'):
        res['valu_instr_per_trial'] = out['SQ_INSTS_VALU'] * 64 / trials
        res['salu_instr_per_trial'] = out['SQ_INSTS_SALU'] * 64 / trials
        res['waves_per_launch'] = out['SQ_WAVES']
    if out.get('GRBM_GUI_ACTIVE') and out.get('instr_ns'):
        res['eff_clock_ghz'] = out['GRBM_GUI_ACTIVE'] / 8 / out['instr_ns']
    if out.get('SQ_ACTIVE_INST_VALU') and out.get('busy_ns'):
        cyc = out['busy_ns'] * res.get('eff_clock_ghz', 2.4)
        res['valu_busy_frac'] = out['SQ_ACTIVE_INST_VALU'] * 4 / 256 / cyc / 4  # 4 SIMDs per CU
        res['wave_cycles_per_trial'] = out['SQ_WAVE_CYCLES'] * 4 * 64 / trials
    if out.get('SQ_INSTS_VALU_INT32') is not None:
        res['int32_per_trial'] = out['SQ_INSTS_VALU_INT32'] * 64 / trials
        res['int64_per_trial'] = out['SQ_INSTS_VALU_INT64'] * 64 / trials
    if out.get('FETCH_SIZE') is not None:
        res['fetch_kb_per_launch'] = out['FETCH_SIZE']
    if out.get('WRITE_SIZE') is not None:
        res['write_kb_per_launch'] = out['WRITE_SIZE']
    if out.get('FETCH_SIZE') is not None and out.get('WRITE_SIZE') is not None:
        res['hbm_bytes_per_launch_upper'] = (2 * out['FETCH_SIZE'] + out['WRITE_SIZE']) * 1024
    print(json.dumps({'raw': out, 'derived': res}, indent=1))


if __name__ == '__main__':
    main()
