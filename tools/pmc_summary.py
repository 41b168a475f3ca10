#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output for bm_search_kernel (per launch, averaged).

    python tools/pmc_summary.py gpurun_out/pmc_r01 [trials_per_launch] > profiles/pmc_latest.json

The summary is stamped with the build it measured ("build"): the md5 of the libbmpow_hip.so the GPU
box ran (OUTDIR/lib.md5, written by tools/profile_pmc.sh) and of its device code (OUTDIR/code.md5,
tools/lib_code_md5.py: the .hip_fatbin section, reproduced by a rebuild), the library's version string from the
bench line, and the git commit checked out here when summarising.

Derived (MI355X_MICROARCH.md conventions):
  * issued VALU instructions per trial = SQ_INSTS_VALU x 64 / trials
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (sum over XCDs)
  * VALU issue utilisation = (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SIMD quad-cycles, with
    SIMD quad-cycles = 1,024 SIMDs x (GRBM_GUI_ACTIVE / 8) / 4: the share of every SIMD's quad-cycles
    in which it issued at least one VALU instruction (SQ_ACTIVE_INST_VALU counts one quad-cycle per
    wave-instruction -- it equals SQ_INSTS_VALU here -- and SQ_ACTIVE_INST_VALU2 the quad-cycles in
    which a SIMD issued two); dual-issue share = VALU2 / ACTIVE_INST_VALU.  rocprof's own VALUBusy
    (100 x ACTIVE_INST_VALU / CUs / GRBM, its gfx94x formula) is reported beside it.
  * HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE reads half the bytes of wide streams
    on gfx950 (guide §HBM); this kernel's reads are scalar/64-bit, so the doubled figure is an upper bound.
"""
import collections
import csv
import json
import os
import subprocess
import sys

KERNEL = os.environ.get('PMC_KERNEL', 'bm_search_kernel')  # bm_search1_kernel: run()'s kernel (PMC_ONE)


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
    for p in ['instr', 'busy', 'issue', 'valu', 'fetch', 'write']:
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
        if out.get('SQ_INSTS_SALU') is not None:
            res['salu_instr_per_trial'] = out['SQ_INSTS_SALU'] * 64 / trials
            res['waves_per_launch'] = out['SQ_WAVES']
    if out.get('GRBM_GUI_ACTIVE') and out.get('instr_ns'):
        res['eff_clock_ghz'] = out['GRBM_GUI_ACTIVE'] / 8 / out['instr_ns']
    if out.get('SQ_ACTIVE_INST_VALU2') is not None and out.get('GRBM_GUI_ACTIVE'):
        quad = 1024 * out['GRBM_GUI_ACTIVE'] / 8 / 4  # SIMD quad-cycles per launch
        res['valu_issue_util'] = (out['SQ_ACTIVE_INST_VALU'] - out['SQ_ACTIVE_INST_VALU2']) / quad
        res['valu_instr_per_simd_quad_cycle'] = out['SQ_ACTIVE_INST_VALU'] / quad
        res['dual_issue_share'] = out['SQ_ACTIVE_INST_VALU2'] / out['SQ_ACTIVE_INST_VALU']
        res['rocprof_VALUBusy_pct'] = 100 * out['SQ_ACTIVE_INST_VALU'] / 256 / out['GRBM_GUI_ACTIVE'] * 8
        if out.get('SQ_BUSY_CU_CYCLES'):
            res['simd_busy_frac'] = out['SQ_BUSY_CU_CYCLES'] / quad
        if out.get('SQ_WAVE_CYCLES'):
            res['wave_issue_stall_share'] = out['SQ_WAIT_INST_ANY'] / out['SQ_WAVE_CYCLES']
            if out.get('SQ_WAIT_ANY') is not None:
                res['wave_wait_share'] = out['SQ_WAIT_ANY'] / out['SQ_WAVE_CYCLES']
        if out.get('issue_ns'):
            res['eff_clock_ghz_issue_pass'] = out['GRBM_GUI_ACTIVE'] / 8 / out['issue_ns']
    if out.get('SQ_INSTS_VALU_INT32') is not None:
        res['int32_per_trial'] = out['SQ_INSTS_VALU_INT32'] * 64 / trials
        res['int64_per_trial'] = out['SQ_INSTS_VALU_INT64'] * 64 / trials
    if out.get('FETCH_SIZE') is not None:
        res['fetch_kb_per_launch'] = out['FETCH_SIZE']
    if out.get('WRITE_SIZE') is not None:
        res['write_kb_per_launch'] = out['WRITE_SIZE']
    if out.get('FETCH_SIZE') is not None and out.get('WRITE_SIZE') is not None:
        res['hbm_bytes_per_launch_upper'] = (2 * out['FETCH_SIZE'] + out['WRITE_SIZE']) * 1024
    build = {}
    md5 = os.path.join(root, 'lib.md5')
    if os.path.exists(md5):
        build['lib_md5'] = open(md5).read().split()[0]
    cmd5 = os.path.join(root, 'code.md5')  # the device code's md5 (tools/lib_code_md5.py): survives rebuilds
    if os.path.exists(cmd5):
        build['code_md5'] = open(cmd5).read().split()[0]
    for p in ['instr', 'kt']:
        bj = os.path.join(root, p + '.bench.json')
        if os.path.exists(bj):
            lines = [l for l in open(bj) if l.startswith('{')]
            if lines:
                build['lib_version'] = json.loads(lines[-1]).get('config', {}).get('lib')
                break
    try:
        build['git_head'] = subprocess.check_output(['git', 'rev-parse', '--short=12', 'HEAD'], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        pass
    build['outdir'] = root
    print(json.dumps({'build': build, 'raw': out, 'derived': res}, indent=1))


if __name__ == '__main__':
    main()
