#!/usr/bin/env python3
"""One serial run() call's host/device timeline from a rocprofv3 trace of `bench.py --config c1`.

    rocprofv3 --kernel-trace --hip-trace --output-format csv -d D -o run -- python3 bench.py --config c1 ...
    python tools/c1_timeline.py D > profiles/r04/c1_trace/timeline.json

Each call of the single-object path (bmpow_host.hip search_one) launches bm_search1_kernel once per
window (a C1 object: one window), possibly with the next window queued behind.  A launch starts a new
call when it is issued after the previous search kernel ended.  The middle call's HIP API calls and
kernels are listed relative to its first launch, and every call's wall interval (first launch to the
next call's first launch), its hit kernel's duration and the host's share around it are summarised.
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = 'bm_search1_kernel'


def rows(root, suffix):
    paths = glob.glob(os.path.join(root, '**', '*' + suffix), recursive=True)
    out = []
    for p in paths:
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def main():
    root = sys.argv[1]
    kern = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows(root, 'kernel_trace.csv')))
    api = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in rows(root, 'hip_api_trace.csv')))
    launches = [a for a in api if a[2] in ('hipLaunchKernel', 'hipExtLaunchKernel', 'hipModuleLaunchKernel')]
    search = [k for k in kern if KERNEL in k[2]]
    # the run's last len(search) launches are the search kernels' (warmup included), in order
    launches = launches[-len(search):]
    first = [0] + [i for i in range(1, len(search)) if launches[i][0] > search[i - 1][1]]
    calls = []
    for a, b in zip(first, first[1:]):
        t0, t1 = launches[a][0], launches[b][0]
        hit = search[b - 1]  # the call's last awaited window holds the answer
        calls.append({'wall_us': (t1 - t0) / 1e3, 'hit_kernel_us': (hit[1] - hit[0]) / 1e3,
                      'launch_to_kernel_us': (search[a][0] - t0) / 1e3, 'kernel_end_to_next_call_us': (t1 - hit[1]) / 1e3,
                      'launches': b - a})
    mid = len(calls) // 2
    t0, t1 = launches[first[mid]][0], launches[first[mid + 1]][0]
    tl = [{'t_us': round((a[0] - t0) / 1e3, 1), 'dur_us': round((a[1] - a[0]) / 1e3, 1), 'what': 'API ' + a[2]}
          for a in api if t0 <= a[0] < t1]
    tl += [{'t_us': round((k[0] - t0) / 1e3, 1), 'dur_us': round((k[1] - k[0]) / 1e3, 1), 'what': 'KER ' + k[2]}
           for k in kern if t0 - 5000000 <= k[0] < t1 and k[1] > t0]
    tl.sort(key=lambda e: e['t_us'])

    def med(key):
        return round(statistics.median(c[key] for c in calls), 1)
    print(json.dumps({
        'source': 'rocprofv3 --kernel-trace --hip-trace over bench.py --config c1 (single-object path); '
                  'tools/c1_timeline.py',
        'calls': len(calls),
        'median': {k: med(k) for k in ('wall_us', 'hit_kernel_us', 'launch_to_kernel_us', 'kernel_end_to_next_call_us',
                                       'launches')},
        'timeline_one_call': tl}, indent=1))


if __name__ == '__main__':
    main()
