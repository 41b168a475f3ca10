#!/usr/bin/env python3
"""Serial run() calls' host/device timeline from a rocprofv3 trace of `bench.py --config c1`.

    rocprofv3 --kernel-trace --hip-trace --output-format csv -d D -o run -- python3 bench.py --config c1 ...
    python tools/c1_timeline.py D > timeline.json

Each call of the single-object path (bmpow_host.hip search_one) launches bm_search1_kernel once per
piece and window (one device: one launch per window; a split call: one per piece), in a burst; a launch
more than 200 us after the previous launch call returned starts a new call.  Per call:

* wall_us: first launch of the call to the first launch of the next call;
* host_exposed_us: the part of wall_us in which none of the call's kernels ran -- the time the
  device(s) waited for the host (the launch latency at the start, the result's trip home and the
  caller's return at the end);
* launch_span_us: first to last launch API call of the call's first window (the pieces' launches);
* api_us: the summed duration of the HIP API calls the calling thread made during the call;
* launch_to_kernel_us, kernel_end_to_next_call_us, launches, kernel_us (the longest kernel).
The middle call's API calls and kernels are listed relative to its first launch.
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = 'bm_search1_kernel'
GAP_NS = 200000
LAUNCH = ('hipLaunchKernel', 'hipExtLaunchKernel', 'hipModuleLaunchKernel')


def rows(root, suffix):
    out = []
    for p in glob.glob(os.path.join(root, '**', '*' + suffix), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def union_len(iv, lo, hi):
    iv = sorted((max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi)
    tot, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def main():
    root = sys.argv[1]
    kern = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows(root, 'kernel_trace.csv')))
    api = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function']) for r in rows(root, 'hip_api_trace.csv')))
    search = [k for k in kern if KERNEL in k[2]]
    launches = [a for a in api if a[2] in LAUNCH]
    # each search kernel's launch: by correlation id when the trace has it, else by issue order
    kr = [r for r in rows(root, 'kernel_trace.csv') if KERNEL in r['Kernel_Name']]
    ar = {r.get('Correlation_Id'): r for r in rows(root, 'hip_api_trace.csv') if r['Function'] in LAUNCH}
    pairs = []
    if kr and all(r.get('Correlation_Id') in ar for r in kr):
        for r in kr:
            a = ar[r['Correlation_Id']]
            pairs.append(((int(a['Start_Timestamp']), int(a['End_Timestamp']), a['Function']),
                          (int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])))
    else:
        pairs = list(zip(launches[-len(search):], sorted(search, key=lambda k: k[0])))
    pairs.sort(key=lambda p: p[0][0])
    # A call issues its launches in a burst (a window's pieces, and the window queued behind); calls
    # are separated by at least a kernel's run.  A launch more than GAP_NS after the previous launch
    # call returned starts a new call.  (A call whose first window ends without a hit launches its next
    # window later and is counted as two calls: for the C1 object of the bench the answer lies in the
    # first window.)
    calls, cur, prev_end = [], [], None
    for a, k in pairs:
        if cur and a[0] - prev_end > GAP_NS:
            calls.append(cur)
            cur = []
        cur.append((a, k))
        prev_end = a[1]
    if cur:
        calls.append(cur)
    out = []
    for c, nxt in zip(calls, calls[1:]):
        t0, t1 = c[0][0][0], nxt[0][0][0]
        ks = [k for _, k in c]
        first_window = [a for a, _ in c if a[0] < min(k[0] for k in ks)] or [c[0][0]]
        busy = union_len([(k[0], k[1]) for k in ks], t0, t1)
        out.append({'wall_us': (t1 - t0) / 1e3, 'host_exposed_us': (t1 - t0 - busy) / 1e3,
                    'launch_span_us': (first_window[-1][1] - first_window[0][0]) / 1e3,
                    'api_us': sum(min(a[1], t1) - a[0] for a in api if t0 <= a[0] < t1) / 1e3,
                    'launch_to_kernel_us': (min(k[0] for k in ks) - t0) / 1e3,
                    'kernel_end_to_next_call_us': (t1 - max(k[1] for k in ks)) / 1e3,
                    'kernel_us': max(k[1] - k[0] for k in ks) / 1e3, 'launches': len(c)})
    mid = len(out) // 2
    t0, t1 = calls[mid][0][0][0], calls[mid + 1][0][0][0]
    tl = [{'t_us': round((a[0] - t0) / 1e3, 1), 'dur_us': round((a[1] - a[0]) / 1e3, 1), 'what': 'API ' + a[2]}
          for a in api if t0 <= a[0] < t1]
    tl += [{'t_us': round((k[0] - t0) / 1e3, 1), 'dur_us': round((k[1] - k[0]) / 1e3, 1), 'what': 'KER ' + k[2]}
           for k in kern if t0 - 5000000 <= k[0] < t1 and k[1] > t0]
    tl.sort(key=lambda e: e['t_us'])

    def med(key):
        return round(statistics.median(x[key] for x in out), 1)
    print(json.dumps({
        'source': 'rocprofv3 --kernel-trace --hip-trace over bench.py --config c1 (single-object path); '
                  'tools/c1_timeline.py',
        'calls': len(out),
        'median': {k: med(k) for k in ('wall_us', 'host_exposed_us', 'launch_span_us', 'api_us', 'launch_to_kernel_us',
                                       'kernel_end_to_next_call_us', 'kernel_us', 'launches')},
        'timeline_one_call': tl}, indent=1))


if __name__ == '__main__':
    main()
