#!/usr/bin/env python3
"""Fixed cost of one single-object launch (bmpow_host.hip search_one, bm_search1_kernel): windows
of N nonces with no hit (target 0), N = 2^20 .. 2^27, 20 calls each; per call the wall time and the
kernel's own span (s_memrealtime, bmpow_stats.kernel_ms).  A least-squares line t = a + N / rate gives
the per-launch fixed cost a (launch, ramp, last partial row) and the streaming rate.

    python3 tools/diag/c1_overhead.py > gpurun_out/.../c1_overhead.json
"""
import ctypes
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from pybitmessage_amd import _lib  # noqa: E402


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    return my - b * mx, b


def main():
    lib = _lib.get()
    ih = hashlib.sha512(b'c1-overhead').digest()
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    st = _lib.BmpowStats()
    rows = []
    for lg in range(20, 28):
        N = 1 << lg
        for _ in range(3):  # warm
            lib.bmpow_search(ih, 0, 1, N, ctypes.byref(n), ctypes.byref(t))
        walls, kms = [], []
        for _ in range(20):
            lib.bmpow_reset_stats()
            c = time.perf_counter()
            rc = lib.bmpow_search(ih, 0, 1, N, ctypes.byref(n), ctypes.byref(t))
            walls.append((time.perf_counter() - c) * 1e3)
            assert rc == _lib.NOT_FOUND, rc
            lib.bmpow_get_stats(ctypes.byref(st))
            assert st.trials == N, (st.trials, N)
            kms.append(st.kernel_ms)
        walls.sort()
        kms.sort()
        rows.append({'nonces': N, 'wall_ms_median': round(walls[10], 4), 'kernel_ms_median': round(kms[10], 4)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    xs = [r['nonces'] for r in rows]
    aw, bw = fit(xs, [r['wall_ms_median'] for r in rows])
    ak, bk = fit(xs, [r['kernel_ms_median'] for r in rows])
    print(json.dumps({'rows': rows,
                      'wall_fit': {'fixed_us': round(aw * 1e3, 2), 'ghs': round(1e-6 / bw, 4)},
                      'kernel_fit': {'fixed_us': round(ak * 1e3, 2), 'ghs': round(1e-6 / bk, 4)},
                      'how': 'least squares t = a + N / rate over the medians of 20 calls per N (target 0, no hit)'},
                     indent=1))


if __name__ == '__main__':
    main()
