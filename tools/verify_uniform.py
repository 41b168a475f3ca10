#!/usr/bin/env python3
"""Launch time of the verification kernel on uniform floods: n objects of one payload length, so every
wave has the same work.  Separates one wave's latency (n = 64 x SIMDs: one wave per SIMD) from the
throughput of several waves sharing a SIMD.  Prints one JSON line per (length, waves per SIMD)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pybitmessage_amd import _lib, targets, verify  # noqa: E402

SIMDS = 1024


def main():
    lib = _lib.get()
    for L in (16384 + 8 - 8, 2048, 46):
        for wps in (1, 2, 4, 6, 8):
            n = 64 * SIMDS * wps
            body = bytes(range(256)) * (L // 256 + 1)
            objs = [i.to_bytes(8, 'big') + body[:L] for i in range(n)]
            with verify.VerifyBatch(objs) as vb:
                first = vb.run()
                for i in (0, n // 2, n - 1):
                    assert int(first[i]) == targets.pow_value(objs[i]), i
                lib.bmpow_reset_stats()
                reps = 10
                t0 = time.perf_counter()
                for _ in range(reps):
                    vb.run(want=False)
                el = time.perf_counter() - t0
                st = _lib.BmpowStats()
                lib.bmpow_get_stats(ctypes.byref(st))
            blocks = (L + 17 + 127) // 128
            print(json.dumps({'payload': L, 'blocks': blocks, 'waves_per_simd': wps, 'objects': n,
                              'kernel_ms': round(st.verify_kernel_ms / reps, 4), 'wall_ms': round(el * 1e3 / reps, 4),
                              'us_per_block_per_wave': round(st.verify_kernel_ms / reps * 1e3 / (blocks + 2) / wps, 3),
                              'binned': os.environ.get('BMPOW_VBINNED')}), flush=True)


if __name__ == '__main__':
    main()
