"""Where PowService's time goes at C5 test-mode scale (100k objects): the raw native service
(one submit, a bare poll loop) against PowService (per-object results), with poll timelines."""
import ctypes
import json
import sys
import time

import numpy as np

sys.path.insert(0, '.')
import bench  # noqa: E402
from pybitmessage_amd import _lib, proofofwork, worker  # noqa: E402

objs, _ = bench.make_objects('c5', 0, 100000, test_mode=True)
lib = _lib.get()
proofofwork.run_batch(objs[:20000])
P64 = ctypes.POINTER(ctypes.c_uint64)
out = {}


def stats():
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    return {'steps': st.steps, 'launches': st.launches, 'kernel_ms': round(st.kernel_ms, 1)}


# raw service: one submit of everything, a bare poll loop
ihs = b''.join(proofofwork._ih_bytes(ih) for _, ih in objs)
tg = np.array([proofofwork._clamp_target(t)[0] for t, _ in objs], dtype=np.uint64)
for rep in range(2):
    lib.bmpow_reset_stats()
    t0 = time.perf_counter()
    s = lib.bmpow_service_create(0, _lib.SERVICE_VERIFY)
    tk = np.zeros(len(objs), dtype=np.uint64)
    lib.bmpow_service_submit(s, len(objs), ihs, tg.ctypes.data_as(P64), tk.ctypes.data_as(P64))
    t1 = time.perf_counter()
    got, tl = 0, []
    a, b, c, d = (np.zeros(4096, dtype=np.uint64) for _ in range(4))
    while got < len(objs):
        k = lib.bmpow_service_poll(s, 4096, 1000, a.ctypes.data_as(P64), b.ctypes.data_as(P64), c.ctypes.data_as(P64),
                                   d.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        assert k >= 0
        got += k
        tl.append((round((time.perf_counter() - t0) * 1e3, 1), k))
    t2 = time.perf_counter()
    lib.bmpow_service_destroy(s)
    out['raw_%d' % rep] = {'submit_ms': round((t1 - t0) * 1e3, 1), 'total_ms': round((t2 - t0) * 1e3, 1),
                           'objects_per_s': round(len(objs) / (t2 - t0)), 'stats': stats(), 'timeline': tl[::8]}

for rep in range(2):
    lib.bmpow_reset_stats()
    t0 = time.perf_counter()
    svc = worker.PowService()
    svc.trace = []
    svc.start()
    t1 = time.perf_counter()
    futs = svc.submit_many(objs)
    t2 = time.perf_counter()
    res = [f.result() for f in futs]
    t3 = time.perf_counter()
    svc.stop(30)
    t4 = time.perf_counter()
    out['service_%d' % rep] = {'start_ms': round((t1 - t0) * 1e3, 1), 'submit_many_ms': round((t2 - t0) * 1e3, 1),
                               'results_ms': round((t3 - t0) * 1e3, 1), 'stop_ms': round((t4 - t0) * 1e3, 1),
                               'objects_per_s': round(len(objs) / (t3 - t0)), 'stats': stats(),
                               'timeline': [(round((t - t0) * 1e3, 1), k) for t, k in svc.trace][::8]}
print(json.dumps(out, indent=1))
