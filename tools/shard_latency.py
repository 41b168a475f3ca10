"""Latency of run_batch for a few C1-sized objects (1 KB msg at defaults, E ~ 1.3e7 trials) with 1
and 8 shards on one device: over several shards a window is capped at ~2E (bmsched::expect_cap)."""
import ctypes
import hashlib
import json
import random
import sys
import time

sys.path.insert(0, '.')
import bench  # noqa: E402
from pybitmessage_amd import _lib, proofofwork  # noqa: E402

lib = _lib.get()
rng = random.Random(5)
out = {}
for nobj in (1, 2, 8):
    objs = [(bench.object_target(1024, 345600), hashlib.sha512(rng.randbytes(1024)).digest()) for _ in range(nobj)]
    for shards in (1, 8):
        ids = (ctypes.c_int * shards)(*([0] * shards))
        _lib.check(lib, lib.bmpow_set_devices(ids, shards), 'set_devices')
        proofofwork.run_batch(objs)
        lib.bmpow_reset_stats()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            res = proofofwork.run_batch(objs)
            ts.append(time.perf_counter() - t0)
        st = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(st))
        out['%d_objects_%d_shards' % (nobj, shards)] = {
            'ms_median': round(sorted(ts)[2] * 1e3, 2), 'trials_per_call': st.trials // 5,
            'useful_per_call': sum(n for _, n in res), 'steps_per_call': st.steps / 5}
ids = (ctypes.c_int * 1)(0)
lib.bmpow_set_devices(ids, 1)
print(json.dumps(out, indent=1))
