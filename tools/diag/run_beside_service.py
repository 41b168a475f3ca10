#!/usr/bin/env python3
"""A serial run() while the batch service is busy (PyBitmessage's API thread, api.py:1304, beside its
worker thread's batches): the latency of C1-like run() calls made while a PowService works through a
batch of hard objects, against the same calls alone, and how far the service's batch got meanwhile.

    python3 tools/diag/run_beside_service.py [calls] [batch_objects]

One JSON line: run() latency (median / max ms) alone and beside the service, the service's objects
finished and trials hashed during the calls, and its rate before and during them.
"""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
U64 = (1 << 64) - 1


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nobj = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    os.environ.setdefault('BMPOW_DEVICES', '0')
    from pybitmessage_amd import proofofwork, worker
    rng = random.Random(77)
    c1 = [(U64 // 12_750_000, rng.randbytes(64)) for _ in range(calls)]  # E ~ C1's 1.3e7 trials

    def timed(objs):
        out = []
        for t, ih in objs:
            t0 = time.perf_counter()
            proofofwork.run(t, ih)
            out.append((time.perf_counter() - t0) * 1e3)
        return out

    timed(c1[:3])  # warm
    alone = timed(c1)
    # the service: hard objects (E ~ 2e9, ~0.3 s each at 6.6 GH/s), more than the calls outlast
    batch = [(U64 // 2_000_000_000, rng.randbytes(64)) for _ in range(nobj)]
    svc = worker.PowService().start()
    futs = svc.submit_many(batch)

    def finished():
        return sum(1 for f in futs if f.done())
    time.sleep(2.0)
    f0 = finished()
    t0 = time.perf_counter()
    beside = timed(c1)
    t1 = time.perf_counter()
    f1 = finished()
    time.sleep(t1 - t0)
    f2 = finished()
    svc.stop(60)
    print(json.dumps({
        'calls': calls, 'service_objects': nobj,
        'alone_ms': {'median': round(statistics.median(alone), 3), 'max': round(max(alone), 3)},
        'beside_service_ms': {'median': round(statistics.median(beside), 3), 'max': round(max(beside), 3),
                              'all': [round(x, 2) for x in beside]},
        'calls_span_s': round(t1 - t0, 3),
        'service_finished_during_calls': f1 - f0, 'service_finished_same_span_after': f2 - f1,
        'service_finished_in_first_2s': f0}), flush=True)


if __name__ == '__main__':
    main()
