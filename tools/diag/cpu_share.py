#!/usr/bin/env python3
"""What a spinning run() takes from another thread that wants the same CPU.

    python3 tools/diag/cpu_share.py [seconds]
A competitor process (a pure-Python counting loop) and a loop of C1 run() calls are pinned to the same
CPU.  Reported: the competitor's iterations per second alone and beside the calls, and the calls' rate
alone and beside it, with the library's spinning wait yielding the CPU every 64 polls (default) and
without (BMPOW_SPIN_YIELD=0).  Children of this script each initialise the GPU at most once."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def competitor(seconds, cpu):
    os.sched_setaffinity(0, {cpu})
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(10000):
            n += 1
    print(json.dumps({'iters_per_s': n / (time.perf_counter() - t0)}), flush=True)


def calls(seconds, cpu):
    os.sched_setaffinity(0, {cpu})
    sys.path.insert(0, ROOT)
    import hashlib
    import random
    from pybitmessage_amd import proofofwork, targets
    payload = random.Random(20250216).randbytes(1024)
    ih = hashlib.sha512(payload).digest()
    t = int(targets.object_target(1024, 345600))
    proofofwork.run(t, ih)
    print('ready', flush=True)
    sys.stdin.readline()
    t0, k = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        proofofwork.run(t, ih)
        k += 1
    el = time.perf_counter() - t0
    print(json.dumps({'calls': k, 'ghs': k * 10909138 / el / 1e9}), flush=True)


def run_pair(seconds, cpu, env_extra, with_comp, with_calls):
    env = dict(os.environ, **env_extra)
    env.setdefault('BMPOW_DEVICES', '0')
    me = os.path.abspath(__file__)
    cp = comp = None
    if with_calls:
        cp = subprocess.Popen([sys.executable, me, 'calls', str(seconds), str(cpu)], env=env, stdin=subprocess.PIPE,
                              stdout=subprocess.PIPE, text=True)
        assert cp.stdout.readline().strip() == 'ready'
    if with_comp:
        comp = subprocess.Popen([sys.executable, me, 'competitor', str(seconds), str(cpu)], stdout=subprocess.PIPE, text=True)
    if cp:
        cp.stdin.write('\n')
        cp.stdin.flush()
    out = {}
    if comp:
        out['competitor'] = json.loads(comp.communicate(timeout=seconds * 4 + 60)[0].strip().splitlines()[-1])
    if cp:
        out['calls'] = json.loads(cp.communicate(timeout=seconds * 4 + 120)[0].strip().splitlines()[-1])
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] in ('competitor', 'calls'):
        {'competitor': competitor, 'calls': calls}[sys.argv[1]](float(sys.argv[2]), int(sys.argv[3]))
        return
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
    cpu = sorted(os.sched_getaffinity(0))[1]
    res = {'cpu': cpu, 'seconds': seconds,
           'competitor_alone': run_pair(seconds, cpu, {}, True, False)['competitor'],
           'calls_alone': run_pair(seconds, cpu, {}, False, True)['calls']}
    for name, env in (('yield', {}), ('no_yield', {'BMPOW_SPIN_YIELD': '0'})):
        r = run_pair(seconds, cpu, env, True, True)
        r['competitor_share'] = round(r['competitor']['iters_per_s'] / res['competitor_alone']['iters_per_s'], 4)
        r['calls_share'] = round(r['calls']['ghs'] / res['calls_alone']['ghs'], 4)
        res[name] = r
    print(json.dumps(res))


if __name__ == '__main__':
    main()
