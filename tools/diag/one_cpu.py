#!/usr/bin/env python3
"""Host CPU of run()'s single-object path while the GPU works, per wait configuration and per thread.

    python3 tools/diag/one_cpu.py            # parent: one child process per configuration, JSON lines
Each child initialises the library on device 0, warms up, then times a no-hit sweep (target 0) of
2^LOG2 nonces and reports its process CPU per wall-second and the CPU of every thread of the process
(/proc/self/task/*/stat utime + stime, with the thread's name), so a busy thread of the HIP runtime
shows up apart from the calling thread."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CONFIGS = [
    {},
    {'BMPOW_ONE_QUERY': '0'},
    {"BMPOW_ONE_EVENT": "0"},
    {'BMPOW_WAIT1': 'spin'},
]


def threads():
    tick = os.sysconf('SC_CLK_TCK')
    out = {}
    for tid in os.listdir('/proc/self/task'):
        try:
            with open('/proc/self/task/%s/stat' % tid) as f:
                s = f.read()
            with open('/proc/self/task/%s/comm' % tid) as f:
                name = f.read().strip()
        except OSError:
            continue
        fields = s[s.rindex(')') + 2:].split()
        out[tid] = (name, (int(fields[11]) + int(fields[12])) / tick)
    return out


def child(log2):
    sys.path.insert(0, ROOT)
    from pybitmessage_amd import _lib
    lib = _lib.get()
    ih = hashlib.sha512(b'one cpu').digest()
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    lib.bmpow_search(ih, 0, 1, 1 << 28, ctypes.byref(n), ctypes.byref(t))
    lib.bmpow_reset_stats()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    th0 = threads()
    w0 = time.perf_counter()
    rc = lib.bmpow_search(ih, 0, 1, 1 << log2, ctypes.byref(n), ctypes.byref(t))
    wall = time.perf_counter() - w0
    th1 = threads()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    st = _lib.BmpowStats()
    lib.bmpow_get_stats(ctypes.byref(st))
    per = sorted(((th1[k][0], round((th1[k][1] - th0.get(k, (None, 0.0))[1]) / wall, 4)) for k in th1),
                 key=lambda x: -x[1])
    print(json.dumps({'rc': rc, 'wall_s': round(wall, 3), 'ghs': round(st.trials / wall / 1e9, 4),
                      'process_cpu_per_s': round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / wall, 4),
                      'threads_cpu_per_s': [p for p in per if p[1] > 0.001],
                      'one_wait_spin_ms': round(st.one_wait_spin_ms, 1), 'one_wait_sleep_ms': round(st.one_wait_sleep_ms, 1)}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        child(int(sys.argv[2]))
        return
    log2 = int(sys.argv[1]) if len(sys.argv) > 1 else 33
    for cfg in CONFIGS:
        env = dict(os.environ)
        env.update(cfg)
        env.setdefault('BMPOW_DEVICES', '0')
        r = subprocess.run([sys.executable, os.path.abspath(__file__), 'child', str(log2)], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith('{')]
        d = json.loads(line[-1]) if line else {'error': r.stderr[-800:]}
        d['env'] = cfg
        print(json.dumps(d), flush=True)


if __name__ == '__main__':
    main()
