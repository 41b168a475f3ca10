"""C1 on one shard at several column counts (BMPOW_COLUMNS, set per child process): trials hashed
against the golden nonce 10,909,138, and call time."""
import ctypes
import json
import os
import subprocess
import sys
import time

if len(sys.argv) > 1 and sys.argv[1] == 'child':
    sys.path.insert(0, '.')
    from pybitmessage_amd import _lib, proofofwork
    lib = _lib.get()
    k = [k for k in json.load(open('tests/golden/first_nonce_kats.json'))['kats'] if k['nonce'] == 10909138][0]
    ih = bytes.fromhex(k['ih'])
    proofofwork.run(k['target'], ih)
    out = []
    for _ in range(6):
        lib.bmpow_reset_stats()
        t0 = time.perf_counter()
        r = proofofwork.run(k['target'], ih)
        dt = time.perf_counter() - t0
        st = _lib.BmpowStats()
        lib.bmpow_get_stats(ctypes.byref(st))
        assert r == [k['trial'], k['nonce']]
        out.append({'trials': st.trials, 'ms': round(dt * 1e3, 3), 'kernel_ms': round(st.kernel_ms, 3)})
    print(json.dumps({'columns': os.environ.get('BMPOW_COLUMNS', 'auto'), 'runs': out}))
else:
    for cols in sys.argv[2:] if len(sys.argv) > 2 else ['0', '1280', '1024', '768', '512', '256']:
        env = dict(os.environ, BMPOW_COLUMNS=cols)
        subprocess.run([sys.executable, __file__, 'child'], env=env, check=True, timeout=120)
