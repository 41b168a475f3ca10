"""Host resident memory (RSS, after gc and malloc_trim) at each step of the layouts the soak test
(tests/test_gpu_soak.py) walks through: where the library's host memory goes when shards are added,
when run() pieces get CU-masked streams, and whether it comes back when the layout shrinks.
One JSON line per step: {"step", "rss_mib", "delta_mib"}."""
import ctypes
import faulthandler
import gc
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

U64 = (1 << 64) - 1


def rss():
    gc.collect()
    ctypes.CDLL(None).malloc_trim(0)
    with open('/proc/self/statm') as f:
        return int(f.read().split()[1]) * os.sysconf('SC_PAGE_SIZE') / 2**20


def smaps_top(k=8):
    """The k largest mappings by resident size: {name: MiB} (anonymous mappings grouped as '[anon]')."""
    out, name = {}, None
    with open('/proc/self/smaps') as f:
        for line in f:
            parts = line.split()
            if parts and '-' in parts[0] and len(parts) >= 5 and not parts[0].endswith(':'):
                name = parts[5] if len(parts) > 5 else '[anon]'
            elif parts and parts[0] == 'Rss:':
                out[name] = out.get(name, 0) + int(parts[1]) / 1024
    return {n: round(v, 1) for n, v in sorted(out.items(), key=lambda x: -x[1])[:k]}


def threads_state():
    """Every thread of this process: comm, state, kernel wait channel and current syscall (a thread
    stuck on a mutex waits in futex; one waiting on the GPU, in an ioctl or a poll)."""
    out = []
    for tid in sorted(os.listdir('/proc/self/task'), key=int):
        d = '/proc/self/task/' + tid
        try:
            comm = open(d + '/comm').read().strip()
            state = open(d + '/stat').read().rsplit(')', 1)[1].split()[0]
            wchan = open(d + '/wchan').read().strip()
            sysc = open(d + '/syscall').read().split()[0]
        except OSError as e:
            comm, state, wchan, sysc = '?', '?', '?', repr(e)
        out.append({'tid': int(tid), 'comm': comm, 'state': state, 'wchan': wchan, 'syscall': sysc})
    return out


def watchdog(stuck_after=20.0):
    """Dump the threads' state to stderr whenever one step has run longer than stuck_after seconds."""
    import threading
    import time
    seen = {'t': time.time(), 'n': 0}

    here = os.path.dirname(os.path.abspath(__file__))
    dump = None
    if os.path.exists(os.path.join(here, 'libstackdump.so')):
        dump = ctypes.CDLL(os.path.join(here, 'libstackdump.so'))
        dump.stackdump_install()
    libc = ctypes.CDLL(None, use_errno=True)

    def loop():
        me = threading.get_native_id()
        signalled = set()
        while True:
            time.sleep(5)
            if time.time() - seen['t'] > stuck_after:
                ths = threads_state()
                print(json.dumps({'stuck_s': round(time.time() - seen['t'], 1), 'threads': ths}),
                      file=sys.stderr, flush=True)
                for t in ths:  # a running thread's native stack, once (SIGUSR2 -> stackdump.c)
                    if dump and t['state'] == 'R' and t['tid'] != me and t['tid'] not in signalled:
                        signalled.add(t['tid'])
                        print(json.dumps({'backtrace_of': t['tid']}), file=sys.stderr, flush=True)
                        libc.syscall(234, os.getpid(), t['tid'], 12)  # tgkill(pid, tid, SIGUSR2)
                        time.sleep(0.5)
    threading.Thread(target=loop, daemon=True).start()
    return seen


def main():
    faulthandler.dump_traceback_later(20, repeat=True)  # a stuck step names itself on stderr
    import time
    dog = watchdog()
    last = [rss()]

    def mark(step):
        r = rss()
        print(json.dumps({'step': step, 'rss_mib': round(r, 1), 'delta_mib': round(r - last[0], 1),
                          'top': smaps_top()}), flush=True)
        last[0] = r
        dog['t'] = time.time()

    mark('start')
    from pybitmessage_amd import _lib, proofofwork, worker
    lib = _lib.get()
    mark('library loaded, 1 shard')
    rng = random.Random(5)

    def runs(k=20):
        for _ in range(k):
            proofofwork.run(U64 // 20000, rng.randbytes(64))

    def layout(ids, split):
        print(json.dumps({'begin': 'set %d shards split=%s' % (len(ids), split)}), flush=True)
        dog['t'] = time.time()
        arr = (ctypes.c_int * len(ids))(*ids)
        assert lib.bmpow_set_devices(arr, len(ids)) == len(ids)
        lib.bmpow_set_run_split(1 if split else 0)

    runs()
    mark('20 run() calls')
    svc = worker.PowService().start()
    [f.result(60) for f in svc.submit_many([(U64 // 20000, rng.randbytes(64)) for _ in range(64)])]
    svc.stop(30)
    mark('PowService, 64 objects')
    for rep in range(2):
        for ids, split in (([0, 0], False), ([0, 0, 0], False), ([0, 0, 0], True), ([0] * 8, True),
                           ([0] * 8, False), ([0], False)):
            layout(ids, split)
            mark('pass %d: set %d shards split=%s' % (rep, len(ids), split))
            runs()
            mark('pass %d: 20 run() calls on %d shards split=%s' % (rep, len(ids), split))


if __name__ == '__main__':
    main()
