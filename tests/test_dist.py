"""Multi-rank bench plumbing on CPU (gloo, world_size 2): object sharding by rank and the
whole-job aggregation (max-over-ranks time, sum-over-ranks work).  The data path has no
collective; gloo carries only timing."""
import json
import os
import socket
import types

import pytest

torch = pytest.importorskip('torch')
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir):
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    d = bench.Dist()
    objs, _ = bench.make_objects('c2', d.rank, 8)
    stats = types.SimpleNamespace(trials=1000 * (rank + 1), kernel_ms=10.0 * (rank + 1), launches=2)
    r = {'desc': 'test', 'objects': 8, 'useful': 900.0 * (rank + 1), 'elapsed': 1.0 + rank, 'stats': stats,
         'pci_bus_id': '0000:%02x:00.0' % (0x10 * (rank + 1))}
    args = types.SimpleNamespace(steps=1, warmup=0)
    d.barrier()
    line = bench.summarize(args, d, r, 'test-lib')
    with open(os.path.join(outdir, 'rank%d.json' % rank), 'w') as f:
        json.dump({'line': line, 'first_ih': objs[0][1].hex()}, f)
    d.close()


def _claim_worker(rank, world, port, outdir):
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    import time
    d = bench.Dist()
    c = bench.Claimer(d, 1000, 7)
    got = []
    for tag in ('a', 'b'):
        c.start(tag)
        mine = []
        while True:
            r = c.claim()
            if r is None:
                break
            mine.append(r)
            time.sleep(0.001 * (rank + 1))  # ranks of different speed
        got.append(mine)
    d.barrier()
    with open(os.path.join(outdir, 'claims%d.json' % rank), 'w') as f:
        json.dump(got, f)
    d.close()


def test_claims_partition_the_global_batch(tmp_path):
    """Work claiming over the TCP store: every object of the global batch is claimed by
    exactly one rank, per step (tag), and the faster rank claims more."""
    port = _free_port()
    mp.spawn(_claim_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    c0 = json.load(open(tmp_path / 'claims0.json'))
    c1 = json.load(open(tmp_path / 'claims1.json'))
    for step in range(2):
        idx = sorted(i for lo, hi in c0[step] + c1[step] for i in range(lo, hi))
        assert idx == list(range(1000))
    assert sum(hi - lo for lo, hi in c0[0]) > sum(hi - lo for lo, hi in c1[0])


def test_single_rank_claims_everything():
    import types
    c = bench.Claimer(types.SimpleNamespace(world=1), 50, 50)
    c.start('x')
    assert c.claim() == (0, 50) and c.claim() is None


def test_two_rank_aggregation(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / 'rank0.json'))
    r1 = json.load(open(tmp_path / 'rank1.json'))
    line = r0['line']
    assert line['n_gpus'] == 2 and line['scaling'] == 'weak'
    # value = (900 + 1800) useful trials / max(1.0, 2.0) s, in GH/s
    assert line['value'] == round(2700 / 2.0 / 1e9, 4)
    assert line['objects_per_s'] == round(16 / 2.0, 3)
    assert line['performed_ghs'] == round(3000 / 2.0 / 1e9, 4)
    assert r1['line']['value'] == line['value']  # every rank sees the same reduction
    # per_rank: which physical GPU each rank drove and its work, in rank order, on every rank
    pr = line['per_rank']
    assert [p['rank'] for p in pr] == [0, 1] and r1['line']['per_rank'] == pr
    assert [p['device_pci_bus_id'] for p in pr] == ['0000:10:00.0', '0000:20:00.0']
    assert [p['trials'] for p in pr] == [1000, 2000] and [p['kernel_ms'] for p in pr] == [10.0, 20.0]
    assert [p['elapsed_s'] for p in pr] == [1.0, 2.0]
    assert set(pr[0]) == {'rank', 'local_rank', 'device_pci_bus_id', 'trials', 'kernel_ms', 'elapsed_s'}
    # the committed PMC traffic (per 2^28-trial launch) scaled to this rank's trials per launch
    pmc = json.load(open(os.path.join(bench.ROOT, 'profiles', 'pmc_latest.json')))
    want = pmc['derived']['hbm_bytes_per_launch_upper'] * (1000 / 2) / pmc['raw']['trials_per_launch']
    assert line['roofline']['traffic'] == round(want) and 'traffic_basis' in line['roofline']
    # each rank works on its own batch (seed + rank): no object is solved twice
    assert r0['first_ih'] != r1['first_ih']


class _FakeLib(object):
    """A CPU stand-in for libbmpow_hip.so's calls made by bench.nonce_sharded: two devices, a no-hit sweep
    counted exactly, batches solved by the oracle's _doSafePoW restatement, per-shard stats."""

    def __init__(self, visible=2):
        import ctypes
        self.ctypes = ctypes
        self.visible, self.ids, self.trials, self.batch = visible, [0], 0, None

    def bmpow_device_count(self):
        return self.visible

    def bmpow_get_devices(self, arr, cap):
        for i, d in enumerate(self.ids[:cap]):
            arr[i] = d
        return len(self.ids)

    def bmpow_set_devices(self, arr, n):
        self.ids = [arr[i] for i in range(n)]
        return n

    def bmpow_reset_stats(self):
        self.trials = 0

    def bmpow_search(self, ih, target, start, count, pn, pt):
        self.trials = count  # target 0: no hit, every nonce once
        return 0

    def bmpow_get_stats(self, ref):
        ref._obj.trials = self.trials

    def bmpow_get_shard_stats(self, tr, ms, cap):
        for i in range(len(self.ids)):
            tr[i], ms[i] = self.trials // len(self.ids), 1.5
        return len(self.ids)

    def bmpow_device_pci_bus_id(self, dev, buf, n):
        buf.value = b'0000:%02x:00.0' % (0x10 * (dev + 1))
        return 0

    def bmpow_batch_create(self, m, ihs, tg, start):
        self.batch = [(int(tg[i]), ihs[64 * i:64 * i + 64]) for i in range(m)]
        return 1

    def bmpow_batch_reset(self, h, start):
        return len(self.batch)

    def bmpow_batch_step(self, h, budget):
        from oracle import oracle
        self.res = [oracle.safe_pow(t, ih) for t, ih in self.batch]
        self.trials += sum(n + 256 for _, n in self.res)
        return 0

    def bmpow_batch_results(self, h, nonce, trial, done, nxt):
        for i, (tv, n) in enumerate(self.res):
            nonce[i], trial[i], done[i] = n, tv, 1
        return 0

    def bmpow_batch_destroy(self, h):
        self.batch = None

    def bmpow_last_error(self):
        return b''


def _ns_worker(rank, world, port, outdir):
    os.environ.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port)})
    import hashlib
    d = bench.Dist()
    lib = _FakeLib()
    objs = [((1 << 64) // 40, hashlib.sha512(b'ns %d' % i).digest()) for i in range(6)]
    line = {}
    # main()'s pattern: a barrier, rank 0 alone runs the leg, a barrier
    d.barrier()
    if d.rank == 0:
        line['nonce_sharded'] = bench.nonce_sharded(lib, d.world, c3_log2=20, c4_objs=objs)
        line['restored'] = lib.ids
    d.barrier()
    with open(os.path.join(outdir, 'ns%d.json' % rank), 'w') as f:
        json.dump(line, f)
    d.close()


def test_nonce_sharded_field(tmp_path):
    """SCALE runs (N > 1) carry `nonce_sharded`: rank 0, after the timed region and while the other
    ranks wait at a barrier, runs C3 and C4 nonce-sharded over N devices in one process (the north
    star's split, which object-sharded ranks never exercise).  gloo world_size 2 with a CPU stand-in for
    the library: the field's shape, one entry per device with its PCI bus id, the rank's own device
    selection restored; rank 1 carries no field."""
    port = _free_port()
    mp.spawn(_ns_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / 'ns0.json'))
    assert json.load(open(tmp_path / 'ns1.json')) == {}
    ns = r0['nonce_sharded']
    assert r0['restored'] == [0]
    assert ns['devices'] == [0, 1] and ns['device_groups'] == 2
    assert set(ns) >= {'c3_ghs', 'c4_ghs', 'c4_wasted_frac', 'c3', 'c4', 'what'}
    assert ns['c3']['trials_exact'] and ns['c3']['not_found'] and ns['c3']['nonces'] == 1 << 20
    assert [p['pci_bus_id'] for p in ns['c4']['per_device']] == ['0000:10:00.0', '0000:20:00.0']
    assert ns['c4']['objects'] == 6 and 0 < ns['c4']['wasted_frac'] < 1
    # one visible device: the leg says it is a rehearsal, one bus id
    lib = _FakeLib(visible=1)
    one = bench.nonce_sharded(lib, 2, c3_log2=16, c4_objs=[((1 << 64) // 10, b'\x01' * 64)])
    assert one['devices'] == [0, 0] and one['device_groups'] == 1 and 'rehearsal' in one['what']
    assert len(one['c3']['per_device']) == 1


def test_c2_workload_is_deterministic():
    a, da = bench.make_objects('c2', 0, 16)
    b, _ = bench.make_objects('c2', 0, 16)
    assert a == b and 'C2' in da
    full, _ = bench.make_objects('c2', 0)
    assert len(full) == 1024
    assert full[:16] == a
    # targets follow the singleWorker formula with TTL 4 d at default difficulty
    from pybitmessage_amd.targets import object_target
    import random
    rng = random.Random(bench.SEED)
    L = rng.randrange(512, 16385)
    assert a[0][0] == int(object_target(L, 345600))


def test_single_rank_line_carries_the_round4_fields(monkeypatch):
    """One rank (no process group): the C1 line names the kernel it timed, carries the per-call
    distribution, the cut lanes and the host CPU figures; `single_object_path` follows BMPOW_ONE and
    the shard count."""
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.delenv('RANK', raising=False)
    d = bench.Dist()
    assert d.world == 1
    stats = types.SimpleNamespace(trials=11_000_000, kernel_ms=1.65, launches=1, cut_trials=40_000)
    per_call = {'ms': {'min': 1.6, 'median': 1.67, 'p90': 1.7, 'max': 1.8}}
    host = {'process_cpu_per_s': 0.9, 'stepper_cpu_per_s': [], 'stepper_policy': [], 'wait': 'sleep', 'what': ''}
    r = {'desc': 'C1', 'objects': 1, 'useful': 10_909_138.0, 'elapsed': 0.0017, 'stats': stats,
         'kernel': 'bm_search1_kernel', 'call_ms': 1.7, 'path': 'single-object', 'per_call': per_call,
         'host_cpu': host}
    args = types.SimpleNamespace(steps=1, warmup=0, devices=0, shards_per_device=1, throttle=None)
    line = bench.summarize(args, d, r, 'test-lib')
    assert line['roofline']['kernel'] == 'bm_search1_kernel'
    assert line['per_call'] == per_call and line['call_ms'] == 1.7 and line['path'] == 'single-object'
    assert line['cut_trials'] == 40_000
    assert line['wasted_frac_incl_cut'] == round(1.0 - 10_909_138.0 / (11_000_000 + 20_000), 5)
    assert line['host_cpu_per_s'] == 0.9
    assert 'frac_vs_mix_ceiling' not in line['roofline'] and 'frac_vs_baseline_md_peak' not in line['roofline']
    monkeypatch.setenv('BMPOW_ONE', '1')
    assert bench.single_object_path(args)
    # round 5: run() takes the single-object path on any number of shards (pieces per device)
    assert bench.single_object_path(types.SimpleNamespace(devices=1, shards_per_device=8))
    monkeypatch.setenv('BMPOW_ONE', '0')
    assert not bench.single_object_path(args)


def test_rank_device_selection():
    """Each rank drives its LOCAL_RANK's device; with one visible device per rank (a launcher that sets
    HIP_VISIBLE_DEVICES per rank) every rank drives its own device 0; --share-device puts all on 0; a
    rank without a GPU stops with a message."""
    d = types.SimpleNamespace(rank=3, local_rank=3)
    assert bench.rank_device(d, visible=8) == 3
    assert bench.rank_device(d, visible=1) == 0
    assert bench.rank_device(d, share=True, visible=8) == 0
    assert bench.rank_device(types.SimpleNamespace(rank=0, local_rank=0), visible=1) == 0
    with pytest.raises(SystemExit):
        bench.rank_device(d, visible=2)


def test_nonce_sharded_child_wrapper():
    """rank 0 runs the nonce-sharded leg in a child process under a time limit: its JSON comes back; a
    child that fails, prints nothing or overruns is an `error` entry, never a lost scaling line."""
    import sys
    ok = bench.run_nonce_sharded_child(2, argv=[sys.executable, '-c', 'print("noise"); print(\'{"c3_ghs": 1.5}\')'])
    assert ok == {'c3_ghs': 1.5}
    bad = bench.run_nonce_sharded_child(2, argv=[sys.executable, '-c', 'import sys; sys.exit(3)'])
    assert bad['error'] == 'exit status 3'
    slow = bench.run_nonce_sharded_child(2, timeout=1, argv=[sys.executable, '-c', 'import time; time.sleep(5)'])
    assert 'timed out' in slow['error']
