"""Host-side logic that needs no GPU: ABI export table, Python mirror of the reference
interface, target formulas, verifier, interrupt loop (against a scripted test double of the
C ABI -- the double lives here in tests/, the product has no fallback)."""
import ctypes
import hashlib
import os
import random
import re
import threading

import pytest

from tests.conftest import ROOT

from pybitmessage_amd import _lib, proofofwork, state, targets

HEADER = os.path.join(ROOT, 'include', 'bmpow.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'BMPOW_API\s+[\w\s\*]+?\b(\w+)\s*\(', text)))


@pytest.fixture(scope='module')
def rawlib():
    path = _lib.lib_path()
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(['make', '-C', os.path.join(ROOT, 'pybitmessage_amd', 'csrc')])
    return ctypes.CDLL(path)


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ['bmpow_init', 'bmpow_search', 'bmpow_search_batch', 'bmpow_trials', 'bmpow_abort',
              'bmpow_batch_create', 'bmpow_batch_step', 'bmpow_batch_results', 'bmpow_batch_destroy',
              'bmpow_set_devices', 'bmpow_last_error', 'BitmessagePOW', 'bmpow_pow_values',
              'bmpow_verify_batch', 'bmpow_pow_sufficient', 'bmpow_vbatch_create', 'bmpow_vbatch_run',
              'bmpow_vbatch_destroy', 'bmpow_pubkeys', 'bmpow_address_search', 'bmpow_address_search_random', 'bmpow_batch_set_pending', 'bmpow_verify_batch_ptrs',
              'bmpow_addr_set_comb', 'bmpow_addr_last_comb', 'bmpow_fe_probe', 'bmpow_min_trial',
              'bmpow_min_trial_batch', 'bmpow_batch_add', 'bmpow_batch_take_done', 'bmpow_service_create',
              'bmpow_service_submit', 'bmpow_service_poll', 'bmpow_service_cancel', 'bmpow_service_outstanding',
              'bmpow_service_stop', 'bmpow_service_destroy', 'bmpow_set_device_count', 'bmpow_trials_len',
              'bmpow_search_len', 'bmpow_min_trial_var', 'bmpow_batch_add_var', 'bmpow_service_submit_var',
              'bmpow_get_shard_rates', 'bmpow_get_shard_stats', 'bmpow_get_thread_info', 'bmpow_set_shard_throttle',
              'bmpow_set_run_split', 'bmpow_get_run_pieces', 'bmpow_device_pci_bus_id', 'bmpow_set_engine_split',
              'bmpow_atexit']:
        assert s in syms
    assert len(syms) == 62


def test_exit_hook_registered_and_final(monkeypatch, tmp_path):
    """The library is released at process exit before the HIP runtime's own exit handlers (round 5's
    traced runs with CU-masked streams alive segfaulted in them): _lib.get() registers bmpow_atexit with
    Python's atexit once, and bmpow_atexit is final -- a fresh copy of the library refuses to initialise
    after it (E_STATE), so no stream can be created after the teardown.  No GPU needed."""
    import atexit
    import shutil
    calls = []

    class Fake(object):
        def bmpow_init(self):
            return 1

        def bmpow_atexit(self):
            calls.append('atexit')
    fake = Fake()
    registered = []
    monkeypatch.setattr(_lib, 'load', lambda path=None: fake)
    monkeypatch.setattr(_lib, '_lib', None)
    monkeypatch.setattr(_lib, '_exit_hooked', False)
    monkeypatch.setattr(atexit, 'register', lambda fn, *a: registered.append((fn, a)))
    assert _lib.get() is fake
    assert registered == [(_lib._at_exit, (fake,))]
    monkeypatch.setattr(_lib, '_lib', None)
    _lib.get()
    assert len(registered) == 1  # once per process
    _lib._at_exit(fake)
    assert calls == ['atexit']
    # the real export: final, and safe with nothing initialised
    path = _lib.lib_path()
    if not os.path.exists(path):
        pytest.skip('library not built')
    copy = tmp_path / 'libbmpow_copy.so'
    shutil.copy(path, copy)
    lib = ctypes.CDLL(str(copy))
    lib.bmpow_atexit()
    lib.bmpow_atexit()  # idempotent
    assert lib.bmpow_init() == _lib.E_STATE
    lib.bmpow_last_error.restype = ctypes.c_char_p
    assert b'exiting' in lib.bmpow_last_error()


def test_library_exports_every_declared_symbol(rawlib):
    for s in declared_symbols():
        assert hasattr(rawlib, s), s


def test_stats_struct_matches_the_header(tmp_path):
    """The ctypes mirror of bmpow_stats has the C struct's size and field offsets (a field added
    on one side only would make bmpow_get_stats write past the Python buffer)."""
    import subprocess
    fields = [f for f, _ in _lib.BmpowStats._fields_]
    src = tmp_path / 'sz.c'
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "bmpow.h"\nint main(void) {\n'
                   '  printf("%zu", sizeof(bmpow_stats));\n' +
                   ''.join('  printf(" %%zu", offsetof(bmpow_stats, %s));\n' % f for f in fields) +
                   '  return 0;\n}\n')
    exe = tmp_path / 'sz'
    subprocess.check_call(['gcc', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got[0] == ctypes.sizeof(_lib.BmpowStats)
    assert got[1:] == [getattr(_lib.BmpowStats, f).offset for f in fields]


def test_python_binding_covers_header():
    bound = sorted(n for n, _, _ in _lib.SIGNATURES)
    assert bound == declared_symbols()


def test_load_binds_all_signatures(rawlib):
    lib = _lib.load()
    assert lib.bmpow_version().startswith(b'bmpow 1 gfx950')
    assert lib.bmpow_get_step_trials() > 0


def test_step_trials_setting():
    """The per-step budget (host state only): at least one chunk, and 0 restores the default."""
    lib = _lib.load()
    default = lib.bmpow_get_step_trials()
    assert default == 1 << 29
    lib.bmpow_set_step_trials(1 << 20)
    assert lib.bmpow_get_step_trials() == 1 << 20
    lib.bmpow_set_step_trials(5)
    assert lib.bmpow_get_step_trials() == 8192
    lib.bmpow_set_step_trials(0)
    assert lib.bmpow_get_step_trials() == default


@pytest.mark.skipif(os.path.exists('/dev/kfd'), reason='a GPU is present')
def test_shard_rates_without_devices():
    """bmpow_get_shard_rates reads host state only: no shard selected yet, and a null buffer with a
    positive capacity is an argument error rather than a crash."""
    lib = _lib.load()
    rates = (ctypes.c_double * 4)(-1, -1, -1, -1)
    assert lib.bmpow_get_shard_rates(rates, 4) == 0
    assert list(rates) == [-1, -1, -1, -1]
    assert lib.bmpow_get_shard_rates(None, 4) == _lib.E_ARG
    assert lib.bmpow_get_shard_rates(None, 0) == 0
    # the per-shard stats and the stepper threads' info are host state too (no stepper yet)
    assert lib.bmpow_get_shard_stats(None, None, 4) == 0
    assert lib.bmpow_get_thread_info(None, None, 4) == 0
    assert lib.bmpow_set_shard_throttle(0, 1.0) == _lib.E_STATE


@pytest.mark.skipif(os.path.exists('/dev/kfd'), reason='a GPU is present')
def test_no_device_fails_loudly():
    lib = _lib.load()
    assert lib.bmpow_device_count() == 0
    assert lib.bmpow_init() == _lib.E_NODEV
    assert b'gfx950' in lib.bmpow_last_error()
    n, t = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.bmpow_search(bytes(64), 1, 1, 10, ctypes.byref(n), ctypes.byref(t)) == _lib.E_NODEV
    with pytest.raises(_lib.BmpowUnavailable):
        proofofwork.run(2 ** 60, bytes(64))
    assert proofofwork.getPowType() == 'none'
    assert proofofwork.init() == 0


def test_ih_is_hashed_as_given():
    """_doSafePoW hashes pack('>Q', nonce) + initialHash at its own length (src/proofofwork.py:
    104-107): no zero-padding to the _doCPoW buffer's 64 bytes (round 2 padded)."""
    assert proofofwork._ih_bytes(b'') == b''
    assert proofofwork._ih_bytes(b'ab') == b'ab'
    assert proofofwork._ih_bytes('ab') == b'ab'
    assert proofofwork._ih_bytes(bytes(65)) == bytes(65)
    assert proofofwork._ih_bytes(bytearray(200)) == bytes(200)
    with pytest.raises(ValueError):
        proofofwork._ih_bytes(bytes(_lib.MAX_IH_LEN + 1))


def test_target_clamp():
    assert proofofwork._clamp_target(2 ** 64) == (2 ** 64 - 1, True)
    assert proofofwork._clamp_target(2.0 ** 70) == (2 ** 64 - 1, True)
    assert proofofwork._clamp_target(12345.9) == (12345, True)
    assert proofofwork._clamp_target(-1) == (0, False)


def test_estimate_matches_reference():
    assert proofofwork.estimate(5) == 1
    assert proofofwork.estimate(100) == 10
    assert proofofwork.estimate(100, format=True) is None


def test_targets_match_golden(golden):
    for t in golden('config_targets.json')['targets']:
        if t['kind'] == 'singleWorker':
            f = targets.object_target(t['L'], t['ttl'], t['ntpb'], t['extra'])
        else:
            f = targets.api_target(t['L'], t['ntpb'], t['extra'])
        assert f.hex() == t['target_float']
        assert targets.int_target(f) == t['target']


def test_verifier_matches_reference(golden):
    for k in golden('verifier_kats.json')['kats']:
        obj = bytes.fromhex(k['object'])
        assert targets.isProofOfWorkSufficient(obj, k['ntpb'], k['extra'], k['recvTime']) == k['sufficient']
        nxt = targets.attach_nonce(int.from_bytes(obj[:8], 'big') + 1, obj[8:])
        assert targets.isProofOfWorkSufficient(nxt, k['ntpb'], k['extra'], k['recvTime']) == \
            k['object_next_nonce_sufficient']
        assert targets.isProofOfWorkSufficient(obj, k['ntpb'], k['extra'], k['recvTime'] - 10 ** 6) == \
            k['recvTime_minus_1e6_sufficient']


# ---------------- interrupt / loop logic against a scripted C-ABI double ----------------
class ScriptedLib(object):
    """Test double of the C ABI: bmpow_search answers from the C oracle over the bounded
    window it is asked for (so loop/resume logic is exercised exactly)."""

    def __init__(self, coracle, stop_after=None, corrupt=False):
        self.co = coracle
        self.calls = []
        self.stop_after = stop_after
        self.corrupt = corrupt  # answer with a wrong trial value (a faulty device)

    def bmpow_search_len(self, ih, ih_len, target, start, max_trials, pn, pt):
        assert len(ih) == ih_len
        self.calls.append((start, max_trials))
        if self.stop_after is not None and len(self.calls) >= self.stop_after:
            state.shutdown = 1
        res = self.co.search_len(ih, target, start, max_trials)
        if res is None:
            return _lib.NOT_FOUND
        pt._obj.value, pn._obj.value = res
        if self.corrupt:
            pt._obj.value ^= 1
        return _lib.FOUND

    def bmpow_get_devices(self, ids, cap):
        ids[0] = 0
        return 1

    def bmpow_last_error(self):
        return b''


@pytest.fixture
def scripted(monkeypatch, coracle):
    def make(**kw):
        lib = ScriptedLib(coracle, **kw)
        monkeypatch.setattr(_lib, 'get', lambda: lib)
        return lib
    yield make
    state.shutdown = 0


def test_run_resumes_across_bounded_calls(scripted, monkeypatch):
    lib = scripted()
    monkeypatch.setattr(proofofwork, 'CALL_TRIALS', 100)
    ih = hashlib.sha512(b'hello').digest()
    assert proofofwork.run(2 ** 64 // 1000, ih) == [2417842470843601, 1315]
    assert lib.calls[0] == (1, 100) and lib.calls[-1] == (1301, 100) and len(lib.calls) == 14


def test_run_raises_interrupted_between_calls(scripted, monkeypatch):
    lib = scripted(stop_after=3)
    monkeypatch.setattr(proofofwork, 'CALL_TRIALS', 10)
    with pytest.raises(StopIteration, match='Interrupted'):
        proofofwork.run(0, bytes(64))
    assert len(lib.calls) == 3


def test_run_refuses_during_shutdown(scripted):
    scripted()
    state.shutdown = 1
    with pytest.raises(RuntimeError):
        proofofwork.run(10, bytes(64))


def test_negative_target_spins_until_shutdown(scripted):
    lib = scripted()
    timer = threading.Timer(0.2, lambda: setattr(state, 'shutdown', 1))
    timer.start()
    with pytest.raises(StopIteration):
        proofofwork.run(-5, bytes(64))
    assert lib.calls == []


def test_run_any_length_matches_reference(scripted, golden):
    """run() over initialHashes that are not 64 bytes answers the reference's _doSafePoW (the
    fixture, tests/golden/make_len_golden.py) through the bounded-call loop; the C oracle stands
    in for the device."""
    scripted()
    for k in golden('len_kats.json')['first']:
        ih = bytes.fromhex(k['ih'])
        assert len(ih) == k['len']
        assert proofofwork.run(k['target'], ih) == [k['trial'], k['nonce']], k['len']


def test_wrong_gpu_answer_disables_the_backend(scripted, monkeypatch, caplog):
    """A wrong answer disables the GPU backend as _doGPUPoW disables OpenCL
    (src/proofofwork.py:176-190): the reference's error line, enabledGpus cleared, the UI told,
    getPowType() 'none', later calls refused until resetPoW()."""
    from pybitmessage_amd import hippow
    lib = scripted(corrupt=True)
    hippow.initCL()
    assert hippow.openclEnabled()
    seen = []
    monkeypatch.setattr(proofofwork, 'ui_notify', seen.append)
    ih = hashlib.sha512(b'hello').digest()
    try:
        with caplog.at_level('ERROR', logger='default'):
            with pytest.raises(_lib.BmpowError, match='did not calculate correctly'):
                proofofwork.run(2 ** 64 // 1000, ih)
        assert 'did not calculate correctly, disabling OpenCL' in caplog.text
        assert seen and 'disabling' in seen[0]
        assert hippow.enabledGpus == [] and not hippow.openclEnabled()
        assert proofofwork.getPowType() == 'none'
        ncalls = len(lib.calls)
        with pytest.raises(_lib.BmpowUnavailable, match='disabled'):
            proofofwork.run(2 ** 64 // 1000, ih)
        assert len(lib.calls) == ncalls  # refused before touching the device
        with pytest.raises(_lib.BmpowUnavailable):
            next(proofofwork.iter_batch([(2 ** 64 // 1000, ih)]))
        # resetPoW re-enables (reference resetPoW -> openclpow.initCL)
        lib.corrupt = False
        monkeypatch.setattr(_lib, 'reset', lambda: None)
        proofofwork.resetPoW()
        assert hippow.openclEnabled() and proofofwork.getPowType() == 'HIP'
        assert proofofwork.run(2 ** 64 // 1000, ih) == [2417842470843601, 1315]
    finally:
        proofofwork._disabled = None


def test_reset_pow_keeps_the_configured_vendor(scripted, monkeypatch):
    """resetPoW after the user picked another vendor in the settings (bitmessageqt/settings.py:452-458
    puts it in keys.dat, then resetPoW -> initCL re-reads it, src/proofofwork.py:328-330,
    src/openclpow.py:45): the HIP devices stay present but disabled; picking HIP again enables them."""
    from pybitmessage_amd import hippow
    scripted()
    monkeypatch.setattr(_lib, 'reset', lambda: None)
    hippow.initCL('NVIDIA Corporation')
    assert hippow.openclAvailable() and not hippow.openclEnabled()
    proofofwork.resetPoW()
    assert hippow.openclAvailable() and not hippow.openclEnabled()
    hippow.initCL('HIP')
    proofofwork.resetPoW()
    assert hippow.openclEnabled()


def test_do_opencl_pow_any_length_and_negative_target(scripted, golden):
    """hippow.do_opencl_pow: the _doSafePoW nonce for a hex initialHash of any length, and a
    negative target raises at once (the reference's numpy packing never blocks on it)."""
    from pybitmessage_amd import hippow
    scripted()
    hippow.initCL()
    for k in golden('len_kats.json')['first'][:12]:
        assert hippow.do_opencl_pow(k['ih'], k['target']) == k['nonce']
    with pytest.raises(ValueError):
        hippow.do_opencl_pow('00' * 64, -1)


def test_verify_rejects_wrong_gpu_answer():
    ih = hashlib.sha512(b'hello').digest()
    try:
        proofofwork._verify(2 ** 64 // 1000, ih, 2417842470843601, 1315)
        with pytest.raises(_lib.BmpowError):
            proofofwork._verify(2 ** 64 // 1000, ih, 2417842470843602, 1315)
        with pytest.raises(_lib.BmpowError):
            proofofwork._verify(10, ih, 2417842470843601, 1315)
    finally:
        proofofwork._disabled = None


def test_sender_targets_match_the_reference_expressions(golden):
    """targets.object_target against the reference's own _doPOWDefaults and sendMsg target
    statements (class_singleWorker.py:222-230, 1256-1264), evaluated by
    tests/golden/make_target_golden.py: bit-exact floats, at network-default and test-mode
    difficulty, int and float (requestPubKey) TTLs, recipient difficulties."""
    d = golden('sender_targets_ref.json')
    assert len(d['cases']) > 700
    for c in d['cases']:
        t = targets.object_target(c['L'], c['ttl'], c['ntpb'], c['extra'])
        assert t == float.fromhex(c['target_float']), c
        assert int(t) == c['target']


def test_library_identity_is_reproducible():
    """The PMC counters' provenance (bench.py pmc_counters): the library's version names its sources
    (BM_SRC_ID, an md5 of every source), not a build time, and the device-code md5
    (tools/lib_code_md5.py, the .hip_fatbin section) is what `counters.stale` compares."""
    import bench
    from tools.lib_code_md5 import code_md5
    path = _lib.lib_path()
    if not os.path.exists(path):
        pytest.skip('library not built')
    lib = ctypes.CDLL(path)
    lib.bmpow_version.restype = ctypes.c_char_p
    v = lib.bmpow_version().decode()
    assert re.search(r' src [0-9a-f]{12}', v) and 'built' not in v, v
    md5 = code_md5(path)
    assert md5 and re.fullmatch(r'[0-9a-f]{32}', md5) and code_md5(path) == md5
    c = bench.pmc_counters()
    assert c['benched_code_md5'] == md5 and isinstance(c['stale'], bool)
    assert c['stale'] == (c['build'].get('code_md5', c['build'].get('lib_md5')) !=
                          (md5 if c['build'].get('code_md5') else c['benched_lib_md5']))
