"""The host-only scheduler unit (pybitmessage_amd/csrc/bmpow_sched.cpp -- window planning and
slicing over shards, the per-object min-reduction, resident sessions with slot reuse, min-trial
reduction, verification layout and multi-threaded padding) built with g++ and run against a CPU
stand-in for the kernels (tests/native/sched_sim.cpp, trial function from the C oracle) under
ThreadSanitizer and under AddressSanitizer + UBSan, with the library's concurrency: a host thread
per shard, producer threads feeding a locked session, parallel padding (SURVEY.md section 5:
"Run TSAN on the host library in this container").  No GPU."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

SRC = [os.path.join(ROOT, 'tests', 'native', 'sched_sim.cpp'),
       os.path.join(ROOT, 'pybitmessage_amd', 'csrc', 'bmpow_sched.cpp')]
ORACLE_C = os.path.join(ROOT, 'oracle', 'bmpow_oracle.c')
OUT = os.path.join(ROOT, 'build', 'native')

FLAVOURS = {
    'tsan': ['-fsanitize=thread'],
    'asan_ubsan': ['-fsanitize=address,undefined', '-fno-sanitize-recover=undefined', '-fno-omit-frame-pointer'],
}


def build(flavour):
    os.makedirs(OUT, exist_ok=True)
    flags = FLAVOURS[flavour]
    obj = os.path.join(OUT, 'oracle_%s.o' % flavour)
    exe = os.path.join(OUT, 'sched_sim_%s' % flavour)
    # the oracle's hashing (pure computation on thread-local data) is built without instrumentation
    subprocess.check_call(['gcc', '-O3', '-c', ORACLE_C, '-o', obj])
    subprocess.check_call(['g++', '-std=c++17', '-O1', '-g', '-Wall', '-pthread'] + flags + SRC + [obj, '-o', exe, '-lcrypto'])
    return exe


@pytest.mark.parametrize('flavour', sorted(FLAVOURS))
def test_scheduler_unit_under_sanitizer(flavour):
    exe = build(flavour)
    env = dict(os.environ)
    env['TSAN_OPTIONS'] = 'halt_on_error=1 exitcode=66 second_deadlock_stack=1'
    env['ASAN_OPTIONS'] = 'halt_on_error=1 detect_leaks=1'
    env['UBSAN_OPTIONS'] = 'halt_on_error=1 print_stacktrace=1'
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert 'all scenarios passed' in r.stderr
    assert 'WARNING: ThreadSanitizer' not in r.stderr and 'runtime error' not in r.stderr
