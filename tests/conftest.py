import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and libbmpow_hip.so')
    config.addinivalue_line('markers', 'slow: long-running (minutes)')


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope='session')
def golden():
    return load_golden


@pytest.fixture(scope='session')
def coracle():
    """The C restatement (oracle/liboracle.so), built on demand with make."""
    from oracle import oracle
    if not oracle.have_c_oracle():
        import subprocess
        subprocess.check_call(['make', '-C', os.path.join(ROOT, 'oracle'), 'liboracle.so'])
    return oracle.COracle()


@pytest.fixture(scope='session')
def gpulib():
    """libbmpow_hip.so initialised on the GPU (gpu tests only)."""
    from pybitmessage_amd import _lib
    return _lib.get()


@pytest.fixture
def shards(gpulib):
    """Run a test body under several shard layouts, restoring one shard per device after."""
    import ctypes

    def use(ids):
        arr = (ctypes.c_int * len(ids))(*ids)
        assert gpulib.bmpow_set_devices(arr, len(ids)) == len(ids)
    yield use
    gpulib.bmpow_set_devices(None, 0)
    gpulib.bmpow_set_step_trials(0)  # the library's default


@pytest.fixture
def engine_split(gpulib):
    """bmpow_set_engine_split for the test body (every shard its own device group: the multi-device
    split rehearsed on one GPU), restored after."""
    prev = gpulib.bmpow_set_engine_split(-1)
    yield lambda on: gpulib.bmpow_set_engine_split(1 if on else 0)
    gpulib.bmpow_set_engine_split(prev)


@pytest.fixture(autouse=True)
def _reenable_backend():
    """A test that feeds a wrong GPU answer disables the backend process-wide (proofofwork.gpu_failed,
    as the reference's _doGPUPoW clears openclpow.enabledGpus); the next test starts enabled."""
    yield
    from pybitmessage_amd import hippow, proofofwork
    proofofwork._disabled = None
    hippow._setting = None  # the keys.dat opencl value hippow.initCL remembers
