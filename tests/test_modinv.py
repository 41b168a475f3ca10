"""Field inversion of the address search (pybitmessage_amd/csrc/modinv_dev.h, Bernstein-Yang
divsteps) compiled for the HOST from the same source the gfx950 kernel includes, checked against
Python's pow(x, -1, p).  The GPU side of the same code is pinned end to end by
tests/test_addressgen.py (public keys of the reference's pointMult and sample vectors)."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT

P = 2 ** 256 - 2 ** 32 - 977
CSRC = os.path.join(ROOT, 'pybitmessage_amd', 'csrc')

HARNESS = r'''
#include "modinv_dev.h"
extern "C" void inv_batch(const uint32_t* a, uint32_t* r, int n) {
  for (int k = 0; k < n; ++k) {
    uint32_t x[8], y[8];
    for (int i = 0; i < 8; ++i) x[i] = a[8 * k + i];
    mi::inv_mod_p(y, x);
    for (int i = 0; i < 8; ++i) r[8 * k + i] = y[i];
  }
}
'''


@pytest.fixture(scope='module')
def hostinv(tmp_path_factory):
    d = tmp_path_factory.mktemp('modinv')
    src, so = d / 'h.cpp', d / 'libh.so'
    src.write_text(HARNESS)
    subprocess.check_call(['g++', '-O2', '-std=c++17', '-Wall', '-Werror', '-Wno-unknown-pragmas', '-fPIC', '-shared',
                           '-fsanitize=undefined', '-fno-sanitize-recover=all',
                           '-I', CSRC, '-o', str(so), str(src)])
    lib = ctypes.CDLL(str(so))
    lib.inv_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

    def inv(xs):
        n = len(xs)
        a = (ctypes.c_uint32 * (8 * n))()
        for k, x in enumerate(xs):
            for i in range(8):
                a[8 * k + i] = (x >> (32 * i)) & 0xFFFFFFFF
        r = (ctypes.c_uint32 * (8 * n))()
        lib.inv_batch(a, r, n)
        return [sum(r[8 * k + i] << (32 * i) for i in range(8)) for k in range(n)]
    return inv


def test_edge_values(hostinv):
    xs = [1, 2, 3, 977, 2 ** 32, 2 ** 32 + 977, P - 1, P - 2, (P - 1) // 2, (P + 1) // 2,
          2 ** 255, 2 ** 256 - 2 ** 32 - 978, 2 ** 240, 2 ** 240 - 1, 2 ** 30, 2 ** 30 - 1,
          0xFFFFFFFF, 2 ** 224 + 1]
    xs += [2 ** i for i in range(256)]
    xs += [P - 2 ** i for i in range(32, 256)]
    got = hostinv(xs)
    for x, r in zip(xs, got):
        assert r == pow(x, -1, P), hex(x)


def test_random_values(hostinv):
    rng = random.Random(11)
    xs = [rng.randrange(1, P) for _ in range(3000)]
    # sparse and dense limb patterns (carry chains of the 30/32-bit repacking)
    for _ in range(500):
        x = 0
        for i in range(8):
            x |= rng.choice([0, 0xFFFFFFFF, rng.getrandbits(32)]) << (32 * i)
        if 0 < x < P:
            xs.append(x)
    got = hostinv(xs)
    bad = [hex(x) for x, r in zip(xs, got) if r != pow(x, -1, P)]
    assert not bad, bad[:5]
