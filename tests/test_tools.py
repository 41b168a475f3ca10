"""The measurement tools behind the round-5 bench-line fields (no GPU): the per-call timeline of serial
run() calls (tools/c1_timeline.py) on a synthetic rocprofv3 trace, and the device-code md5 that stamps
the PMC passes (tools/lib_code_md5.py) on a synthetic ELF."""
import csv
import hashlib
import json
import os
import struct
import subprocess
import sys

from tests.conftest import ROOT


def _write_trace(d, kernels, apis):
    with open(os.path.join(d, 'run_kernel_trace.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Correlation_Id', 'Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
        w.writerows(kernels)
    with open(os.path.join(d, 'run_hip_api_trace.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Correlation_Id', 'Function', 'Start_Timestamp', 'End_Timestamp'])
        w.writerows(apis)


def test_c1_timeline_groups_split_calls(tmp_path):
    """Three calls of two pieces each (launches in a burst, calls 1.5 ms apart; the second call's pieces
    start behind the first call's kernels): per call the wall time, the host-exposed time (no kernel of
    the call running), the launch span and the launch-to-kernel latency."""
    k, a = [], []
    cid = 0
    for c in range(3):
        t0 = c * 1_500_000  # ns
        for p in range(2):
            cid += 1
            a.append((cid, 'hipLaunchKernel', t0 + p * 3000, t0 + p * 3000 + 2000))
            a.append((1000 + cid, 'hipEventRecord', t0 + p * 3000 + 2000, t0 + p * 3000 + 2500))
            k.append((cid, 'void bm_search1_kernel<true>(bm_one_args)', t0 + 10_000 + p * 1000, t0 + 1_400_000))
    _write_trace(str(tmp_path), k, a)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'c1_timeline.py'), str(tmp_path)],
                         capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d['calls'] == 2  # the last call has no successor to end its wall interval
    m = d['median']
    assert m['wall_us'] == 1500.0 and m['launches'] == 2
    assert m['launch_span_us'] == 5.0 and m['launch_to_kernel_us'] == 10.0
    # busy from 10 us to 1,400 us of the 1,500 us call
    assert m['host_exposed_us'] == 110.0 and m['kernel_end_to_next_call_us'] == 100.0


def _elf_with(section_name, payload):
    """A minimal 64-bit ELF: a null section, the named section and .shstrtab."""
    shstr = b'\0' + section_name + b'\0.shstrtab\0'
    data_off = 64
    shstr_off = data_off + len(payload)
    shoff = (shstr_off + len(shstr) + 7) & ~7
    hdr = bytearray(64)
    hdr[:4] = b'\x7fELF'
    hdr[4] = 2
    hdr[5] = 1
    struct.pack_into('<Q', hdr, 0x28, shoff)
    struct.pack_into('<HHH', hdr, 0x3A, 64, 3, 2)
    body = bytes(hdr) + payload + shstr
    body += b'\0' * (shoff - len(body))

    def sh(name, off, size):
        return struct.pack('<IIQQQQIIQQ', name, 1, 0, 0, off, size, 0, 0, 1, 0)
    body += sh(0, 0, 0) + sh(1, data_off, len(payload)) + sh(1 + len(section_name) + 1, shstr_off, len(shstr))
    return body


def test_lib_code_md5_reads_the_fatbin_section(tmp_path):
    sys.path.insert(0, ROOT)
    from tools.lib_code_md5 import code_md5
    payload = b'device code object bytes' * 10
    p = tmp_path / 'lib.so'
    p.write_bytes(_elf_with(b'.hip_fatbin', payload))
    assert code_md5(str(p)) == hashlib.md5(payload).hexdigest()
    q = tmp_path / 'other.so'
    q.write_bytes(_elf_with(b'.text', payload))
    assert code_md5(str(q)) is None
    assert code_md5(str(tmp_path / 'missing.so')) is None
