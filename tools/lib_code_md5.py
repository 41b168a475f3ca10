#!/usr/bin/env python3
"""md5 of a library's device code: the .hip_fatbin section of libbmpow_hip.so (every gfx950 code
object), which a rebuild of the same sources reproduces bit for bit -- unlike the whole file, whose host
code carries the build time (bmpow_version).  The PMC counters describe the device code, so this is their
provenance key (tools/profile_pmc.sh stamps it, bench.py compares it with the library it loaded).

    python3 tools/lib_code_md5.py [path]
"""
import hashlib
import struct
import sys


def code_md5(path, section=b'.hip_fatbin'):
    """md5 hex digest of the ELF section `section` of `path`, or None."""
    try:
        with open(path, 'rb') as f:
            data = f.read()
    except OSError:
        return None
    if data[:4] != b'\x7fELF' or data[4] != 2:  # 64-bit ELF only
        return None
    shoff, = struct.unpack_from('<Q', data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', data, 0x3A)
    def sh(i):
        return struct.unpack_from('<IIQQQQIIQQ', data, shoff + i * shentsize)
    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        name, _, _, _, off, size = sh(i)[:6]
        end = data.index(b'\0', stroff + name)
        if data[stroff + name:end] == section:
            return hashlib.md5(data[off:off + size]).hexdigest()
    return None


if __name__ == '__main__':
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    print(code_md5(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, 'pybitmessage_amd', 'lib', 'libbmpow_hip.so')))
