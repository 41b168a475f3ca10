#!/usr/bin/env python3
"""The issue ceiling of bm_search_kernel's own instruction mix (VERDICT r02 "measure the real
ceiling, then decide whether kernel tuning continues").

Generates tools/ubench_mix.hip: kernels whose body is the search kernel's nonce-loop VALU stream,
opcode for opcode and in the compiler's order, with the data dependences removed -- every
instruction reads registers written >= 24 instructions earlier, and every v_bitop3_b32 reads three
different VGPR banks (the bank-split form that co-issues).  Whatever such a stream issues per SIMD
per quad-cycle is the most the mix can issue: the kernel's own dependences can only lower it.

    python tools/ubench_mix.py build/isa/bmpow_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
    hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mix tools/ubench_mix.hip
    ./tools/ubench_mix                     (on the GPU box; one JSON line per variant)

Variants, each at 4..8 waves per SIMD (the VGPR count set by a clobber, as the kernel's own
__launch_bounds__ does):
  order    the kernel's exact opcode sequence (the 31 other VALU ops -- moves, readlanes, compares --
           as v_mov_b32);
  spread   the same multiset with the bitop3 spaced evenly among the half-rate ops;
  grouped  the same multiset with each round's bitop3 issued back to back (BM_GROUP_BITOP3's shape).
  phased   (round 4) every bitop3 of the iteration first, then the single-issue ops, in 1,024-lane
           workgroups (all 4 waves of a SIMD from one workgroup) that meet at a barrier each
           iteration, so the waves sharing a SIMD run their bitop3 at the same time: what the mix
           issues when every bitop3 finds a partner -- the all-pairs bound, measured, not argued;
  phased_nobar  the same stream without the barrier (the waves drift apart);
  order_bar  the compiler's order in the phased workgroups (phasing without regrouping).
Reported: VALU instructions per SIMD per quad-cycle (IPQ) = waves x instructions / (SIMDs x cycles
/ 4), cycles from the kernel time and the s_memtime / s_memrealtime clock of block 0.
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from isa_census import kernel_lines  # noqa: E402

POOL = 48  # 32-bit registers v0..v47 take the stream's results (v48.. stay the compiler's)
WAVES = {2: 256, 4: 128, 5: 96, 6: 80, 7: 72, 8: 64}  # waves/SIMD -> VGPRs that give that occupancy


def loop_ops(path, name='bm_search_kernel'):
    body = kernel_lines(path, name)
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.match(r'^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)', l)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i and (best is None or i - labels[tgt] > best[1] - best[0]):
                best = (labels[tgt], i)
    ops = []
    for l in body[best[0]:best[1] + 1]:
        m = re.match(r'^\s+(v_[a-z0-9_]+)', l)
        if m:
            ops.append(m.group(1))
    return ops


def classify(op):
    if op.startswith('v_alignbit_b32'):
        return 'A'
    if op.startswith('v_bitop3_b32'):
        return 'B'
    if op.startswith('v_lshl_add_u64'):
        return 'L'
    if op.startswith('v_lshrrev_b64'):
        return 'S'
    return 'M'


class Regs(object):
    """Round-robin destinations; sources are the registers written longest ago."""

    def __init__(self):
        self.i = 0

    def r32(self):
        r = self.i % POOL
        self.i += 5  # 5 is odd and prime to 48: destinations cycle through every bank
        return r

    def pair(self):
        r = (self.i % POOL) & ~1
        self.i += 6
        return r

    def old32(self, back, bank=None):
        for k in range(back, back + 64):
            r = (self.i - 5 * k) % POOL
            if bank is None or r % 4 == bank:
                return r
        raise AssertionError

    def oldpair(self, back):
        return ((self.i - 6 * back) % POOL) & ~1


def emit(kinds):
    regs = Regs()
    out = []
    for k in kinds:
        if k == 'A':
            s1, s2 = regs.old32(24), regs.old32(26)
            d = regs.r32()
            out.append('v_alignbit_b32 v%d, v%d, v%d, 7' % (d, s1, s2))
        elif k == 'B':
            s1 = regs.old32(24)
            s2 = regs.old32(25, (s1 + 1) % 4)
            s3 = regs.old32(26, (s1 + 2) % 4)
            d = regs.r32()
            out.append('v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96' % (d, s1, s2, s3))
        elif k == 'L':
            s1, s2 = regs.oldpair(12), regs.oldpair(14)
            d = regs.pair()
            out.append('v_lshl_add_u64 v[%d:%d], v[%d:%d], 0, v[%d:%d]' % (d, d + 1, s1, s1 + 1, s2, s2 + 1))
        elif k == 'S':
            s1 = regs.oldpair(12)
            d = regs.pair()
            out.append('v_lshrrev_b64 v[%d:%d], 7, v[%d:%d]' % (d, d + 1, s1, s1 + 1))
        else:
            s1 = regs.old32(24)
            d = regs.r32()
            out.append('v_mov_b32 v%d, v%d' % (d, s1))
    return out


def spread(kinds):
    b = kinds.count('B')
    rest = [k for k in kinds if k != 'B']
    out, acc = [], 0.0
    step = len(rest) / float(b)
    bi = 0
    for i, k in enumerate(rest):
        out.append(k)
        acc += 1
        while bi < b and acc >= step * (bi + 1):
            out.append('B')
            bi += 1
    out += ['B'] * (b - bi)
    return out


def grouped(kinds, per=8):
    """bitop3 held back and issued in groups of `per` at the position of the group's last one."""
    out, held = [], 0
    for k in kinds:
        if k == 'B':
            held += 1
            if held == per:
                out += ['B'] * per
                held = 0
        else:
            out.append(k)
    return out + ['B'] * held


def phased(kinds):
    return ['B'] * kinds.count('B') + [k for k in kinds if k != 'B']


def kernel_src(name, lines, waves, threads=256, barrier=False):
    regs_needed = WAVES[waves]
    clob = ', '.join('"v%d"' % i for i in range(POOL)) + ', "v%d"' % (regs_needed - 1)
    body = '\\n\\t'.join(lines)
    return '''
__global__ __launch_bounds__(%(t)d, %(wb)d) void %(name)s(uint64_t* clk, int iters) {
  uint64_t t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
    %(bar)s
    asm volatile("%(body)s" ::: %(clob)s);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}
''' % {'t': threads, 'wb': max(1, waves * 256 // threads), 'name': name, 'body': body, 'clob': clob,
       'bar': '__syncthreads();' if barrier else ''}


def main():
    path = sys.argv[1]
    ops = loop_ops(path)
    kinds = [classify(o) for o in ops]
    variants = {'order': kinds, 'spread': spread(kinds), 'grouped': grouped(kinds)}
    for v in variants.values():
        assert sorted(v) == sorted(kinds)
    counts = {k: kinds.count(k) for k in 'ABLSM'}
    src = ['// GENERATED by tools/ubench_mix.py from %s -- do not edit' % os.path.basename(path),
           '#include <hip/hip_runtime.h>', '#include <stdint.h>', '#include <stdio.h>']
    table = []
    for vname, vk in variants.items():
        lines = emit(vk)
        for w in sorted(WAVES):
            kn = 'mix_%s_w%d' % (vname, w)
            src.append(kernel_src(kn, lines, w))
            table.append((kn, vname, w, 256))
    ph = phased(kinds)
    assert sorted(ph) == sorted(kinds)
    lines = emit(ph)
    for vname, bar in (('phased', True), ('phased_nobar', False)):
        kn = 'mix_%s_w4' % vname
        src.append(kernel_src(kn, lines, 4, threads=1024, barrier=bar))
        table.append((kn, vname, 4, 1024))
    # the compiler's order in the same phased workgroups: does phasing alone help a spread-out mix?
    kn = 'mix_order_bar_w4'
    src.append(kernel_src(kn, emit(kinds), 4, threads=1024, barrier=True))
    table.append((kn, 'order_bar', 4, 1024))
    # each round's bitop3 moved to the front of its round (about 11 in a run), and two trials per lane
    # interleaved round by round (about 22 in a run, 2 waves per SIMD at twice the registers): how much
    # of the phased pairing survives clusters a dataflow could form
    per = len(kinds) / 160.0
    chunks = [kinds[int(i * per):int((i + 1) * per)] for i in range(160)]
    roundcl = [k for c in chunks for k in (['B'] * c.count('B') + [x for x in c if x != 'B'])]
    roundcl2 = [k for c in chunks for k in (['B'] * (2 * c.count('B')) + [x for x in c + c if x != 'B'])]
    assert sorted(roundcl) == sorted(kinds) and len(roundcl2) == 2 * len(kinds)
    for vname, vk, w, t in (('roundcl_bar', roundcl, 4, 1024), ('roundcl', roundcl, 4, 256),
                            ('roundcl2_bar', roundcl2, 2, 512), ('roundcl2', roundcl2, 2, 128)):
        kn = 'mix_%s_w%d' % (vname, w)
        src.append(kernel_src(kn, emit(vk), w, threads=t, barrier=vname.endswith('_bar')))
        table.append((kn, vname, w, t))
    src.append('''
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \\
  fprintf(stderr, "HIP error %%s at %%s:%%d\\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)
typedef void (*kfn)(uint64_t*, int);
struct Var { kfn f; const char* name; const char* variant; int waves; int threads; int nvalu; };
static const Var kVars[] = {
%s
};
int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, simds = 4 * cus;
  const int nvalu = %d;
  uint64_t* d_clk;
  CHECK(hipMalloc(&d_clk, 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("{\\"device\\": \\"%%s\\", \\"cus\\": %%d, \\"valu_per_iter\\": %%d, \\"mix\\": %s}\\n", p.gcnArchName, cus, nvalu);
  for (const Var& v : kVars) {
    const int iters = 16, blocks = cus * v.waves * 6 * 256 / v.threads;  // 6 rounds of resident workgroups
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(v.f, dim3(blocks), dim3(v.threads), 0, 0, d_clk, 1);
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(v.f, dim3(blocks), dim3(v.threads), 0, 0, d_clk, iters);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      uint64_t clk[2];
      CHECK(hipMemcpy(clk, d_clk, 16, hipMemcpyDeviceToHost));
      const double ghz = clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 0.0;  // memrealtime: 100 MHz
      const double cycles = ms * 1e-3 * ghz * 1e9;
      const double wave_instr = (double)blocks * (v.threads / 64) * iters * v.nvalu;
      const double ipq = wave_instr / (simds * cycles / 4.0);
      printf("{\\"kernel\\": \\"%%s\\", \\"variant\\": \\"%%s\\", \\"waves_per_simd\\": %%d, \\"rep\\": %%d, \\"ms\\": %%.3f, "
             "\\"clock_ghz\\": %%.3f, \\"valu_per_simd_quadcycle\\": %%.4f}\\n", v.name, v.variant, v.waves, rep, ms, ghz, ipq);
      fflush(stdout);
    }
  }
  return 0;
}
''' % (',\n'.join('  {%s, "%s", "%s", %d, %d, %d}' % (kn, kn, vn, w, t, len(kinds) * (2 if '2' in vn else 1)) for kn, vn, w, t in table), len(kinds),
       str(counts).replace("'", '\\"')))
    dst = os.path.join(HERE, 'ubench_mix.hip')
    with open(dst, 'w') as f:
        f.write('\n'.join(src))
    print('wrote %s: %d VALU per iteration %s, %d kernels' % (dst, len(kinds), counts, len(table)))


if __name__ == '__main__':
    main()
