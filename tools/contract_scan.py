"""Floating-point contraction audit of a HIP source compiled with `#pragma clang fp contract(fast)`:
counts the sums whose two operands are both products (a*b + c*d) in the device LLVM IR. The
backend may fuse either product into an FMA, chosen by the schedule, so two kernels built from
the same source expression (or one kernel after a refactor) may round differently. Such sums
must be written with the fused product fixed (acq_fft.hip: fma2). Prints the count per kernel
and the total; exit status 1 if any.
Usage: python3 tools/contract_scan.py SOURCE.hip   (hipcc --cuda-device-only -emit-llvm, gfx950)"""
import collections
import os
import re
import subprocess
import sys
import tempfile


def scan(ll_path):
    amb = collections.Counter()
    cur, defs = None, {}
    for line in open(ll_path):
        m = re.match(r'define .*@(\S+)\(', line)
        if m:
            cur, defs = m.group(1), {}
            continue
        m = re.match(r'\s*(%[\w.]+) = (fmul|fadd|fsub|fneg|call)\b(.*)', line)
        if not m:
            continue
        name, op, rest = m.groups()
        if op == 'call':
            continue
        defs[name] = op
        if op == 'fneg':
            o = re.findall(r'(%[\w.]+)', rest)
            if o and defs.get(o[0]) == 'fmul':
                defs[name] = 'fmul'
        if op in ('fadd', 'fsub') and 'contract' in rest:
            ops = re.findall(r'(%[\w.]+)', rest)[:2]
            if len(ops) == 2 and all(defs.get(o) == 'fmul' for o in ops):
                amb[cur] += 1
    return amb


def main(src):
    inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'include')
    with tempfile.TemporaryDirectory() as d:
        ll = os.path.join(d, 'out.ll')
        subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC',
                        '-ffp-contract=off', '--cuda-device-only', '-S', '-emit-llvm', '-I', inc, src, '-o', ll],
                       check=True, capture_output=True)
        amb = scan(ll)
    for k, v in sorted(amb.items()):
        print(v, k)
    n = sum(amb.values())
    print('ambiguous two-product sums:', n)
    return n


if __name__ == '__main__':
    sys.exit(1 if main(sys.argv[1]) else 0)
