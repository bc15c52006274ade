"""Print the cos/sin(2*pi*m/P) literal tables (fp64) used by csrc/acq_fft.hip for the
prime column DFTs (the fp32 kernels round them to float). Usage:
python3 tools/gen_dft_consts.py 13 29"""
import math
import sys

for P in map(int, sys.argv[1:]):
    c = [math.cos(2 * math.pi * m / P) for m in range(P)]
    s = [math.sin(2 * math.pi * m / P) for m in range(P)]
    fmt = lambda v: ", ".join(repr(x) for x in v)
    print(f"template <> struct PrimeTab<{P}> {{")
    print(f"    static constexpr double c[{P}] = {{{fmt(c)}}};")
    print(f"    static constexpr double s[{P}] = {{{fmt(s)}}};")
    print("};")
