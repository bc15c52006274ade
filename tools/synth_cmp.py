"""Does the CPU oracle's synthetic IF generator (or_synth_if) give the same bytes as the HIP
one (gnss_synth_if_device) for the config-5 scenario? If so, the config-5 golden's oracle runs
can be made on any CPU from or_synth_if's record. Compares 20-ms chunks at the start, the
middle and the end of the bench's 91-s record; prints the differing byte counts.
Run on the GPU box: python tools/synth_cmp.py"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
pkg = importlib.import_module("assignment-for-aae6102_gnss-sdr_amd")
import pyoracle as po  # noqa: E402

ctx = pkg.Context(0)
S = 58000
cfg = pkg.synth.all_prn(32, skip_ms=0)
total = (1000 + 19 + 90000 + 3) * S
bad_total = 0
for start_ms in (0, 500, 45000, 91000):
    n = 20 * S
    s0 = start_ms * S
    if s0 + n > total:
        s0 = total - n
    dev = pkg.DeviceRecord(ctx, 2 * n)
    pkg.synth.generate_device(ctx, cfg, dev, sample0=s0, nsamples=n)
    g = dev.download()
    dev.free()
    c = po.synth_if(cfg, s0, n)
    bad = int(np.count_nonzero(g != c))
    bad_total += bad
    print(f"ms {start_ms}: {bad} of {2 * n} bytes differ", flush=True)
print("SYNTH_EQUAL" if bad_total == 0 else f"SYNTH_DIFFER {bad_total}")
