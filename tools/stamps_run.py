"""Summarise GNSS_STAMPS dumps of the persistent tracking kernel (channel 0, one row per
step of the last launch): per-step latencies in us (100 MHz wall clock). Row layout
(track_run_kernel): [0] step start, [1] computed, [2] partial out, [3] all partials in,
[4] next descriptor ready, for block 0; [5..9] the same for the last block."""
import sys
import numpy as np
ROW = 8 + 3 * 1024
for path in sys.argv[1:]:
    a = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :10].astype(np.int64)
    a = a[(a[:, 0] != 0) & (a[:, 5] != 0)]
    if len(a) < 3:
        print(path, "no rows"); continue
    us = lambda x: np.median(x) * 0.01
    print(path, "steps", len(a))
    for name, i in [("start -> computed", 0), ("computed -> partial out", 1),
                    ("partial out -> all partials in", 2), ("all in -> next desc ready", 3)]:
        print(f"  {name:32s} blk0 {us(a[:, i + 1] - a[:, i]):7.2f}   last {us(a[:, i + 6] - a[:, i + 5]):7.2f}")
    lastout = np.maximum(a[:, 2], a[:, 7])
    print(f"  {'last partial out -> blk0 all in':32s} {us(a[:, 3] - lastout):7.2f}")
    print(f"  {'step period (blk0)':32s} {us(np.diff(a[:, 0])):7.2f}")
