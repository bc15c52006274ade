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
    a = a[np.argsort(a[:, 0])]  # rows wrap (row = step % slots)
    dp = np.diff(a[:, 0]) * 0.01
    dp = dp[dp < 1000]
    print(f"  {'step period (blk0)':32s} {np.median(dp):7.2f}  mean {dp.mean():6.2f}  p90 {np.percentile(dp, 90):6.2f}  p99 {np.percentile(dp, 99):6.2f}  max {dp.max():7.2f}")
    print("  period tail: " + ", ".join(f">{t} us: {int((dp > t).sum())} steps {dp[dp > t].sum():.0f} us"
                                        for t in (8, 10, 15, 30, 100)) + f" (of {dp.sum():.0f} us)")
    big = np.argsort(dp)[-3:]
    for i in big:  # where the slowest steps spent their time (blk0 stamps)
        r, nx = a[i], a[i + 1]
        print(f"   slow step: {dp[i]:.1f} us = corr {(r[1]-r[0])*0.01:.2f} part {(r[2]-r[1])*0.01:.2f} "
              f"xchg {(r[3]-r[2])*0.01:.2f} tail {(r[4]-r[3])*0.01:.2f} gap {(nx[0]-r[4])*0.01:.2f}")
    b = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :14].astype(np.int64)
    b = b[(b[:, 0] != 0) & (b[:, 5] != 0) & (b[:, 10] != 0)]
    if len(b):
        print(f"  blk0 tail: all in -> s_fin {us(b[:, 10] - b[:, 3]):6.2f}, -> loop upd {us(b[:, 11] - b[:, 10]):6.2f}, "
              f"-> code desc {us(b[:, 12] - b[:, 11]):6.2f}, -> carrier desc {us(b[:, 13] - b[:, 11]):6.2f}, "
              f"-> ready {us(b[:, 4] - np.maximum(b[:, 12], b[:, 13])):6.2f}")
    c = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :16].astype(np.int64)
    c = c[(c[:, 14] != 0) & (c[:, 15] != 0) & (c[:, 11] != 0)]
    if len(c):
        print(f"  code role: loop upd -> n {us(c[:, 14] - c[:, 11]):6.2f}, -> colon {us(c[:, 15] - c[:, 14]):6.2f}, "
              f"-> stored {us(c[:, 12] - c[:, 15]):6.2f}")
    r0 = np.fromfile(path, dtype=np.uint64)[:3080].astype(np.int64)
    spans = [(ch, (r0[21 + 3 * ch] - r0[20 + 3 * ch]) * 0.01, r0[22 + 3 * ch]) for ch in range(64) if r0[21 + 3 * ch]]
    if spans:
        print("  per-channel launch span (us) / steps:", ", ".join(f"ch{c} {t:.0f}/{n}" for c, t, n in spans))
    e = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :45].astype(np.int64)
    e = e[(e[:, 40] != 0) & (e[:, 44] != 0)]
    if len(e):  # probe bit 32: block 0 thread 0's lane phases
        print(f"  lane: start->corr entry {us(e[:, 40] - e[:, 0]):6.2f}, boundary search {us(e[:, 41] - e[:, 40]):6.2f}, "
              f"sincos {us(e[:, 42] - e[:, 41]):6.2f}, samples {us(e[:, 43] - e[:, 42]):6.2f}, "
              f"epilogue {us(e[:, 44] - e[:, 43]):6.2f}, -> computed {us(e[:, 1] - e[:, 44]):6.2f}")
    d = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :23].astype(np.int64)
    d = d[(d[:, 16] != 0) & (d[:, 21] != 0) & (d[:, 2] != 0)]
    if len(d):
        print(f"  flush: blk0 start-after-publish {us(d[:, 16] - d[:, 2]):6.2f} dur {us(d[:, 17] - d[:, 16]):6.2f}; "
              f"last dur {us(d[:, 22] - d[:, 21]):6.2f}")
    e = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :25]
    e = e[(e[:, 23] != 0) & (e[:, 3] != 0)]
    if len(e):
        lat = e[:, 23].astype(np.int64); ear = (~e[:, 24]).astype(np.int64)
        print(f"  all blocks: first->last partial out {us(lat - ear):6.2f}; latest partial -> blk0 all in {us(e[:, 3].astype(np.int64) - lat):6.2f}; blk0 partial -> latest {us(lat - e[:, 2].astype(np.int64)):6.2f}")
    e = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :20].astype(np.int64)
    e = e[(e[:, 18] != 0) & (e[:, 19] != 0)]
    if len(e):
        print(f"  tail repeated in place (probe 16): {us(e[:, 19] - e[:, 18]) / 4:6.2f} us per repetition")
        g = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW)[:, :33].astype(np.int64)
        g = g[(g[:, 18] != 0) & (g[:, 25] != 0)]
        if len(g):
            print("   its first repetition by wave (loop update / role end, us from the start): " + ", ".join(
                f"w{w} {us(g[:, 29 + w] - g[:, 18]):.2f}/{us(g[:, 25 + w] - g[:, 18]):.2f}" for w in range(4)))
