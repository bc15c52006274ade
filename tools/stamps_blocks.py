"""Per-block view of a GNSS_STAMPS dump of the persistent tracking kernel (probe builds; channel
0): every block's step start ([40 + blk]) and correlate end ([296 + blk]) per step row, next to
block 0's exchange stamps. Prints the medians over the steps of: a block's correlate time, the
slowest block's, the spread of the blocks' start times, the span from the first start to the
last correlate end, and the blocks that are slowest most often.
Usage: python3 tools/stamps_blocks.py DUMP [nblocks]"""
import sys

import numpy as np

ROW = 8 + 3 * 1024
path = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 96
a = np.fromfile(path, dtype=np.uint64)[:-1].reshape(-1, ROW).astype(np.int64)
st, en = a[:, 40:40 + nb], a[:, 296:296 + nb]
ok = (st > 0).all(axis=1) & (en > 0).all(axis=1) & (a[:, 0] > 0) & (a[:, 3] > 0)
st, en, a = st[ok], en[ok], a[ok]
us = 0.01  # 100 MHz wall clock
dur = (en - st) * us
print(f"{path}: {len(a)} steps x {nb} blocks")
print(f"  block correlate (start -> computed): median {np.median(dur):.2f} us, p90 {np.percentile(dur, 90):.2f}, "
      f"slowest block per step: median {np.median(dur.max(axis=1)):.2f}")
print(f"  block start spread (max - min): median {np.median((st.max(1) - st.min(1)) * us):.2f} us; "
      f"first start -> last computed: median {np.median((en.max(1) - st.min(1)) * us):.2f} us")
print(f"  blk0 start -> blk0 all partials in: median {np.median((a[:, 3] - a[:, 0]) * us):.2f} us; "
      f"last computed -> blk0 all in: median {np.median((a[:, 3] - en.max(1)) * us):.2f} us")
late = np.bincount(np.argmax(en, axis=1), minlength=nb)
top = np.argsort(late)[::-1][:6]
print("  last to finish its correlate, most often: " + ", ".join(f"blk {b} ({late[b]})" for b in top))
slow = np.argsort(np.median(dur, axis=0))[::-1][:6]
print("  slowest median correlate: " + ", ".join(f"blk {b} {np.median(dur[:, b]):.2f}" for b in slow))
late_start = np.argsort(np.median(st - st.min(1, keepdims=True), axis=0))[::-1][:6]
print("  latest median start: " + ", ".join(f"blk {b} +{np.median((st[:, b] - st.min(1)) * us):.2f}" for b in late_start))
# block 0's flush of the previous step (wave 1, stamps [16] / [17]) against its sweep ([2] partial
# out, [3] all partials in)
f0, f1 = a[:, 16], a[:, 17]
m = (f0 > 0) & (f1 > 0)
if m.any():
    print(f"  blk0 flush (wave 1: record, state, C/N0): median {np.median((f1 - f0)[m]) * us:.2f} us, p90 "
          f"{np.percentile((f1 - f0)[m], 90) * us:.2f}; flush end - all partials in: median "
          f"{np.median((f1 - a[:, 3])[m]) * us:+.2f} us; partial out -> flush start {np.median((f0 - a[:, 2])[m]) * us:+.2f}")
    print(f"  blk0: all in -> next ready {np.median((a[:, 4] - a[:, 3])) * us:.2f}; its start vs the earliest block "
          f"{np.median((a[:, 40] - st.min(1))) * us:+.2f}")
# every block's all-in ([552 + blk]) and ready ([808 + blk]) stamps
ai, rd = a[:, 552:552 + nb], a[:, 808:808 + nb]
m = (ai > 0).all(axis=1) & (rd > 0).all(axis=1)
if m.any():
    ai, rd, st2, en2 = ai[m], rd[m], st[m], en[m]
    lastpub = en2.max(1, keepdims=True)
    print(f"  all-in after the last correlate end: blk0 {np.median(ai[:, 0] - lastpub[:, 0]) * us:+.2f}, "
          f"others median {np.median(ai[:, 1:] - lastpub) * us:+.2f} (p10 {np.percentile(ai[:, 1:] - lastpub, 10) * us:+.2f}, "
          f"p90 {np.percentile(ai[:, 1:] - lastpub, 90) * us:+.2f})")
    print(f"  tail (all-in -> ready): blk0 {np.median(rd[:, 0] - ai[:, 0]) * us:.2f}, others {np.median(rd[:, 1:] - ai[:, 1:]) * us:.2f}")
    ai_late = np.argsort(np.median(ai - ai.min(1, keepdims=True), axis=0))[::-1][:6]
    print("  latest all-in: " + ", ".join(f"blk {b} +{np.median(ai[:, b] - ai.min(1)) * us:.2f}" for b in ai_late))
# every block's flush of the previous step (wave 1: [1064 + blk] start, [1320 + blk] end)
f0, f1 = a[:, 1064:1064 + nb], a[:, 1320:1320 + nb]
m = (f0 > 0).all(axis=1) & (f1 > 0).all(axis=1)
if m.any():
    fd = (f1[m] - f0[m]) * us
    fs = (f0[m] - st[m].min(1, keepdims=True)) * us
    top = np.argsort(np.median(fd, axis=0))[::-1][:6]
    print("  longest median flush: " + ", ".join(f"blk {b} {np.median(fd[:, b]):.2f}" for b in top)
          + f"; others median {np.median(fd):.2f}")
    print("  flush start after the earliest step start: " + ", ".join(
        f"blk {b} {np.median(fs[:, b]):+.2f}" for b in top))
# (GNSS_FLUSH_PROBE & 2 builds) block 0's record part cold, then the whole record again warm
f0, f1, f2 = a[:, 2000], a[:, 2001], a[:, 2002]
m = (f0 > 0) & (f1 > 0) & (f2 > 0)
if m.any():
    print(f"  blk0 record: first (cold) {np.median((f1 - f0)[m]) * us:.2f} us, again (warm, all fields) "
          f"{np.median((f2 - f1)[m]) * us:.2f} us")
