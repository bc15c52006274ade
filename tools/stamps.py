"""Summarise GNSS_STAMPS dumps (track.hip timing probe): per-launch wall-clock marks
(100 MHz) of channel 0 relative to its first block's start. Args: file [file...]."""
import sys
import numpy as np
B = 1024
ROW = 8 + 3 * B
for path in sys.argv[1:]:
    a = np.fromfile(path, dtype=np.uint64)
    rows = a[:-1].reshape(-1, ROW).astype(np.int64)
    rows = rows[(rows[:, 7] != 0)]
    st, cm, tk = rows[:, 8:8 + B], rows[:, 8 + B:8 + 2 * B], rows[:, 8 + 2 * B:]
    nb = (st != 0).sum(1)
    big = np.iinfo(np.int64).max
    t0 = np.where(st != 0, st, big).min(1)
    marks = {
        "last block start": st.max(1), "first block computed": np.where(cm != 0, cm, big).min(1),
        "last block computed": cm.max(1), "last ticket issued": tk.max(1), "last has ticket": rows[:, 3],
        "sums final": rows[:, 4], "loop updated": rows[:, 5], "next desc stored": rows[:, 6],
        "state stored": rows[:, 7]}
    if rows[:, 2].any():
        marks.update({"warm: loop start": rows[:, 0], "warm: loop updated": rows[:, 1],
                      "warm: desc stored": rows[:, 2]})
    print(path, "launches", len(rows), "blocks/ch", int(np.median(nb)))
    for k, v in marks.items():
        r = (v - t0) * 0.01
        print(f"  {k:22s} median {np.median(r):7.2f} us  p90 {np.percentile(r, 90):7.2f}")
    print(f"  {'start-to-start':22s} median {np.median(np.diff(t0)) * 0.01:7.2f} us")
