"""HBM traffic of the dominant kernel from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; MI355X_MICROARCH.md HBM section: both in KB per dispatch, FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads on gfx950 -> doubled).
Args: fetch_dir write_dir kernel_substring out.json [workload note] (stamped with the source digest)"""
import csv, glob, json, sys
import numpy as np


def per_dispatch(d, counter, ksub):
    vals = {}
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if ksub in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                key = r.get("Dispatch_Id", r.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return np.array(list(vals.values()))


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
write = per_dispatch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
out = {"kernel": sys.argv[3], "dispatches": [int(fetch.size), int(write.size)],
       "fetch_kb_per_dispatch_raw": float(np.median(fetch)) if fetch.size else None,
       "write_kb_per_dispatch": float(np.median(write)) if write.size else None}
if fetch.size and write.size:
    out["bytes_per_launch"] = 2 * out["fetch_kb_per_dispatch_raw"] * 1024 + out["write_kb_per_dispatch"] * 1024
    out["note"] = ("median over dispatches; FETCH_SIZE doubled (gfx950 16-B/lane streaming reads), "
                   "both KB -> bytes; workload " + (sys.argv[5] if len(sys.argv) > 5 else
                   "tools/track_only.py 1000 40000 (8 ch, the bench trackingCT: one persistent launch = 4000 10-ms steps)"))
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import srcdigest  # noqa: E402
srcdigest.stamp(out)
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
