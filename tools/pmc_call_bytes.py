"""HBM bytes per call of a multi-kernel stage from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE in KB per dispatch; FETCH_SIZE doubled for gfx950's 16-B/lane streaming reads,
MI355X_MICROARCH.md HBM section): every dispatch of the kernels whose names contain one of
the given substrings, summed, divided by the number of calls the workload made.
Args: fetch_dir write_dir ncalls out.json note kernel_substring... (digest-stamped)"""
import csv, glob, json, os, sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import srcdigest  # noqa: E402


def total(d, counter, subs):
    per = {}
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name", "")
            if r.get("Counter_Name") == counter and any(s in name for s in subs):
                k = next(s for s in subs if s in name)
                per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    return per


fd, wd, ncalls, outp, note = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
subs = sys.argv[6:]
f, w = total(fd, "FETCH_SIZE", subs), total(wd, "WRITE_SIZE", subs)
kern = {s: {"bytes_per_call": (2 * f.get(s, 0.0) + w.get(s, 0.0)) * 1024 / ncalls} for s in subs}
out = {"kernels": kern, "bytes_per_call": sum(v["bytes_per_call"] for v in kern.values()), "calls": ncalls,
       "note": "FETCH_SIZE x 2 + WRITE_SIZE, KB -> bytes, all dispatches / calls; workload " + note}
srcdigest.stamp(out)
json.dump(out, open(outp, "w"), indent=1)
print(json.dumps(out))
