"""SQ / TCC counters per kernel from rocprofv3 --pmc passes (counter_collection.csv).
Median per dispatch of every counter found, for each kernel substring given.
Args: out.json dir [dir ...] -- ksub [ksub ...]"""
import csv, glob, json, sys
import numpy as np

args = sys.argv[1:]
out_path, rest = args[0], args[1:]
cut = rest.index("--")
dirs, ksubs = rest[:cut], rest[cut + 1:]
res = {}
for k in ksubs:
    per = {}
    for d in dirs:
        for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(p)):
                if k not in r.get("Kernel_Name", ""):
                    continue
                key = (p, r.get("Dispatch_Id", r.get("Correlation_Id")))
                c = r.get("Counter_Name")
                per.setdefault(c, {}).setdefault(key, 0.0)
                per[c][key] += float(r["Counter_Value"])
    res[k] = {c: {"median_per_dispatch": float(np.median(list(v.values()))), "dispatches": len(v)}
              for c, v in sorted(per.items())}
    durs = []  # the same dispatches' durations (the --kernel-trace of the same passes), us
    for d in dirs:
        for p in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(p)):
                if k in r.get("Kernel_Name", ""):
                    durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if durs:
        res[k]["duration_us"] = {"median_per_dispatch": float(np.median(durs)), "dispatches": len(durs)}
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import srcdigest  # noqa: E402
res["_meta"] = srcdigest.stamp({"dirs": dirs})
json.dump(res, open(out_path, "w"), indent=1)
for k, v in res.items():
    if k == "_meta":
        continue
    print(k, {c: round(x["median_per_dispatch"], 1) for c, x in v.items()})
