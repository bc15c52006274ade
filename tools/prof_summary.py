"""Summarise a rocprofv3 --kernel-trace CSV: per (kernel, grid) count / avg / total us."""
import csv, glob, sys, collections
paths = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
rows = []
for p in paths:
    rows += list(csv.DictReader(open(p)))
agg = collections.defaultdict(list)
for r in rows:
    name = r.get("Kernel_Name", "?")[:70]
    grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':70s} {'grid':>9s} {'n':>6s} {'avg_us':>9s} {'tot_ms':>9s} {'%':>6s}")
for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:70s} {g:>9s} {len(v):6d} {sum(v)/len(v):9.2f} {sum(v)/1e3:9.3f} {100*sum(v)/tot:6.1f}")
