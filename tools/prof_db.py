"""Summarise a rocprofv3 SQLite (rocpd) result: per kernel count / avg / total us.
usage: python tools/prof_db.py results.db [name-filter]"""
import collections, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
views = [r[0] for r in c.execute("select name from sqlite_master where type='view'")]
q = ("select s.kernel_name, d.grid_size_x, d.start, d.end from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
try:
    rows = list(c.execute(q))
except sqlite3.OperationalError:
    rows = list(c.execute("select name, grid_size_x, start, end from kernels"))
agg = collections.defaultdict(list)
for name, gx, t0, t1 in rows:
    if flt in name:
        agg[(name[:80], gx)].append((t1 - t0) / 1000.0)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':80s} {'grid_x':>8s} {'n':>6s} {'avg_us':>10s} {'tot_ms':>9s} {'%':>6s}")
for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:80s} {g:>8} {len(v):6d} {sum(v)/len(v):10.2f} {sum(v)/1e3:9.3f} {100*sum(v)/tot:6.1f}")
