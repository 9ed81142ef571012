"""Per-kernel summary of a rocprofv3 rocpd database (run_results.db):
calls, average and total duration, by kernel name.
  python3 tools/rocpd_summary.py <db> [name-substring ...]"""
import sqlite3
import sys

db = sys.argv[1]
pats = sys.argv[2:]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6, "
                 "min(end-start)/1000.0, max(end-start)/1000.0 from kernels group by name "
                 "order by 4 desc").fetchall()
print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'total_ms':>9s}")
for name, n, avg, tot, mn, mx in rows:
    if pats and not any(p in name for p in pats):
        continue
    print(f"{name[:70]:70s} {n:6d} {avg:10.2f} {mn:9.2f} {mx:9.2f} {tot:9.3f}")
