"""Where the time of a decodes-in-flight bench step goes, from a rocprofv3
kernel trace (run_kernel_trace.csv) of `bench.py --config c3|c5` (chained
pass 3): a window of the kernel timeline (start / end us relative to one tile
pass, queue, kernel) and, over the tile-pass launches after `skip`, the
median tile-pass duration and the median idle gap between one tile pass
ending and the next starting.

usage: python tools/inflight_gaps.py <run_kernel_trace.csv> [skip] [first]"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 8
first = int(sys.argv[3]) if len(sys.argv) > 3 else 14
k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
           for r in rows)
tiles = [x for x in k if "okv_tile_kernel" in x[2]]


def short(n):
    for key, s in (("okv_tile_kernel", "TILE"), ("okv_count_kernel", "COUNT"),
                   ("okv_copy_kernel", "COPY (big blocks)")):
        if key in n:
            return s
    return n[:30]


t0 = tiles[first][0]
for x in k:
    if tiles[first - 1][0] <= x[0] <= tiles[first + 2][1]:
        print(f"  {(x[0] - t0) / 1e3:9.1f} {(x[1] - t0) / 1e3:9.1f}  dur {(x[1] - x[0]) / 1e3:7.1f}"
              f"  queue {x[3]}  {short(x[2])}")
w = tiles[skip:skip + 32]
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(w, w[1:])]
print({"tile_launches": len(w), "tile_us_median": round(st.median((t[1] - t[0]) / 1e3 for t in w), 1),
       "gap_us_median": round(st.median(gaps), 1), "gap_us_min": round(min(gaps), 1)})
