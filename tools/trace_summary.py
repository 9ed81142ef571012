"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into the
bench's untimed launches (guard + warmup) and its timed steps, plus the
roofline fraction the timed average implies.

usage: python tools/trace_summary.py <run_kernel_trace.csv> <kernel substring>
           <untimed launches> <algorithmic bytes per launch> <out.json> [note]
"""
import csv
import json
import sys

path, kern, skip, alg, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), \
    sys.argv[5]
note = sys.argv[6] if len(sys.argv) > 6 else ""
rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
timed = ns[skip:]
avg = sum(timed) / len(timed)
res = {"kernel": rows[0]["Kernel_Name"].split("(")[0] if rows else kern, "source": path,
       "launches": len(ns), "untimed_launches": skip, "timed_launches": len(timed),
       "avg_ns_timed": avg, "min_ns_timed": min(timed), "max_ns_timed": max(timed),
       "avg_ns_all": sum(ns) / len(ns), "per_launch_ns": ns,
       "algorithmic_bytes_per_launch": alg, "achieved_GB_s": alg / avg,
       "frac_of_8TB_s": alg / avg / 8000.0, "note": note}
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(out, json.dumps({k: res[k] for k in ("kernel", "timed_launches", "avg_ns_timed",
                                           "achieved_GB_s", "frac_of_8TB_s")}))
