"""Per-kernel averages of the zstd stage from rocprofv3 kernel-stats CSVs.
usage: python3 tools/zstd_trace_cmp.py <label>=<run_kernel_stats.csv> ..."""
import csv
import sys

rows = {}
for arg in sys.argv[1:]:
    lab, path = arg.split("=", 1)
    for r in csv.DictReader(open(path)):
        if "zstd" in r["Name"]:
            k = r["Name"].split("(")[0].replace("void ", "").replace("okv::", "")
            rows.setdefault(k, {})[lab] = float(r["AverageNs"]) / 1e3
labs = [a.split("=", 1)[0] for a in sys.argv[1:]]
print("kernel (us)".ljust(34) + "".join(lab.rjust(10) for lab in labs))
tot = {lab: 0.0 for lab in labs}
for k, v in sorted(rows.items(), key=lambda kv: -max(kv[1].values())):
    print(k[:34].ljust(34) + "".join(f"{v.get(lab, 0):10.1f}" for lab in labs))
    for lab in labs:
        tot[lab] += v.get(lab, 0)
print("stage sum".ljust(34) + "".join(f"{tot[lab]:10.1f}" for lab in labs))
