"""Summarise tools/pmc_diag.sh passes: per kernel (name prefix), the mean of
each counter over its launches, plus derived figures (wave-state shares,
average L2-miss queue level / requests = latency in L2 cycles).

usage: python tools/pmc_diag_summary.py <gpurun_out/tag> [kernel-substring ...]
"""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
pats = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].replace("void ", "")
            if pats and not any(p in name for p in pats):
                continue
            key = (name[:90], r.get("Grid_Size", ""))
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"== {key[0]}  grid={key[1]}  launches={max(len(v) for v in cs.values())}")
    for c in sorted(m):
        print(f"   {c:36s} {m[c]:16.4g}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_VMEM"):
            if c in m:
                print(f"   {c + ' / WAVE_CYCLES':36s} {m[c] / wc:16.3f}")
    if m.get("TCC_EA0_RDREQ_sum"):
        print(f"   {'RDREQ_LEVEL / RDREQ (cycles)':36s} "
              f"{m['TCC_EA0_RDREQ_LEVEL_sum'] / m['TCC_EA0_RDREQ_sum']:16.1f}")
        if "TCC_HIT_sum" in m:
            print(f"   {'L2 hit rate':36s} "
                  f"{m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):16.3f}")
    if m.get("TCC_EA0_WRREQ_sum"):
        print(f"   {'WRREQ_LEVEL / WRREQ (cycles)':36s} "
              f"{m['TCC_EA0_WRREQ_LEVEL_sum'] / m['TCC_EA0_WRREQ_sum']:16.1f}")
