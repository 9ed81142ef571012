"""Per-arm HBM traffic of the tile-pass ablation arms (tools/ablate_tile.py run
under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE [/ EA request counters], one pass
each) with the output-class bytes the script prints (ABL_CLASSES=1).

usage: python tools/pmc_arms_summary.py <gpurun_out/tag> <out.json>
FETCH_SIZE is doubled (gfx950 reports half of a 16-B-per-lane streaming read,
MI355X_MICROARCH.md; the 4 GiB calibration kernels in the same call confirm
k_read = 2.000 when present).  Median over each kernel's launches."""
import collections
import csv
import glob
import json
import os
import re
import sys

src, dst = sys.argv[1], sys.argv[2]


def load(d):
    agg = collections.defaultdict(list)
    fs = glob.glob(os.path.join(src, d, "**", "run_counter_collection.csv"), recursive=True)
    if not fs:
        return agg
    for r in csv.DictReader(open(fs[0])):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def med(x):
    return sorted(x)[len(x) // 2] if x else None


F, W = load("pmc_FETCH_SIZE"), load("pmc_WRITE_SIZE")
EA = load("pmc_TCC_EA0_WRREQ_sum")
classes = None
for lf in glob.glob(os.path.join(src, "*.log")):
    for line in open(lf, errors="replace"):
        if line.startswith("classes "):
            classes = {k: int(v) for k, v in re.findall(r"(\w+)~?=(\d+)", line)}
arms = {}
for (n, c), v in W.items():
    if "tile_kernel" not in n or c != "WRITE_SIZE":
        continue
    e = {k.replace("TCC_EA0_", "").replace("_sum", ""): med(EA.get((n, k), []))
         for k in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_RDREQ_sum",
                   "TCC_EA0_RDREQ_128B_sum")}
    arms[n] = {"launches": len(v), "write_bytes": med(v) * 1024,
               "read_bytes": med(F.get((n, "FETCH_SIZE"), [0])) * 1024 * 2,
               **({"ea_requests": e} if any(e.values()) else {})}
out = {"source": src, "classes": classes, "arms": arms,
       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/ablate_tile.py "
                 "(every arm in one process, 2 steps per arm); bytes per launch, median"}
if classes:
    alg_w = classes["soa"] + classes["blocks"] + classes["keys"] + classes["vals"]
    out["algorithmic_write_bytes"] = alg_w
    for a in arms.values():
        a["write_vs_algorithmic"] = round(a["write_bytes"] / alg_w, 4)
os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
json.dump(out, open(dst, "w"), indent=1)
for n, a in sorted(arms.items()):
    print(f"{n[-48:]:48s} write {a['write_bytes'] / 1e9:.4f} GB  read {a['read_bytes'] / 1e9:.4f} GB")
