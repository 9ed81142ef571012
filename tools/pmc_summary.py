"""Summarise rocprofv3 --pmc passes (tools/pmc_run.sh) into profiles/pmc_<cfg>_<mode>.json.

HBM bytes per launch of a kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of a
16-byte-per-lane streaming read (MI355X_MICROARCH.md §HBM), which this
script re-checks on tools/copybw's known 4 GiB kernels (calibration block).

usage: python tools/pmc_summary.py gpurun_out/pmc_r1 c3 full
"""
import collections
import csv
import json
import os
import sys

src, cfg, mode = sys.argv[1], sys.argv[2], sys.argv[3]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pass_dir):
    agg = collections.defaultdict(list)
    with open(os.path.join(src, pass_dir, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
cal_f, cal_w = load("cal_FETCH"), load("cal_WRITE")
known = 4 << 30
cal = {}
for k in ("copy_blk", "readsum", "copy_gs", "fill"):
    f = cal_f.get((k, "FETCH_SIZE"))
    w = cal_w.get((k, "WRITE_SIZE"))
    cal[k] = {"fetch_KiB": f, "write_KiB": w,
              "fetch_ratio_to_read_bytes": None if f is None else f * 1024 / known,
              "write_ratio_to_written_bytes": None if w is None else w * 1024 / known}
kernels = {}
for (name, c), v in fetch.items():
    wv = write.get((name, "WRITE_SIZE"), 0.0)
    kernels[name] = {"FETCH_SIZE_KiB": v, "WRITE_SIZE_KiB": wv,
                     "hbm_read_bytes": 2 * v * 1024, "hbm_write_bytes": wv * 1024,
                     "hbm_bytes": (2 * v + wv) * 1024}
gather = [k for k in kernels if "okv_gather_kernel" in k]
out = {"config": cfg, "mode": mode, "source": src,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with "
                 "--kernel-trace; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024, the x2 checked on "
                 "4 GiB calibration kernels below",
       "copy_kernel_hbm_bytes_per_launch": kernels[gather[0]]["hbm_bytes"] if gather else None,
       "kernels": kernels, "calibration_4GiB": cal}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
path = os.path.join(ROOT, "profiles", f"pmc_{cfg}_{mode}.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print(path, json.dumps({k: round(v["hbm_bytes"] / 1e9, 3) for k, v in kernels.items()}))
