"""Summarise the rocprofv3 --pmc passes of tools/pmc_run.sh into JSON.

HBM bytes per launch of a kernel = FETCH_SIZE * k_read + WRITE_SIZE (KiB):
on gfx950 FETCH_SIZE reports half of a 16-byte-per-lane streaming read
(MI355X_MICROARCH.md §HBM).  k_read is measured, not assumed: the 4 GiB
calibration kernels of tools/copybw3 (`cal`) read/write known byte counts,
and k_read = known read bytes / (FETCH_SIZE KiB * 1024) of read_gs.

usage: python tools/pmc_summary.py <gpurun_out/tag> <out.json> [extra json fields]
"""
import collections
import csv
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
extra = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}


def load(pass_dir):
    agg = collections.defaultdict(list)
    with open(os.path.join(src, pass_dir, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
cal_f, cal_w = load("cal_FETCH"), load("cal_WRITE")
known = 4 << 30


def cal_of(kernel_prefix, counter, table):
    for (name, c), (v, _n) in table.items():
        if name.startswith(kernel_prefix) and c == counter:
            return v
    return None


rf = cal_of("read_gs", "FETCH_SIZE", cal_f)
k_read = known / (rf * 1024) if rf else 2.0
cal = {}
for k, rd, wr in (("read_gs", known, 0), ("fill_gs", 0, known), ("copy_gs", known, known),
                  ("copy_dma", known, known)):
    f, w = cal_of(k, "FETCH_SIZE", cal_f), cal_of(k, "WRITE_SIZE", cal_w)
    cal[k] = {"known_read_bytes": rd, "known_write_bytes": wr, "FETCH_SIZE_KiB": f,
              "WRITE_SIZE_KiB": w,
              "read_bytes_est": None if f is None else f * 1024 * k_read,
              "write_bytes_est": None if w is None else w * 1024}
kernels = {}
for (name, c), (v, n) in fetch.items():
    wv = write.get((name, "WRITE_SIZE"), (0.0, 0))[0]
    kernels[name] = {"launches": n, "FETCH_SIZE_KiB": v, "WRITE_SIZE_KiB": wv,
                     "hbm_read_bytes": v * 1024 * k_read, "hbm_write_bytes": wv * 1024,
                     "hbm_bytes": v * 1024 * k_read + wv * 1024}
out = dict(extra)
out.update({"source": src, "k_read": k_read,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with "
                      "--kernel-trace; bytes = FETCH_SIZE*1024*k_read + WRITE_SIZE*1024, k_read "
                      "from the 4 GiB read_gs calibration kernel in the same call",
            "kernels": kernels, "calibration_4GiB": cal})
os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
with open(dst, "w") as f:
    json.dump(out, f, indent=1)
print(dst, f"k_read={k_read:.3f}",
      json.dumps({k: round(v["hbm_bytes"] / 1e9, 4) for k, v in kernels.items()}))
