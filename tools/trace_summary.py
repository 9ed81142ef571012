"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into the
bench's untimed launches (guard + warmup) and its timed steps, plus the
roofline fraction the timed average implies.

usage: python tools/trace_summary.py <run_kernel_trace.csv> <kernel substring>
           <untimed launches> <algorithmic bytes per launch> <out.json> [note]
           [--sha <decode source sha>] [--bench-log <the traced bench's stdout/stderr>]
           [--per-step K] [--event-key copy|zstd]

--per-step K: the kernel runs K launches per step (a two-piece decode launches
the tile pass twice): consecutive launches are summed in groups of K, and
every count below (launches, untimed launches) is in steps.

--event-key: which of the bench line's kernel_ms to compare with (default
copy, pass 3; zstd: the zstd stage, whose kernels --per-step sums per decode).

--sha lets bench.py attach the trace to its roofline only while the kernel
sources are the traced ones; --bench-log records the bench's own HIP-event
time for the same kernel in the traced process (kernel_ms.copy of its JSON
line), so event and trace timings are compared on one box and one process.
"""
import csv
import json
import sys

argv = sys.argv[1:]
opts = {}
for flag in ("--sha", "--bench-log", "--per-step", "--event-key"):
    if flag in argv:
        i = argv.index(flag)
        opts[flag] = argv[i + 1]
        del argv[i:i + 2]
path, kern, skip, alg, out = argv[0], argv[1], int(argv[2]), int(argv[3]), argv[4]
note = argv[5] if len(argv) > 5 else ""
rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
K = int(opts.get("--per-step", "1"))
if K > 1:  # per step: the K launches of one decode, summed
    ns = [sum(ns[i:i + K]) for i in range(0, len(ns) - len(ns) % K, K)]
timed = ns[skip:]
avg = sum(timed) / len(timed)
names = sorted({r["Kernel_Name"].split("(")[0] for r in rows})
label = names[0] if len(names) == 1 else f"{kern}* ({len(names)} kernels summed per step)"
res = {"kernel": label if rows else kern, "kernels": names, "source": path,
       "launches": len(ns), "untimed_launches": skip, "timed_launches": len(timed),
       "avg_ns_timed": avg, "min_ns_timed": min(timed), "max_ns_timed": max(timed),
       "avg_ns_all": sum(ns) / len(ns), "per_launch_ns": ns,
       "algorithmic_bytes_per_launch": alg, "achieved_GB_s": alg / avg,
       "frac_of_8TB_s": alg / avg / 8000.0, "note": note}
res["launches_per_step"] = K
if "--sha" in opts:
    res["source_sha"] = opts["--sha"]
if "--bench-log" in opts:
    line = None
    for ln in open(opts["--bench-log"], errors="replace"):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    if line:
        res["bench_event_ms_same_process"] = line.get("kernel_ms", {}).get(
            opts.get("--event-key", "copy"))
        res["bench_event_vs_trace"] = (res["bench_event_ms_same_process"] * 1e6 / avg
                                       if res["bench_event_ms_same_process"] else None)
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(out, json.dumps({k: res[k] for k in ("kernel", "timed_launches", "avg_ns_timed",
                                           "achieved_GB_s", "frac_of_8TB_s")}))
