"""The bench line's evidence attachments (CPU): PMC traffic and kernel-trace
averages attach only from runs of the kernel sources being timed, traffic is
scaled by the launches one step makes, and tools/trace_summary.py groups a
step's launches."""
import csv
import json
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _profiles(tmp_path, monkeypatch, name, payload):
    d = tmp_path / "profiles" / bench.PMC_ROUND
    d.mkdir(parents=True)
    (d / name).write_text(json.dumps(payload))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_sha", lambda paths=bench.DECODE_SOURCES: "sha-now")


def test_pmc_traffic_same_sources_and_launches_per_step(tmp_path, monkeypatch):
    _profiles(tmp_path, monkeypatch, "pmc_c3_full.json", {
        "source_sha": "sha-now", "launches_per_step": {"okv_tile_kernel": 2},
        "kernels": {"void okv::okv_tile_kernel<16384u, 256u, true>": {"hbm_bytes": 100.0},
                    "okv::okv_copy_kernel": {"hbm_bytes": 3.0},
                    "okv::okv_count_kernel": {"hbm_bytes": 50.0}}})
    got, src = bench.pmc_traffic("c3", "full", ("okv_tile_kernel", "okv_copy_kernel"))
    assert got == 203.0 and src.endswith("pmc_c3_full.json")


def test_pmc_traffic_stale_sources(tmp_path, monkeypatch):
    _profiles(tmp_path, monkeypatch, "pmc_c3_full.json",
              {"source_sha": "sha-before", "kernels": {"okv_tile_kernel": {"hbm_bytes": 1.0}}})
    got, src = bench.pmc_traffic("c3", "full", "okv_tile_kernel")
    assert got is None and src.startswith("stale")


def test_trace_roofline_attaches_only_the_timed_sources(tmp_path, monkeypatch):
    _profiles(tmp_path, monkeypatch, "trace_c3.json", {
        "source_sha": "sha-now", "kernel": "okv_tile_kernel", "avg_ns_timed": 1.0e6,
        "timed_launches": 40, "launches_per_step": 1, "bench_event_ms_same_process": 1.01,
        "bench_event_vs_trace": 1.01})
    t = bench.trace_roofline("c3", 4.0e9)
    assert t["avg_ms"] == 1.0 and t["frac"] == round(4.0e9 / 1e-3 / 1e9 / bench.HBM_PEAK_GBS, 4)
    assert t["event_over_trace_same_process"] == 1.01
    monkeypatch.setattr(bench, "source_sha", lambda paths=bench.DECODE_SOURCES: "sha-later")
    assert "stale" in bench.trace_roofline("c3", 4.0e9)


def test_zstd_trace_keyed_on_the_zstd_sources():
    assert "objectkv_amd/csrc/okv_zstd.hip" in bench.ZSTD_SOURCES
    assert set(bench.DECODE_SOURCES) <= set(bench.ZSTD_SOURCES)


def test_trace_summary_sums_launches_per_step(tmp_path):
    rows = []
    t = 0
    for step in range(5):  # 3 kernels per step: 10 + 20 + 30 ns
        for k, dur in (("okv::okv_zstd_a(int)", 10), ("okv::okv_zstd_b(int)", 20),
                       ("okv::okv_zstd_c(int)", 30)):
            rows.append({"Kernel_Name": k, "Start_Timestamp": t, "End_Timestamp": t + dur})
            t += 100
    rows.append({"Kernel_Name": "okv::okv_tile_kernel(x)", "Start_Timestamp": t,
                 "End_Timestamp": t + 999})
    path = tmp_path / "run_kernel_trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    log = tmp_path / "bench.log"
    log.write_text(json.dumps({"metric": "m", "kernel_ms": {"zstd": 6.0e-5, "copy": 1.0}}) + "\n")
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), str(path),
                    "okv_zstd_", "2", "600", str(out), "note", "--per-step", "3", "--sha", "x",
                    "--bench-log", str(log), "--event-key", "zstd"], check=True,
                   capture_output=True)
    d = json.load(open(out))
    assert d["launches"] == 5 and d["timed_launches"] == 3 and d["avg_ns_timed"] == 60
    assert d["launches_per_step"] == 3 and len(d["kernels"]) == 3
    assert d["kernel"].startswith("okv_zstd_*") and d["source_sha"] == "x"
    assert abs(d["bench_event_vs_trace"] - 1.0) < 1e-9
