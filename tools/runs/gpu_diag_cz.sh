#!/bin/bash
# Round 6: diagnostic counters of the zstd stage (CZ, one decode at a time):
# tools/pmc_diag.sh's four passes (wave states, L2 hit rate and miss latency,
# DRAM share of the L2 misses, TA stalls), summarised per okv_zstd_* kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r6dgcz}; O="$R/gpurun_out/$T"; mkdir -p "$O"
timeout -k 10 900 "$R/tools/pmc_diag.sh" "$T/diag" python3 bench.py --config cz --steps 3 --warmup 1 --no-cpu --no-verify --decode-inflight 1 > "$O/diag.log" 2>&1
rc=$?; echo "[diag] exit $rc"; tail -5 "$O/diag.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/pmc_diag_summary.py "$O/diag" okv_zstd > "$O/diag_sum.log" 2>&1
rc=$?; echo "[diag_sum] exit $rc"; exit $rc
