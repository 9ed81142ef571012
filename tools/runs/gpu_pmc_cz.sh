#!/bin/bash
# Round 6: HBM traffic of the zstd stage (CZ, one decode at a time):
# FETCH_SIZE / WRITE_SIZE passes + calibration (tools/pmc_run.sh), summarised
# per kernel into profiles/r6/pmc_cz_full.json keyed on the zstd sources; then
# the CZ line again (it attaches the summed okv_zstd_* bytes as traffic).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r6pmcz}; O="$R/gpurun_out/$T"; mkdir -p "$O"
ZSHA=$(python3 -c "import bench; print(bench.source_sha(bench.ZSTD_SOURCES))")
timeout -k 10 900 "$R/tools/pmc_run.sh" "$T/pmc_cz" bench.py --config cz --steps 3 --warmup 1 --no-cpu --no-verify --decode-inflight 1 > "$O/pmc_cz.log" 2>&1
rc=$?; echo "[pmc_cz] exit $rc"; tail -3 "$O/pmc_cz.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 tools/pmc_summary.py "$O/pmc_cz" "$O/pmc_cz_full.json" "{\"source_sha\": \"$ZSHA\", \"config\": \"cz\", \"mode\": \"full\", \"source\": \"gpurun_out/$T/pmc_cz\", \"launches_per_step\": {}}" > "$O/pmc_cz_sum.log" 2>&1
rc=$?; echo "[pmc_cz_sum] exit $rc"; tail -5 "$O/pmc_cz_sum.log"; [ $rc -ne 0 ] && exit $rc
mkdir -p profiles/r6 && cp "$O/pmc_cz_full.json" profiles/r6/
timeout -k 10 600 python3 bench.py --config cz > "$O/bench_cz.log" 2>&1
rc=$?; echo "[bench_cz] exit $rc"; tail -1 "$O/bench_cz.log" | cut -c1-300; exit $rc
