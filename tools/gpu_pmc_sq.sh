#!/bin/bash
# SQ wave-state / L2 counter passes (tools/pmc_diag.sh) over the CM and CZ
# benches: where the small-block gather and the zstd sequence stage spend
# their cycles.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 ./tools/pmc_diag.sh pmc_cm python3 "$R/bench.py" --config cm --steps 2 --warmup 1 --no-cpu --no-verify \
  && timeout -k 10 600 ./tools/pmc_diag.sh pmc_cz python3 "$R/bench.py" --config cz --steps 3 --warmup 1 --no-cpu --no-verify --decode-inflight 1
rc=$?
for t in pmc_cm pmc_cz; do python3 tools/pmc_diag_summary.py gpurun_out/$t gather_small count_kernel zstd_seq zstd_exec > gpurun_out/$t/summary.txt 2>&1; done
exit $rc
