#!/bin/bash
# rocprofv3 evidence for a bench config (run on the GPU box via gpurun):
#   1. kernel trace + stats of `bench.py --config <cfg>` (per-kernel durations)
#   2. FETCH_SIZE and WRITE_SIZE PMC passes of the same command (tools/pmc_run.sh)
# Every step has its own time limit; a failure ends the script.
#   tools/gpu_profile.sh <tag> <cfg> [extra bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1
CFG=$2
shift 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --config "$CFG" --steps 20 --warmup 5 --no-cpu --no-verify "$@" \
  > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log" | cut -c1-300
"$R/tools/pmc_run.sh" "$TAG/pmc" bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu \
  --no-verify "$@" || exit 1
find "$OUT" -name '*stats.csv' -o -name '*counter_collection.csv' | head -20
