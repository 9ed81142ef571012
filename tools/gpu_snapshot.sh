#!/bin/bash
# Measurement snapshot at HEAD (run on the GPU box via gpurun):
#   1. C3 kernel trace, one decode at a time (per-kernel durations)
#   2. okv_tile_kernel phase probe (ablation build, product form + timestamps)
#   3. bench lines for C4 / CZ / CM / C5 (no CPU leg)
#   4. C4 encode trace + FETCH/WRITE PMC passes
# Every GPU step has its own time limit; the first failure ends the script.
#   tools/gpu_snapshot.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=${1:-snap}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {  # step <name> <seconds> <cmd...>: run, log, stop the script on failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc"
  tail -2 "$OUT/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step c3_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/c3_trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --no-cpu --no-verify --decode-inflight 1
step tile_probe 200 python3 tools/tile_probe.py 16xd7
for c in c4 cz cm c5; do
  step "bench_$c" 300 python3 bench.py --config $c --no-cpu
done
"$R/tools/gpu_profile.sh" "$TAG/c4prof" c4 --c4-inflight 1 || exit 1
echo snapshot done
