#!/bin/bash
# GPU test suite, then an A/B of library builds (tools/ab_lib.py, one process
# per run, alternating A B A B ...), then the product C3 bench one at a time
# and the tile phase probe.  Each step has its own time limit; the first
# failure ends the script.
#   tools/gpu_ab.sh <tag> <libA.so> <libB.so> [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; N=${4:-2}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc"
  tail -3 "$OUT/$name.log" | cut -c1-600
  [ $rc -ne 0 ] && exit $rc
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
for i in $(seq 1 "$N"); do
  step "ab_A_$i" 200 python3 tools/ab_lib.py "$A" A
  step "ab_B_$i" 200 python3 tools/ab_lib.py "$B" B
done
step bench_c3_one 300 python3 bench.py --config c3 --no-cpu --no-verify --decode-inflight 1
step bench_c3 300 python3 bench.py --config c3 --no-cpu --no-verify
step tile_probe 200 python3 tools/tile_probe.py 16xd7
echo ab done
