#!/bin/bash
# One iteration on the GPU box: GPU test suite, then A/B arms of the tile pass
# (tools/ablate_tile.py, ablation build), the product C3 bench, the tile phase
# probe.  Every step has its own time limit; the first failure ends the script.
#   tools/gpu_iter.sh <tag> [ablate arms...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
TAG=${1:-iter}
shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc"
  tail -4 "$OUT/$name.log" | cut -c1-600
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[ $# -gt 0 ] && step ablate 400 python3 tools/ablate_tile.py "$@"
step bench_c3 300 python3 bench.py --config c3 --no-cpu
step bench_c3_one 300 python3 bench.py --config c3 --no-cpu --no-verify --decode-inflight 1
step tile_probe 200 python3 tools/tile_probe.py 16xd7
echo iter done
