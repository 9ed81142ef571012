#!/bin/bash
# Round 5: C4 whole-segment throughput against the number of segments in flight.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5inf; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -o '"ms_per_step": [0-9.]*' "$O/$n.log") $(grep -o '"latency_ms_per_segment": [0-9.]*' "$O/$n.log") $(grep -o '"device_only_ms_per_step": [0-9.]*' "$O/$n.log")"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for r in 1 2; do
  for k in 2 3 4; do
    step c4_inf${k}_$r 300 python3 bench.py --config c4 --steps 20 --warmup 3 --no-cpu --no-verify --c4-inflight $k
  done
done
echo "r5inf done"
