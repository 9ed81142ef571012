#!/bin/bash
# Round 5: the C4 bench line (defaults: CPU baseline, oracle check) and the C5 /
# C2 / C1 lines with their CPU baselines, into gpurun_out/final5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final5; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-300)"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step bench_c4 900 python3 bench.py --config c4
step bench_c5 600 python3 bench.py --config c5
step bench_c2 600 python3 bench.py --config c2
step bench_c1 600 python3 bench.py --config c1
echo "c4line done"
