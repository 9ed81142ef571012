#!/bin/bash
# Round 5: the C4 bench line (defaults: CPU baseline, oracle check) into gpurun_out/final5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final5; mkdir -p $O
timeout -k 10 900 python3 bench.py --config c4 > $O/bench_c4.log 2>&1
rc=$?
echo "[bench_c4] exit $rc: $(grep -v amdgpu.ids $O/bench_c4.log | tail -1 | cut -c1-400)"
exit $rc
