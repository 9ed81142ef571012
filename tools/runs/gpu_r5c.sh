#!/bin/bash
# Round 5: the one-launch per-block decode (OKV_VALUE_SWEEP=9 / 10) -- parity
# on the edge shapes, then timed against the tile pass on C3 (one process,
# outputs compared bit for bit between arms, the first arm vs the oracle).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
OKV_ABLATE=1 timeout -k 10 300 python3 tools/ablate_check.py enc_arms > $O/enc_arms.log 2>&1
rc=$?; tail -9 $O/enc_arms.log; [ $rc -ne 0 ] && exit $rc
for a in block block512; do
  OKV_ABLATE=1 timeout -k 10 300 python3 tools/ablate_check.py $a > $O/check_$a.log 2>&1
  rc=$?; tail -2 $O/check_$a.log; [ $rc -ne 0 ] && exit $rc
done
OKV_ABLATE=1 ABL_VERIFY=1 ABL_ROUNDS=5 timeout -k 10 400 python3 tools/ablate_tile.py 8:16x 9 10 11 > $O/block_ab.log 2>&1
rc=$?; tail -8 $O/block_ab.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r5a.sh
