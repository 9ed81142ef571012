#!/bin/bash
# Round 5, first call: (1) A/B of the count kernel's arrival (release/acquire vs
# drained sc1 + relaxed add), alternating processes; (2) 64 KiB / 1024- and
# 512-thread tile forms vs the 16 KiB product form in one process (ablation
# build, outputs compared bit-for-bit between arms).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5a; mkdir -p $O
for r in 1 2 3; do
  for L in release relaxed; do
    timeout -k 10 240 python3 tools/ab_lib.py tools/ab/r5/lib_$L.so $L >> $O/ab_count.log 2>$O/ab_err.log || exit $?
    tail -1 $O/ab_count.log
  done
done
OKV_ABLATE=1 ABL_ROUNDS=5 timeout -k 10 400 python3 tools/ablate_tile.py 8:16x 8:64xw1024 8:64xw512 8:32xw512 > $O/tile64.log 2>&1
rc=$?; tail -20 $O/tile64.log; exit $rc
