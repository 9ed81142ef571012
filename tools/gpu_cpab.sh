#!/bin/bash
# C3 tile pass: cache policy of its LDS DMA (product builds with -DOKV_TILE_DMA_CPOL), alternating
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cpab; mkdir -p $O
for r in 1 2 3; do
  for v in 0 2 16 18; do
    timeout -k 10 200 python3 tools/ab_lib.py tools/ab/libokv_cp$v.so cpol_$v > $O/cp${v}_$r.log 2>&1
    rc=$?; echo "[cpol $v run $r] exit $rc $(grep '^{' $O/cp${v}_$r.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
