#!/bin/bash
# Round 5: A/B on one box -- the pack kernel keeping FirstKeys for the meta
# kernel (product) vs the meta kernel reading each block's first line from
# the segment (OKV_ENC_NO_FK=1), ablation build, C4 line, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
for r in 1 2 3; do
  for fk in 0 1; do
    timeout -k 10 300 env OKV_ABLATE=1 OKV_ENC_NO_FK=$fk python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu > $O/nofk${fk}_$r.log 2>&1
    rc=$?
    echo "[nofk=$fk run $r] exit $rc $(grep -o '"device_only_ms_per_step[^}]*}' $O/nofk${fk}_$r.log)"
    [ $rc -ne 0 ] && exit $rc
  done
done
echo "r5m done"
