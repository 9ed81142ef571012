#!/bin/bash
# CM decode stage: count-kernel prefetch off / on (ablation build, OKV_COUNT_PREFETCH)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-cmpf}; mkdir -p $O
for r in 1 2; do
for pf in 0 1; do
  OKV_ABLATE=1 OKV_COUNT_PREFETCH=$pf timeout -k 10 300 python3 bench.py --config cm --no-cpu --steps 10 --warmup 2 > $O/pf_${pf}_$r.log 2>&1
  rc=$?; echo "[prefetch $pf run $r] exit $rc $(grep -o '"stage_ms": {[^}]*}\|"frac": [0-9.]*' $O/pf_${pf}_$r.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
