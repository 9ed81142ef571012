#!/bin/bash
# decodes in flight: C3 and CZ lines at 1..4 (alternating, one box)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/inflight; mkdir -p $O
for r in 1 2; do
for cfg in c3 cz; do
for n in 2 3 4; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu --no-verify --steps 20 --warmup 5 --decode-inflight $n > $O/${cfg}_$n_$r.log 2>&1
  rc=$?; echo "[$cfg inflight $n run $r] exit $rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"latency_ms_per_step": [0-9.]*' $O/${cfg}_$n_$r.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done; done; done
exit 0
