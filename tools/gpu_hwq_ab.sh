#!/bin/bash
# C3 four decodes in flight: HIP's default hardware queues (4) vs 8
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/hwq; mkdir -p $O
for r in 1 2 3; do
  for q in def 8; do
    if [ $q = def ]; then
      timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 40 --warmup 5 > $O/${q}_$r.log 2>&1
    else
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-verify --steps 40 --warmup 5 > $O/${q}_$r.log 2>&1
    fi
    rc=$?; echo "[$q run $r] exit $rc $(grep -o '"ms_per_step": [0-9.]*\|"latency_ms_per_step": [0-9.]*' $O/${q}_$r.log | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
