#!/bin/bash
# CM decode stage vs the small-block gather's grid (ablation build, OKV_GATHER_GRID)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-cmgrid}; mkdir -p $O
for g in 0 2048 4096 8192 16384 32768; do
  if [ $g = 0 ]; then E="OKV_ABLATE=1"; else E="OKV_ABLATE=1 OKV_GATHER_GRID=$g"; fi
  env $E timeout -k 10 300 python3 bench.py --config cm --no-cpu --steps 10 --warmup 2 > $O/grid_$g.log 2>&1
  rc=$?; echo "[grid $g] exit $rc $(grep -o '"stage_ms": {[^}]*}\|"frac": [0-9.]*' $O/grid_$g.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cm" -o run --output-format csv \
  -- python3 "$R/bench.py" --config cm --steps 5 --warmup 1 --no-cpu --no-verify > $O/trace_cm.log 2>&1
rc=$?; echo "[trace cm] exit $rc"; [ $rc -ne 0 ] && exit $rc
exit 0
