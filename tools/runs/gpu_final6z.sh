#!/bin/bash
# End-of-round-6 evidence after the zstd-only changes (okv_zstd.hip): the GPU
# suite and smoke as the driver runs them, the CZ kernel trace (summarised as
# in gpu_final6.sh part b) and the CZ bench line.  Copied into profiles/r6 by
# tools/runs/collect_r6.sh <tag>.
#   tools/runs/gpu_final6z.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r6finz}
O="$R/gpurun_out/$T"
mkdir -p "$O"
step() {
  local n=$1 s=$2
  shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc"
  grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
ZSHA=$(python3 -c "import bench; print(bench.source_sha(bench.ZSTD_SOURCES))")
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step trace_cz 300 rocprofv3 --kernel-trace --stats -d "$O/trace_cz" -o run --output-format csv \
  -- python3 "$R/bench.py" --config cz --steps 10 --warmup 2 --no-cpu --no-verify --decode-inflight 1
CSV=$(find "$O/trace_cz" -name 'run_kernel_trace.csv' | head -1)
ALG=$(python3 -c "import json; l=[json.loads(x) for x in open('$O/trace_cz.log') if x.startswith('{')][-1]; print(l['roofline']['algorithmic_bytes_per_launch'])")
step trace_cz_sum 60 python3 tools/trace_summary.py "$CSV" okv_zstd_ 4 "$ALG" "$O/trace_cz.json" \
  "CZ one decode at a time (bench.py --decode-inflight 1, 10 steps + 2 warmup + guard + plan); the zstd stage's 9 kernels summed per decode" \
  --sha "$ZSHA" --bench-log "$O/trace_cz.log" --per-step 9 --event-key zstd
step bench_cz 600 python3 bench.py --config cz
echo "final6z done"
