#!/bin/bash
# End of round 5, final sources: the GPU suite and smoke as the driver runs
# them, the C4 PMC passes and line (encode sources changed after part a), the
# driver's bench command once more.  Into gpurun_out/final5 (collect_r5.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=final5; O=gpurun_out/$T; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
ESHA=$(python3 -c "import bench; print(bench.source_sha(bench.ENCODE_SOURCES))")
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-verify --c4-inflight 1
step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
mkdir -p profiles/r5 && cp "$O/pmc_c4_encode.json" profiles/r5/
step bench_c4 600 python3 bench.py --config c4
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1 --no-verify
step bench_cm 600 python3 bench.py --config cm
step bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
echo "final5c done"
