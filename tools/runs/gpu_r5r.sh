#!/bin/bash
# Round 5: C4 evidence at the final encode sources (tests, PMC passes, line,
# kernel trace) into gpurun_out/final5 (tools/collect_r5.sh copies it).
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
step enc_tests 600 python -u -m pytest tests/test_encode_gpu.py tests/test_snapshot_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step pmc_c4 600 "$R/tools/pmc_run.sh" "$T/pmc_c4" bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-verify --c4-inflight 1
step pmc_c4_sum 60 python3 tools/pmc_summary.py "$O/pmc_c4" "$O/pmc_c4_encode.json" "{\"source_sha\": \"$ESHA\", \"config\": \"c4\", \"mode\": \"encode\", \"source\": \"gpurun_out/$T/pmc_c4\"}"
mkdir -p profiles/r5 && cp "$O/pmc_c4_encode.json" profiles/r5/
step bench_c4 600 python3 bench.py --config c4
step trace_c4_enc 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4_enc -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-verify --c4-inflight 1
echo "r5r done"
