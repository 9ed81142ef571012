#!/bin/bash
# Round 5: GetRow through okv_point_get (one row back) with the run-length
# speculated walk -- tests, C++ latency (fixed and Zipf rows), phases; then
# the FirstKey A/B of the encode (tools/gpu_r5m.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step point_tests 300 $T tests/test_point_gpu.py tests/test_reader_gpu.py -m gpu
step getrow 120 tools/getrow_bench 2000
step getrow_phases 120 tools/getrow_bench_ablate 500
grep config $O/getrow.log $O/getrow_phases.log
tools/gpu_r5m.sh
