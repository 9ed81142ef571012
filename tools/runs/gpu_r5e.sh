#!/bin/bash
# Round 5: point path with LDS-DMA staging (tests + C++ GetRow latency), the
# C4 kernel trace (tile cut timing), the C3 line with the relaxed arrival.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step point_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_point_gpu.py tests/test_reader_gpu.py -m gpu
step getrow 120 tools/getrow_bench 2000
cat $O/getrow.log
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
step bench_c3 300 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu
echo "r5e done"
