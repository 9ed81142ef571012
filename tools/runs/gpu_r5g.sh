#!/bin/bash
# Round 5: encode with the four-block jump tables (tests, C4 trace + line),
# the point kernel's lean walk (tests, GetRow latency, kernel trace), the
# zstd suite on the product configuration with the exit-line recorder.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step enc_tests 600 $T tests/test_encode_gpu.py -m gpu
step point_tests 300 $T tests/test_point_gpu.py tests/test_reader_gpu.py -m gpu
step getrow 120 tools/getrow_bench 2000
cat $O/getrow.log | grep config
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
step bench_c4 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu
step zstd_ztrace 400 env OKV_ZTRACE=1 $T tests/test_zstd_gpu.py -m gpu
step trace_getrow 200 rocprofv3 --kernel-trace --stats -d $O/trace_getrow -o run -- tools/getrow_bench 300
echo "r5g done"
