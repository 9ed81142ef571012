#!/bin/bash
# Round 5: encode with the doubling over 4-tile chunks (tests, C4 trace,
# line, HBM traffic passes).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5j; mkdir -p $O
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
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
step bench_c4 300 python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu
step pmc_c4 900 tools/pmc_run.sh r5j/pmc_c4 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
echo "r5j done"
