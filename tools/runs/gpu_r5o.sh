#!/bin/bash
# Round 5: encode tests with the FirstKey chunks from the pack kernel's store
# loop, then the FirstKey A/B (tools/gpu_r5m.sh) and a C4 trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5o; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-400 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step enc_tests 600 $T tests/test_encode_gpu.py tests/test_snapshot_gpu.py -m gpu
tools/gpu_r5m.sh || exit 1
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1
echo "r5o done"
