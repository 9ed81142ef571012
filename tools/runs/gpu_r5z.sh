#!/bin/bash
# Round 5: C4 kernel trace and SQ instruction counters at the current encode
# sources (which side kernel to take next).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r5z}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step trace_c4 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu --c4-inflight 1 --no-verify
step sq_c4 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/sq_c4 -o run -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu --c4-inflight 1 --no-verify
echo "r5z done"
