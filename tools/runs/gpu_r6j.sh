#!/bin/bash
# Round 6: kernel traces of the decodes-in-flight bench (C5, C3, chained pass 3)
# for tools/inflight_gaps.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6j}; mkdir -p $O
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc: $(grep -v amdgpu.ids "$O/$n.log" | tail -1 | cut -c1-250 | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step trace_c5_if 300 rocprofv3 --kernel-trace -d $O/trace_c5_if -o run --output-format csv -- python3 bench.py --config c5 --steps 40 --warmup 5 --no-cpu --no-verify
step trace_c3_if 300 rocprofv3 --kernel-trace -d $O/trace_c3_if -o run --output-format csv -- python3 bench.py --config c3 --steps 20 --warmup 5 --no-cpu --no-verify
echo "r6j done"
