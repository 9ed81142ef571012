#!/bin/bash
# End-of-round-6 GPU suite and smoke at the final sources (as the driver runs
# them).  tools/runs/gpu_final6s.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=${1:-r6fins}; O="$R/gpurun_out/$T"; mkdir -p "$O"
step() {
  local n=$1 s=$2; shift 2
  timeout -k 10 "$s" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "[$n] exit $rc"; grep -v amdgpu.ids "$O/$n.log" | tail -2 | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
echo "final6s done"
