#!/bin/bash
# quick check: selected GPU tests, then named tools/bench commands, each step bounded
#   tools/gpu_quick.sh <tag> "<pytest files>" ["cmd1" "cmd2" ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
T=$1; F=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
if [ -n "$F" ]; then
  timeout -k 10 600 python -u -m pytest $F -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "[tests] exit $rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
fi
i=0
for c in "$@"; do
  i=$((i+1))
  timeout -k 10 400 bash -c "$c" > $O/cmd$i.log 2>&1
  rc=$?; echo "[cmd$i: $c] exit $rc"; grep -v amdgpu.ids $O/cmd$i.log | grep -v "copy_(torch" | tail -3 | cut -c1-500; [ $rc -ne 0 ] && exit $rc
done
exit 0
