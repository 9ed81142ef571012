#!/bin/bash
# The whole GPU suite (as the driver runs it) and smoke(), each under its own limit.
#   tools/gpu_full.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
T=${1:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "passed|failed" gpurun_out/${T}_pytest.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?
echo "smoke exit $rc"; tail -3 gpurun_out/${T}_smoke.log
exit $rc
