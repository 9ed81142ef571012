#!/bin/bash
# rocprofv3 kernel trace + stats of the C4 encode bench (run under gpurun).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${1:-c4}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o c4 --output-format csv -- python3 "$R/bench.py" --config c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_prof.log 2>&1
echo "rocprof exit $?"
tail -1 gpurun_out/${TAG}_prof.log
find gpurun_out/${TAG}_prof -name '*stats*'
