#!/bin/bash
# GPU check run for gpurun: tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=${1:-run}
ok() {  # continue on 0 (pass) or 1 (test failures); stop on crash/timeout
  local rc=$1 name=$2
  echo "[$name] exit $rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name"; exit "$rc"; fi
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; ok $? pytest
tail -5 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; ok $? smoke
tail -3 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py --config c2 --no-cpu > gpurun_out/${TAG}_bench_c2.log 2>&1; ok $? bench_c2
tail -1 gpurun_out/${TAG}_bench_c2.log
timeout -k 10 500 python bench.py --config c3 > gpurun_out/${TAG}_bench_c3.log 2>&1; ok $? bench_c3
tail -1 gpurun_out/${TAG}_bench_c3.log
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_c3" -o c3 --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_prof_c3.log 2>&1; ok $? rocprof
tail -1 gpurun_out/${TAG}_prof_c3.log
find gpurun_out/${TAG}_prof_c3 -name '*stats*' | head
