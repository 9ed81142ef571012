#!/bin/bash
# CM bench kernel trace (per-kernel time of the decode / merge / encode stages)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/trace_cm; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv \
  -- python3 "$R/bench.py" --config cm --steps 5 --warmup 1 --no-cpu > $O/bench.log 2>&1
rc=$?
f=$(find $O/tr -name run_kernel_stats.csv | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv
exit $rc
