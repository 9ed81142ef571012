#!/bin/bash
# C3 kernel trace with the bench's default four decodes in flight: gaps between
# consecutive tile-pass launches and the count kernels' overlap with them.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/trace_c3if; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv \
  -- python3 "$R/bench.py" --config c3 --steps 20 --warmup 5 --no-cpu --no-verify > $O/bench.log 2>&1
rc=$?
f=$(find $O/tr -name run_kernel_trace.csv | head -1); [ -n "$f" ] && cp "$f" $O/kernel_trace.csv
exit $rc
