#!/bin/bash
# GetRow latency, bimodal block sizes, then the 2-rank one-GPU rehearsals.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p profiles/r4 gpurun_out
timeout -k 10 300 python3 tools/getrow_latency.py > profiles/r4/getrow_latency.log 2>&1; rc=$?
echo "[getrow] exit $rc: $(tail -1 profiles/r4/getrow_latency.log | cut -c1-400)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/mixed_blocks.py > profiles/r4/mixed_blocks.log 2>&1; rc=$?
echo "[mixed] exit $rc"; tail -3 profiles/r4/mixed_blocks.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
./tools/gpu_rehearse.sh r4
