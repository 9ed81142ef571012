#!/bin/bash
# zstd error-line trace (ablation build prints every corrupt-input exit's line)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
OKV_ABLATE=1 timeout -k 10 240 python -u -m pytest tests/test_zstd_gpu.py \
  -k "${1:-test_zstd_cases and one_pass and (text_l1 or zeros)}" -s -q --timeout 200 > gpurun_out/ztrace.log 2>&1
rc=$?
echo "pytest exit $rc"
grep "zstd err" gpurun_out/ztrace.log | sort | uniq -c | sort -rn | head
tail -3 gpurun_out/ztrace.log
