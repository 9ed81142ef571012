#!/bin/bash
# round-3 library + tests (a2ca982 snapshot under tools/ab/r3tree) vs the current
# tree: the one-pass zstd cases on each.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
(cd tools/ab/r3tree && timeout -k 10 240 python -u -m pytest tests/test_zstd_gpu.py -k "${1:-test_zstd_cases and one_pass}" -q --timeout 200 > "$R/gpurun_out/r3cmp_r3.log" 2>&1)
echo "[r3 tree] exit $?: $(tail -1 gpurun_out/r3cmp_r3.log)"
timeout -k 10 240 python -u -m pytest tests/test_zstd_gpu.py -k "${1:-test_zstd_cases and one_pass}" -q --timeout 200 > gpurun_out/r3cmp_cur.log 2>&1
echo "[current] exit $?: $(tail -1 gpurun_out/r3cmp_cur.log)"
