#!/bin/bash
# Round 6: zstd stage phase counters (ablation build, OKV_ZSTD_PROF) on CZ.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${AB_TAG:-r6t}; mkdir -p $O
timeout -k 10 300 python3 tools/zstd_prof.py 16384 > $O/zstd_prof.log 2>&1
rc=$?; echo "[zstd_prof] exit $rc"; tail -8 $O/zstd_prof.log; exit $rc
