#!/bin/bash
# A/B: tile pass value-run stores plain vs non-temporal (ablation build), C3, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out/r3n
OKV_ABLATE=1 timeout -k 10 500 python3 tools/ablate_tile.py 8:16x 8:16xd10 > gpurun_out/r3n/ablate.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r3n/ablate.log | tail -4; exit $rc
