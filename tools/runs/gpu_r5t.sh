#!/bin/bash
# Round 5: tools/gpu_r5s.sh (wave count walk: tests + CM A/B) then
# tools/gpu_r5r.sh (C4 evidence at the final encode sources).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
tools/gpu_r5s.sh && tools/gpu_r5r.sh
