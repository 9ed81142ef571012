#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/zdebug.py "$@" > gpurun_out/zdebug.log 2>&1
rc=$?; echo "exit $rc"; grep -v amdgpu.ids gpurun_out/zdebug.log | tail -20; exit $rc
