#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_snapshot_gpu.py > gpurun_out/t_snap.log 2>&1 || exit 1
for st in 1 0; do
  OKV_MERGE_STAGE=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cm_tr$st -o run --output-format csv -- python3 bench.py --config cm --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/cm_tr$st.log 2>&1 || exit 1
done
