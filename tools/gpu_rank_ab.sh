#!/bin/bash
# merge rank kernel: window staging with every load in flight (libokv_rank) vs per-stream loop (head)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_snapshot_gpu.py tests/test_encode_gpu.py" "--config cm --no-cpu --steps 10 --warmup 2" 3 \
  tools/ab/libokv_rank.so tools/ab/libokv_head.so
