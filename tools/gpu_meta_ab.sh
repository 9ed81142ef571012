#!/bin/bash
# encode meta entries: FirstKey from the written segment (libokv_meta) vs through the row arrays (head)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_encode_gpu.py tests/test_snapshot_gpu.py tests/test_full_size_gpu.py" "--config c4 --no-cpu --c4-inflight 1 --steps 10 --warmup 2" 3 \
  tools/ab/libokv_meta.so tools/ab/libokv_head.so
