#!/bin/bash
# E9 meta offsets from E8's entry-size prefix (libokv_moff) vs a re-read of each block's first key length (head)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_encode_gpu.py tests/test_full_size_gpu.py" "--config c4 --no-cpu --c4-inflight 1 --steps 10 --warmup 2" 2 \
  tools/ab/libokv_moff.so tools/ab/libokv_meta.so
