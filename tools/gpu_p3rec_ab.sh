#!/bin/bash
# C3 in-flight: the chain event recorded before the big-block pass vs after it
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py" "--config c3 --no-cpu --no-verify --steps 40 --warmup 5" 3 \
  tools/ab/libokv_p3rec.so tools/ab/libokv_head.so
