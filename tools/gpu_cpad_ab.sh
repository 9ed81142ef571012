#!/bin/bash
# CM count-kernel occupancy (dynamic-LDS pad) A/B: product libraries, CM bench, 2 rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py" "--config cm --no-cpu --steps 10 --warmup 2" 2 \
  tools/ab/libokv_cpad28672.so tools/ab/libokv_head.so tools/ab/libokv_cpad14336.so tools/ab/libokv_cpad57344.so
