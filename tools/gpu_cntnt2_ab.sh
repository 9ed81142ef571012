#!/bin/bash
# pass-1 header reads non-temporal for large blocks only (libokv_cnt_nt2) vs head: C3 four decodes in
# flight (the driver's mode) and one at a time
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py" "--config c3 --no-cpu --no-verify --steps 40 --warmup 5" 4 \
  tools/ab/libokv_cnt_nt2.so tools/ab/libokv_head.so || exit $?
