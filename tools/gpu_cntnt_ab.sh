#!/bin/bash
# pass-1 header reads non-temporal (libokv_cnt_nt) vs default (head): tests, C3 one decode at a
# time (count kernel time), CM
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py" "--config c3 --no-cpu --no-verify --steps 30 --warmup 5 --decode-inflight 1" 3 \
  tools/ab/libokv_cnt_nt.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_c3
./tools/gpu_libab.sh "" "--config cm --no-cpu --steps 10 --warmup 2" 2 tools/ab/libokv_cnt_nt.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_cm
