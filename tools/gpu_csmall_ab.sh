#!/bin/bash
# small-block pass 1 staged in LDS (libokv_csmall) vs the lane-per-block HBM walk (head):
# decode-path GPU tests, then CM and C1 alternating
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py tests/test_tile_gpu.py tests/test_reader_gpu.py tests/test_snapshot_gpu.py tests/test_encode_gpu.py" "--config cm --no-cpu --steps 10 --warmup 2" 2 \
  tools/ab/libokv_csmall.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_cm
./tools/gpu_libab.sh "" "--config c1 --no-cpu --steps 20 --warmup 3" 2 tools/ab/libokv_csmall.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_c1
