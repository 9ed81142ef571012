#!/bin/bash
# pass-1 record table in registers (libokv_creg) vs LDS chunks (head): decode tests,
# C3 (four chained decodes in flight + one at a time) and CM, alternating
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py tests/test_tile_gpu.py tests/test_reader_gpu.py tests/test_snapshot_gpu.py" "--config c3 --no-cpu --no-verify --steps 40 --warmup 5" 3 \
  tools/ab/libokv_creg.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_c3
./tools/gpu_libab.sh "" "--config cm --no-cpu --steps 10 --warmup 2" 2 tools/ab/libokv_creg.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_cm
