#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
./tools/gpu_libab.sh "tests/test_decode_gpu.py tests/test_reader_gpu.py tests/test_snapshot_gpu.py tests/test_tile_gpu.py" "--config cm --no-cpu --steps 10 --warmup 2" 2 tools/ab/libokv_bs.so tools/ab/libokv_head.so || exit $?
mv gpurun_out/libab gpurun_out/libab_cm
for c in c2 c1; do
  ./tools/gpu_libab.sh "" "--config $c --no-cpu --steps 20 --warmup 3" 2 tools/ab/libokv_bs.so tools/ab/libokv_head.so || exit $?
  mv gpurun_out/libab gpurun_out/libab_$c
done
